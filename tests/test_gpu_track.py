"""GPU: the tracking matchers ORBmatcher::SearchByProjection (last frame, ORBmatcher.cc:
1503-1667; local map, :59-154) through the C ABI vs the CPU oracle, bit-exact: the written
mvpMapPoints slot per keypoint and nmatches (including the reference's double counting of
overwritten slots and of rotation-filtered pushes).

Scenes: frame t-1 / t of the synthetic pan sequence, extracted by the oracle; map points
back-projected from t-1 at a common depth (synthetic.tracking_scene / map_projections).
"""
import ctypes as C

import numpy as np
import pytest

from orb_slam2_test_amd import Frame, MapPointProjections, ORBmatcher, synthetic as S
from orb_slam2_test_amd import _lib as L

pytestmark = pytest.mark.gpu

H, W = 376, 1241
FX, FY, CX, CY, BF = S.KITTI_FX, S.KITTI_FY, S.KITTI_CX, S.KITTI_CY, S.KITTI_BF


@pytest.fixture(scope="module")
def scene(oracle):
    seed = S.DEFAULT_SEED + 5
    seq = S.sequence(3, H, W, seed=seed)
    pos = S.sequence_positions(3, seed=seed)
    p = oracle.params(nfeatures=2000)
    r = [oracle.extract(p, seq[t]) for t in range(3)]
    shift = (float(-(pos[1, 1] - pos[0, 1])), float(-(pos[1, 0] - pos[0, 0])))
    sf = np.array([p.scale[l] for l in range(8)], np.float32)
    return r, shift, sf


def cur_frame(r, uright=None, taken=None, Tcw=None):
    F = Frame.from_extraction(r["kps"], r["desc"], W, H)
    F.mvuRight, F.taken, F.mTcw = uright, taken, Tcw
    F.fx, F.fy, F.cx, F.cy, F.mbf, F.mb = FX, FY, CX, CY, BF, BF / FX
    return F


def synthetic_uright(r, seed, depth=10.0):
    rng = np.random.default_rng(seed)
    ur = (r["kps"]["x"] - np.float32(BF / depth)).astype(np.float32)
    ur += rng.uniform(-3, 3, len(ur)).astype(np.float32)
    ur[rng.random(len(ur)) < 0.3] = -1.0        # no stereo match
    return ur


def run_lastframe(oracle, r, sf, shift, th, mono, check_ori, uright=None, taken=None, tz=0.0,
                  seed=0):
    pts, Tcw, Tlw = S.tracking_scene(r[0]["kps"], shift, seed=S.DEFAULT_SEED + seed, tz=tz)
    last = Frame.from_extraction(r[0]["kps"], r[0]["desc"], W, H)
    last.mTcw, last.points, last.point_desc = Tlw, pts, r[0]["desc"]
    F = cur_frame(r[1], uright, taken, Tcw)
    m = ORBmatcher(0.9, check_ori)
    n, match = m.SearchByProjection(F, last, th, mono)
    cam = oracle.track_cam(Tcw, Tlw, FX, FY, CX, CY, BF, BF / FX, mono)
    rn, rmatch = oracle.search_by_projection_lastframe(r[1]["kps"], r[1]["desc"], uright, taken,
                                                       (0, W, 0, H), sf, pts, r[0]["desc"], cam,
                                                       th, check_ori)
    assert np.array_equal(match, rmatch)
    assert n == rn
    return n, match, cam


@pytest.mark.parametrize("th,check_ori", [(15, True), (30, True), (15, False), (4, True)])
def test_lastframe_mono(oracle, scene, th, check_ori):
    r, shift, sf = scene
    n, match, _ = run_lastframe(oracle, r, sf, shift, th, True, check_ori)
    assert n > 300


@pytest.mark.parametrize("tz", [0.0, -2.0, 2.0])
def test_lastframe_stereo_directions(oracle, scene, tz):
    """bForward / bBackward / both-ways level ranges (tz moves the camera along z) and the
    uRight test."""
    r, shift, sf = scene
    ur = synthetic_uright(r[1], 3)
    _, _, cam = run_lastframe(oracle, r, sf, shift, 7, False, True, uright=ur, tz=tz)
    f, b = oracle.track_direction(cam)
    assert (f, b) == ((0, 0) if tz == 0.0 else ((1, 0) if tz < 0 else (0, 1)))


def test_lastframe_taken_keypoints(oracle, scene):
    r, shift, sf = scene
    taken = (np.random.default_rng(5).random(len(r[1]["kps"])) < 0.2).astype(np.uint8)
    run_lastframe(oracle, r, sf, shift, 15, True, True, taken=taken, seed=9)


@pytest.mark.parametrize("th,nnratio,stereo", [(1.0, 0.8, False), (3.0, 0.8, True),
                                               (1.0, 0.6, True), (5.0, 0.9, False)])
def test_local_map(oracle, scene, th, nnratio, stereo):
    r, shift, sf = scene
    mp = S.map_projections(r[0]["kps"], shift, seed=S.DEFAULT_SEED + int(th * 10))
    ur = synthetic_uright(r[1], 4) if stereo else None
    taken = (np.random.default_rng(6).random(len(r[1]["kps"])) < 0.1).astype(np.uint8)
    F = cur_frame(r[1], ur, taken)
    n, match = ORBmatcher(nnratio).SearchByProjection(F, MapPointProjections(mp, r[0]["desc"]), th)
    rn, rmatch = oracle.search_by_projection_local(r[1]["kps"], r[1]["desc"], ur, taken,
                                                   (0, W, 0, H), sf, mp, r[0]["desc"], th,
                                                   nnratio)
    assert np.array_equal(match, rmatch)
    assert n == rn and n > 200


def test_dense_candidates_force_rescan(oracle, scene):
    """A wide window (th = 60) gives most queries far more than K = 8 candidates, and every
    third keypoint starts taken, so K-lists run out and the exact rescan decides."""
    r, shift, sf = scene
    taken = (np.arange(len(r[1]["kps"])) % 3 == 0).astype(np.uint8)
    run_lastframe(oracle, r, sf, shift, 60, True, True, taken=taken, seed=11)
    # 90 % taken: nearly every K-list is exhausted
    taken9 = (np.random.default_rng(13).random(len(r[1]["kps"])) < 0.9).astype(np.uint8)
    n, _, _ = run_lastframe(oracle, r, sf, shift, 40, True, False, taken=taken9, seed=13)
    assert n > 0
    mp = S.map_projections(r[0]["kps"], shift, seed=S.DEFAULT_SEED + 12)
    F = cur_frame(r[1], None, taken)
    n, match = ORBmatcher(0.8).SearchByProjection(F, MapPointProjections(mp, r[0]["desc"]), 8.0)
    rn, rmatch = oracle.search_by_projection_local(r[1]["kps"], r[1]["desc"], None, taken,
                                                   (0, W, 0, H), sf, mp, r[0]["desc"], 8.0, 0.8)
    assert np.array_equal(match, rmatch) and n == rn


def test_empty_and_degenerate(oracle, scene):
    r, shift, sf = scene
    m = ORBmatcher(0.9, True)
    pts, Tcw, Tlw = S.tracking_scene(r[0]["kps"], shift)
    last = Frame.from_extraction(r[0]["kps"][:0], r[0]["desc"][:0], W, H)
    last.mTcw, last.points, last.point_desc = Tlw, pts[:0], r[0]["desc"][:0]
    n, match = m.SearchByProjection(cur_frame(r[1], Tcw=Tcw), last, 15, True)
    assert n == 0 and np.all(match == -1)
    # points behind the camera / no valid flag: nothing matches
    pts2 = pts.copy()
    pts2["z"] = -pts2["z"]
    last.points, last.point_desc = pts2, r[0]["desc"]
    n, match = m.SearchByProjection(cur_frame(r[1], Tcw=Tcw), last, 15, True)
    assert n == 0 and np.all(match == -1)
    # an empty current frame
    F0 = cur_frame({"kps": r[1]["kps"][:0], "desc": r[1]["desc"][:0]}, Tcw=Tcw)
    last.points = pts
    n, match = m.SearchByProjection(F0, last, 15, True)
    assert n == 0 and len(match) == 0


def test_batch_device_matches_host(oracle, scene):
    """orbg_search_by_projection_batch_device over three frames (one stereo) equals three
    host calls of the oracle."""
    import torch
    r, shift, sf = scene
    frames = []
    for k, (a, b) in enumerate([(0, 1), (1, 2), (0, 1)]):
        sh = shift if (a, b) == (0, 1) else (shift[0], shift[1])
        pts, Tcw, Tlw = S.tracking_scene(r[a]["kps"], sh, seed=S.DEFAULT_SEED + 20 + k,
                                         tz=(-1.0 if k == 2 else 0.0))
        frames.append((r[b], r[a], pts, Tcw, Tlw, k == 2))
    B = len(frames)
    fc = max(len(f[0]["kps"]) for f in frames)
    qc = max(len(f[2]) for f in frames)
    kps = np.zeros((B, fc), L.KP_DTYPE)
    desc = np.zeros((B, fc, 32), np.uint8)
    ur = np.full((B, fc), -1.0, np.float32)
    q = np.zeros((B, qc), L.LF_DTYPE)
    qd = np.zeros((B, qc, 32), np.uint8)
    cnt = np.zeros(B, np.int32)
    qcnt = np.zeros(B, np.int32)
    bounds = np.tile(np.array([0, W, 0, H], np.float32), (B, 1))
    cams = (L.TrackCamera * B)()
    refs = []
    for f, (cur, last, pts, Tcw, Tlw, stereo) in enumerate(frames):
        n = len(cur["kps"])
        kps[f, :n] = cur["kps"]
        desc[f, :n] = cur["desc"]
        u = synthetic_uright(cur, 7 + f) if stereo else None
        if stereo:
            ur[f, :n] = u
        q[f, :len(pts)] = pts
        qd[f, :len(pts)] = last["desc"]
        cnt[f], qcnt[f] = n, len(pts)
        cams[f] = L.track_camera(Tcw, Tlw, FX, FY, CX, CY, BF, BF / FX, not stereo)
        cam = oracle.track_cam(Tcw, Tlw, FX, FY, CX, CY, BF, BF / FX, not stereo)
        refs.append(oracle.search_by_projection_lastframe(cur["kps"], cur["desc"], u, None,
                                                          (0, W, 0, H), sf, pts, last["desc"],
                                                          cam, 15, True))
    dev = "cuda"
    t = {k: torch.from_numpy(np.ascontiguousarray(v).view(np.uint8).reshape(-1)).to(dev)
         for k, v in dict(kps=kps, desc=desc, ur=ur, q=q, qd=qd, cnt=cnt, qcnt=qcnt,
                          bounds=bounds).items()}
    cam_t = torch.from_numpy(np.frombuffer(bytes(cams), np.uint8).copy()).to(dev)
    match = torch.full((B * fc,), -7, dtype=torch.int32, device=dev)
    nm = torch.zeros(B, dtype=torch.int32, device=dev)
    tb = L.TrackBatch()
    tb.kps, tb.desc, tb.uright = t["kps"].data_ptr(), t["desc"].data_ptr(), t["ur"].data_ptr()
    tb.taken0 = None
    tb.counts, tb.bounds, tb.frame_cap = t["cnt"].data_ptr(), t["bounds"].data_ptr(), fc
    tb.queries, tb.qdesc = t["q"].data_ptr(), t["qd"].data_ptr()
    tb.qcounts, tb.query_cap = t["qcnt"].data_ptr(), qc
    tb.cams, tb.th, tb.nnratio, tb.check_ori = cam_t.data_ptr(), 15.0, 0.0, 1
    tb.match, tb.nmatches = match.data_ptr(), nm.data_ptr()
    from orb_slam2_test_amd.orbmatcher import _ctx
    ctx = _ctx(0)
    torch.cuda.synchronize()
    L.check(L.lib().orbg_search_by_projection_batch_device(ctx.handle, L.TRACK_LASTFRAME,
                                                           C.byref(tb), B), "batch")
    ctx.sync()
    match = match.cpu().numpy().reshape(B, fc)
    nm = nm.cpu().numpy()
    for f in range(B):
        rn, rm = refs[f]
        assert nm[f] == rn
        assert np.array_equal(match[f, :cnt[f]], rm)
