"""GPU: ORBmatcher paths (HIP) vs the CPU oracle -- bit-exact.

knn2 (all-pairs Hamming 2-NN), SearchForInitialization (vnMatches12, nmatches and the
updated vbPrevMatched), on host-data entry points and on the batched device path.
"""
import numpy as np
import pytest

from orb_slam2_test_amd import Frame, ORBextractor, ORBmatcher, synthetic as S
from orb_slam2_test_amd import _lib

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pairs(oracle, kitti_seq):
    p = oracle.params()
    outs = [oracle.extract(p, kitti_seq[t]) for t in range(4)]
    p4 = oracle.params(nfeatures=4000)
    outs4 = [oracle.extract(p4, kitti_seq[t]) for t in range(2)]
    return outs, outs4


def prev_of(r):
    return np.ascontiguousarray(np.stack([r["kps"]["x"], r["kps"]["y"]], 1).astype(np.float32))


def check_sfi(oracle, a, b, window=100, nnratio=0.9, check_ori=True, prev=None, w=1241, h=376):
    prev = prev_of(a) if prev is None else prev
    m = ORBmatcher(nnratio, check_ori)
    gp = prev.copy()
    F1 = Frame.from_extraction(a["kps"], a["desc"], w, h)
    F2 = Frame.from_extraction(b["kps"], b["desc"], w, h)
    n, m12 = m.SearchForInitialization(F1, F2, gp, window)
    rn, rm12, rprev = oracle.search_for_initialization(a["kps"], a["desc"], b["kps"], b["desc"],
                                                       prev, (0, w, 0, h), window, nnratio,
                                                       check_ori)
    assert n == rn
    assert np.array_equal(m12, rm12)
    assert np.array_equal(gp, rprev)
    return n


def test_knn2_parity(oracle, pairs):
    outs, _ = pairs
    m = ORBmatcher()
    for t in range(3):
        q, tr = outs[t + 1]["desc"], outs[t]["desc"]
        got = m.hamming_knn2(q, tr)
        ref = oracle.knn2(q, tr)
        for g, r in zip(got, ref):
            assert np.array_equal(g, r)


def test_knn2_ties_and_edges(oracle):
    rng = np.random.default_rng(11)
    t = rng.integers(0, 256, (700, 32), dtype=np.uint8)
    t[300:320] = t[5]            # duplicate train rows: lowest index must win
    q = np.concatenate([t[:50], rng.integers(0, 256, (300, 32), dtype=np.uint8)])
    m = ORBmatcher()
    for qq, tt in ((q, t), (q[:1], t), (q, t[:1]), (q, t[:257])):
        got = m.hamming_knn2(qq, tt)
        ref = oracle.knn2(qq, tt)
        for g, r in zip(got, ref):
            assert np.array_equal(g, r)
    bi, bd, sd = m.hamming_knn2(q, t[:0])
    assert np.all(bi == -1) and np.all(bd == 2**31 - 1)


def test_knn2_distance_extremes_and_train_chunks(oracle):
    """d = 0 and d = 256 (bitwise complements), and a train set past the MFMA kernel's 13-bit
    index (8191 rows per launch): duplicates straddling the chunk boundary keep the lowest
    index."""
    rng = np.random.default_rng(12)
    t = rng.integers(0, 256, (9000, 32), dtype=np.uint8)
    q = rng.integers(0, 256, (200, 32), dtype=np.uint8)
    t[8500] = q[0]                  # only exact match, in the second chunk
    t[40] = q[1]; t[8191] = q[1]    # exact match in both chunks: index 40
    t[8192] = q[2]                  # first row of the second chunk
    t[7] = ~q[3]                    # complement only (d = 256 is the farthest)
    m = ORBmatcher()
    for tt in (t, t[:8191], t[:8192]):
        got = m.hamming_knn2(q, tt)
        ref = oracle.knn2(q, tt)
        for g, r in zip(got, ref):
            assert np.array_equal(g, r)
    qq = np.stack([~t[0], t[0]])
    bi, bd, sd = m.hamming_knn2(qq, t[:1])
    assert bd.tolist() == [256, 0] and bi.tolist() == [0, 0] and np.all(sd == 2**31 - 1)


@pytest.mark.parametrize("window,nnratio,ori", [(100, 0.9, True), (10, 0.9, True),
                                                (50, 0.6, True), (200, 0.9, False)])
def test_search_for_initialization(oracle, pairs, window, nnratio, ori):
    outs, _ = pairs
    for t in range(3):
        check_sfi(oracle, outs[t], outs[t + 1], window, nnratio, ori)


def test_search_for_initialization_mono_init_4000(oracle, pairs):
    _, outs4 = pairs
    n = check_sfi(oracle, outs4[0], outs4[1])
    assert n > 50


def test_sfi_perturbed_prev_positions(oracle, pairs):
    outs, _ = pairs
    rng = np.random.default_rng(12)
    prev = prev_of(outs[0]) + rng.normal(0, 20, (len(outs[0]["kps"]), 2)).astype(np.float32)
    prev[::17] = -500  # windows entirely outside the grid
    check_sfi(oracle, outs[0], outs[1], prev=np.ascontiguousarray(prev))


def _synthetic_pair(rng, n2=24, nmatch=12):
    """F2 keys with distinct descriptors; F1 queries first copy the first nmatch of them
    exactly (dist 0 -> matched), then near-copies whose 8 nearest candidates are all
    already matched with a smaller distance: the GPU's top-K list is exhausted and the
    exact rescan path must reproduce the sequential filter."""
    d2 = rng.integers(0, 256, (n2, 32), dtype=np.uint8)
    k2 = np.zeros(n2, _lib.KP_DTYPE)
    k2["x"] = 300 + rng.integers(0, 40, n2)
    k2["y"] = 150 + rng.integers(0, 40, n2)
    k2["angle"] = rng.uniform(0, 360, n2)
    k2["octave"] = 0
    n1 = nmatch + 10
    d1 = np.zeros((n1, 32), np.uint8)
    d1[:nmatch] = d2[:nmatch]
    for i in range(nmatch, n1):
        d1[i] = d2[i % nmatch]
        d1[i, 0] ^= 1  # distance 1 to an already matched candidate
    k1 = np.zeros(n1, _lib.KP_DTYPE)
    k1["x"] = 320
    k1["y"] = 170
    k1["angle"] = k2["angle"][np.arange(n1) % n2]
    return {"kps": k1, "desc": d1}, {"kps": k2, "desc": d2}


def test_sfi_topk_exhaustion_fallback(oracle):
    rng = np.random.default_rng(13)
    for _ in range(5):
        a, b = _synthetic_pair(rng)
        check_sfi(oracle, a, b, window=100, nnratio=0.9, check_ori=False)
        check_sfi(oracle, a, b, window=100, nnratio=0.9, check_ori=True)


def test_sfi_conflict_stealing(oracle):
    """two queries competing for one F2 key: the later, closer one steals it."""
    rng = np.random.default_rng(14)
    d2 = rng.integers(0, 256, (5, 32), dtype=np.uint8)
    k2 = np.zeros(5, _lib.KP_DTYPE)
    k2["x"], k2["y"], k2["octave"] = 400, 200, 0
    k2["x"] += np.arange(5)
    d1 = np.stack([d2[0].copy(), d2[0].copy()])
    d1[0, :2] ^= 0xFF  # distance 16 (matched first)
    d1[1, 0] ^= 0x01   # distance 1 -> steals
    k1 = np.zeros(2, _lib.KP_DTYPE)
    k1["x"], k1["y"] = 400, 200
    check_sfi(oracle, {"kps": k1, "desc": d1}, {"kps": k2, "desc": d2})


def test_batch_match_device(oracle):
    import torch
    B = 24
    frames = S.sequence(B, 376, 1241, seed=91)
    d = torch.from_numpy(frames).cuda()
    ext = ORBextractor(2000, 1.2, 8, 20, 7, max_batch=B)
    ext.extract_batch_device(d.data_ptr(), B, 1241, 376)
    f1 = (np.arange(B) - 1) % B
    f2 = np.arange(B)
    ext.match_batch_device(f1, f2, 100, 0.9, True)
    ext.ctx.sync()
    for pidx in (0, 1, 7, B - 1):
        ka, da = ext.download_frame(int(f1[pidx]))
        kb, db = ext.download_frame(int(f2[pidx]))
        knn, m12, nm = ext.download_matches(pidx, max(len(ka), len(kb)))
        bi, bd, sd = oracle.knn2(db, da)
        assert np.array_equal(knn[:len(kb), 0], bi)
        assert np.array_equal(knn[:len(kb), 1], bd)
        assert np.array_equal(knn[:len(kb), 2], sd)
        rn, rm12, _ = oracle.search_for_initialization(
            ka, da, kb, db, np.ascontiguousarray(np.stack([ka["x"], ka["y"]], 1)), (0, 1241, 0, 376),
            100, 0.9, True)
        assert nm == rn
        assert np.array_equal(m12[:len(ka)], rm12)
    # the summary used by the bench's RCCL gather
    out = torch.zeros(2 * B, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()  # the fill (torch's stream) before the summary (context stream)
    ext.ctx.batch_summary(out.data_ptr())
    ext.ctx.sync()
    s = out.cpu().numpy()
    assert s[0] == len(ext.download_frame(0)[0])


def test_sharded_sequence_gpu(oracle):
    """Batched-sequence mode on the GPU: each shard (block + 1-frame halo, as a rank would
    run it) through liborbg's batch entry points; the concatenated per-frame summary equals
    the oracle's single-process run of the whole cyclic sequence."""
    from orb_slam2_test_amd import ORBextractor, sequence, synthetic
    frames = synthetic.sequence(7, 376, 1241, seed=synthetic.DEFAULT_SEED + 9)
    p = oracle.params(nfeatures=2000)
    ref_nkp, ref_nm = oracle.frames_batch(p, frames, nthreads=4, window=100, nnratio=0.9)
    be = sequence.GpuBackend(ORBextractor(2000, 1.2, 8, 20, 7, max_batch=8))
    for world in (1, 2, 3):
        nkp, nm = [], []
        for r in range(world):
            lo, hi = sequence.shard(len(frames), world, r)
            k, m = be(frames[sequence.local_indices(len(frames), lo, hi)])
            nkp.append(k[1:])
            nm.append(m[1:])
        assert np.array_equal(np.concatenate(nkp), ref_nkp), world
        assert np.array_equal(np.concatenate(nm), ref_nm), world


def test_sharded_sequence_gpu_match_indices(oracle):
    """SURVEY 8e's per-frame gather payload: the vnMatches12 rows exported by
    orbg_batch_matches (every pair of a batch, -1 past the first frame's keypoints) for each
    shard (block + 1-frame halo) equal the oracle's SearchForInitialization output of the
    whole cyclic sequence, row for row."""
    from orb_slam2_test_amd import ORBextractor, sequence, synthetic
    n, h, w = 5, 376, 1241
    frames = synthetic.sequence_block(n, 0, n, h, w, seed=synthetic.DEFAULT_SEED + 13)
    # frames = [halo (frame n-1), 0 .. n-1]: the single-process reference over the cycle
    p = oracle.params(nfeatures=2000)
    ex = [oracle.extract(p, im) for im in frames]
    ref = {}
    for t in range(1, n + 1):
        a, b = ex[t - 1], ex[t]
        prev = np.ascontiguousarray(np.stack([a["kps"]["x"], a["kps"]["y"]], 1))
        k, m, _ = oracle.search_for_initialization(a["kps"], a["desc"], b["kps"], b["desc"],
                                                   prev, (0, w, 0, h), 100, 0.9, True)
        ref[t - 1] = (k, m)  # global frame t - 1 (row of pair (t-2, t-1))
    be = sequence.GpuBackend(ORBextractor(2000, 1.2, 8, 20, 7, max_batch=n + 1),
                             with_matches=True)
    glob = frames[1:]
    for world in (1, 2):
        for r in range(world):
            lo, hi = sequence.shard(n, world, r)
            k, nm, m12 = be(glob[sequence.local_indices(n, lo, hi)])
            for i, t in enumerate(range(lo, hi)):
                rk, rm = ref[t]
                row = m12[i + 1]
                assert nm[i + 1] == rk, (world, t)
                assert np.array_equal(row[:len(rm)], rm), (world, t)
                assert (row[len(rm):] == -1).all(), (world, t)
                assert (row >= 0).sum() == rk


def test_sharded_sequence_gpu_pose_stub(oracle):
    """SURVEY 8e's pose/trajectory stub: per frame t, PoseOptimization over the matches of
    (t-1, t) with frame t-1's keypoints back-projected at sequence.POSE_DEPTH
    (orbg_match_pose_batch_device) -- SE3Quat and inlier count bit-identical to the oracle
    (oracle/pose_oracle.c orc_match_pose over the oracle's own extraction and matches), for
    every shard as a rank would run it."""
    from orb_slam2_test_amd import ORBextractor, sequence, synthetic
    n, h, w = 6, 376, 1241
    frames = synthetic.sequence_block(n, 0, n, h, w, seed=synthetic.DEFAULT_SEED + 17)
    p = oracle.params(nfeatures=2000)
    ex = [oracle.extract(p, im) for im in frames]
    ref = {}
    for t in range(1, n + 1):
        a, b = ex[t - 1], ex[t]
        prev = np.ascontiguousarray(np.stack([a["kps"]["x"], a["kps"]["y"]], 1))
        _, m, _ = oracle.search_for_initialization(a["kps"], a["desc"], b["kps"], b["desc"],
                                                   prev, (0, w, 0, h), 100, 0.9, True)
        ref[t - 1] = oracle.match_pose(p, a["kps"], b["kps"], m, sequence.POSE_CAM,
                                       sequence.POSE_DEPTH)
    be = sequence.GpuBackend(ORBextractor(2000, 1.2, 8, 20, 7, max_batch=n + 1), with_pose=True)
    glob = frames[1:]
    ninl = []
    for world in (1, 2):
        for r in range(world):
            lo, hi = sequence.shard(n, world, r)
            _, nm, pose = be(glob[sequence.local_indices(n, lo, hi)])
            for i, t in enumerate(range(lo, hi)):
                rn, rq, rt = ref[t]
                assert pose[i + 1, 7] == rn, (world, t)
                assert np.array_equal(pose[i + 1, :4], rq), (world, t)
                assert np.array_equal(pose[i + 1, 4:7], rt), (world, t)
                ninl.append(rn)
    # the stub sees the pan: most matches are inliers of one camera motion
    assert np.median(ninl) > 100
