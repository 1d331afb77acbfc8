"""GPU: the quadtree launches' cross-launch flags, on the bench's pipelined step, against the
oracle (DistributeOctTree, ORBextractor.cc:668-951; SearchForInitialization and knn2 over
the pairs, ORBmatcher.cc:487-631).

A pipelined batch (orbg_set_pipeline, the bench default) runs level 0's quadtree as a split
pair of k_octree_lds launches -- the first at two workgroups per CU, then the frames past its
candidate cap -- followed by the k_octree fallback for levels past the LDS capacity.  The
second launch and k_octree exit at once unless an earlier launch of the batch flagged a level
for them (d_err[3], d_err[2], cleared ahead of each batch).  These tests run consecutive
pipelined BenchStep batches (B = 16 pairs, 17 frames) whose level-0 candidate counts fall in
every band:
  - at most the first launch's cap (plain frames ~9.5k; a constant band over a quarter of
    the frame ~7.3k);
  - past it, up to the second launch's (a 60-px noise stripe ~10.3k, stripes 11.8k / 13k);
  - past the LDS capacity (noise stripes 17-26k, pure noise ~42k), which k_octree takes;
in the order: overflow at the first, middle and last frame / no overflow of either cap / one
overflow (the pair's second launch idle) / the second launch for every frame / the first
block again / no overflow again.  So each gate
is seen raised, cleared by the next batch, and raised again.  Every frame's keypoints and
descriptors, every pair's knn2 rows and vnMatches12, and the summary are compared with the
oracle; ORBG_OCT_GATE=0 (every fallback launch scans) must give identical outputs.
The non-pipelined batch with ORBG_BIG_SIDE=1 (k_octree concurrent with the LDS launches, the
ADVICE r05 race on lvl_cnt) is checked on the overflow block as well.
"""
import os

import numpy as np
import pytest
import torch

from orb_slam2_test_amd import ORBextractor, sequence, synthetic as S

pytestmark = pytest.mark.gpu

W, H = 1241, 376
B = 16
NIMG = B + 1
KP = 28


def _threads():
    n = len(os.sched_getaffinity(0))
    share = os.environ.get("OMP_NUM_THREADS", "")
    if share.isdigit() and int(share) > 0:
        n = min(n, int(share))
    return max(1, min(n, 32))


def _noise(seed):
    return S.pure_noise(H, W, seed=seed)


def _blocks():
    a = S.sequence(NIMG, H, W, seed=7101)
    for f in (0, 8, NIMG - 1):  # level 0 overflows k_octree_lds: first, middle, last frame
        a[f] = _noise(7200 + f)
    a[2, :, :300] = 128          # first launch of the split pair
    for f, wdt in ((3, 100), (4, 150), (5, 300), (9, 400), (11, 600)):
        a[f, :, :wdt] = _noise(7300 + f)[:, :wdt]
    b = S.sequence(NIMG, H, W, seed=7102)
    b[:, :, :300] = 128          # every frame within the first launch's cap
    c = S.sequence(NIMG, H, W, seed=7103)
    c[5] = _noise(7405)          # one overflow
    d = S.sequence(NIMG, H, W, seed=7104)  # the split pair's second launch for every frame
    d[:, :, :60] = _noise(7500)[:, :60]
    return [np.ascontiguousarray(x) for x in (a, b, c, d)]


ORDER = [0, 1, 2, 3, 0, 1]


@pytest.fixture(scope="module")
def blocks():
    return _blocks()


@pytest.fixture(scope="module")
def refs(oracle, blocks):
    p = oracle.params()
    out = [oracle.frames_full(p, blk, nthreads=_threads(), window=100, nnratio=0.9)
           for blk in blocks]
    # the bands the docstring promises are really there (level-0 FAST candidates)
    cc = [[int(oracle.extract(p, blk[f], with_desc=False)["cand_counts"][0]) for f in range(NIMG)]
          for blk in blocks]
    return out, cc


def _run_pipelined(blocks, env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        ext = ORBextractor(2000, 1.2, 8, 20, 7, max_batch=NIMG)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    stream = torch.cuda.Stream()
    ext.ctx.set_stream(stream.cuda_stream)
    ext._keep_stream = stream
    ext.ctx.set_pipeline(True)
    assert ext.ctx.pipelined()
    bstep = sequence.BenchStep(ext, B, "mono")
    caps = []

    def capture(st):
        ms = st.mstream
        kp, de, cn, fc = ext.batch_outputs()
        knn, _, _, _ = ext.match_outputs()
        with torch.cuda.stream(ms):
            out = {"fc": fc, "counts": _dev_copy(cn, NIMG * 4),
                   "kps": _dev_copy(kp, NIMG * fc * KP), "desc": _dev_copy(de, NIMG * fc * 32),
                   "knn": _dev_copy(knn, B * fc * 3 * 4),
                   "summary": st.summary.clone(), "m12": st.m12.clone()}
        caps.append(out)

    bstep.capture = capture
    dev = [torch.from_numpy(b).cuda() for b in blocks]
    torch.cuda.synchronize()
    for k in ORDER:
        bstep(dev[k].data_ptr(), W, H)
    ext.ctx.sync()
    torch.cuda.synchronize()
    host = []
    for cap in caps:
        fc = cap["fc"]
        host.append(dict(
            fc=fc,
            counts=cap["counts"].cpu().numpy().view(np.int32).copy(),
            kps=cap["kps"].cpu().numpy().reshape(NIMG, fc, KP),
            desc=cap["desc"].cpu().numpy().reshape(NIMG, fc, 32),
            knn=cap["knn"].cpu().numpy().view(np.int32).reshape(B, fc, 3),
            summary=cap["summary"].cpu().numpy(), m12=cap["m12"].cpu().numpy()))
    ext.close()
    return host


def _dev_copy(ptr, nbytes):
    """a uint8 tensor copy of nbytes at a raw liborbg device pointer (current stream)."""
    import ctypes as C
    t = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    lib = C.CDLL("libamdhip64.so")
    rc = lib.hipMemcpyAsync(C.c_void_p(t.data_ptr()), C.c_void_p(ptr), C.c_size_t(nbytes), 3,
                            C.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0, rc
    return t


def _check_against_oracle(host, refs):
    out, _ = refs
    for step, k in enumerate(ORDER):
        nkp, nm, rk, rd, rknn, rm12 = out[k]
        h = host[step]
        cnt = h["counts"]
        assert np.array_equal(cnt, nkp), "step %d counts" % step
        for f in range(NIMG):
            n = cnt[f]
            assert np.array_equal(h["kps"][f, :n].reshape(-1), rk[f].view(np.uint8).reshape(-1)), \
                "step %d frame %d keypoints" % (step, f)
            assert np.array_equal(h["desc"][f, :n], rd[f]), "step %d frame %d descriptors" % (step, f)
        assert np.array_equal(h["summary"][:NIMG], nkp), "step %d summary counts" % step
        assert np.array_equal(h["summary"][NIMG:], nm[1:]), "step %d summary matches" % step
        for pr in range(B):
            f = pr + 1
            assert np.array_equal(h["knn"][pr, :cnt[f]], rknn[f]), "step %d pair %d knn2" % (step, pr)
            assert np.array_equal(h["m12"][pr, :cnt[pr]], rm12[f]), "step %d pair %d m12" % (step, pr)
            assert (h["m12"][pr, cnt[pr]:] == -1).all()


def test_candidate_bands_are_covered(blocks, refs):
    """The level-0 candidate counts (oracle) against the plan's caps (orbg_get_quadtree_caps):
    every band of the split pair and the fallback occurs, where the docstring says."""
    _, cc = refs
    ext = ORBextractor(2000, 1.2, 8, 20, 7, max_batch=NIMG)
    d = torch.from_numpy(blocks[3]).cuda()
    ext.extract_batch_device(d.data_ptr(), NIMG, W, H)
    ext.ctx.sync()
    first, l0, upper = ext.ctx.quadtree_caps()
    ext.close()
    assert 0 < first < l0 <= 16384 and upper > 0
    a, b, c, dd = (np.array(x) for x in cc)
    assert a[[0, 8, NIMG - 1]].min() > l0 and c[5] > l0     # k_octree (d_err[2])
    assert a[5] > l0 and a[9] > l0 and a[11] > l0           # noise stripes past the LDS cap
    assert a[2] <= first and b.max() <= first               # the first launch only
    assert first < a[3] <= l0 and first < a[4] <= l0         # the second launch (d_err[3])
    assert np.delete(c, 5).max() <= first  # k_octree's gate raised, the pair's second clear
    assert dd.min() > first and dd.max() <= l0              # every frame: the second launch


def test_pipelined_gates_every_frame_vs_oracle(blocks, refs):
    _check_against_oracle(_run_pipelined(blocks, {}), refs)


def test_pipelined_gates_off_identical(blocks, refs):
    """ORBG_OCT_GATE=0: the split pair's second launch and k_octree scan every batch; the
    outputs must be the gated run's (and so the oracle's)."""
    gated = _run_pipelined(blocks, {})
    open_ = _run_pipelined(blocks, {"ORBG_OCT_GATE": "0"})
    for step in range(len(ORDER)):
        g, o = gated[step], open_[step]
        for key in ("counts", "summary", "m12"):
            assert np.array_equal(g[key], o[key]), (step, key)
        cnt = g["counts"]
        for f in range(NIMG):  # the rows past a frame's count are never written
            assert np.array_equal(g["kps"][f, :cnt[f]], o["kps"][f, :cnt[f]]), (step, f)
            assert np.array_equal(g["desc"][f, :cnt[f]], o["desc"][f, :cnt[f]]), (step, f)
        for pr in range(B):
            n = cnt[pr + 1]
            assert np.array_equal(g["knn"][pr, :n], o["knn"][pr, :n]), (step, pr)
    _check_against_oracle(open_, refs)


def test_big_side_overflow_block(oracle, blocks, refs):
    """ORBG_BIG_SIDE=1, non-pipelined: k_octree runs on its own stream beside the k_octree_lds
    launches and owns the lvl_cnt entries of the levels left to it (OctLdsDims.keep_cnt)."""
    out, _ = refs
    old = os.environ.get("ORBG_BIG_SIDE")
    os.environ["ORBG_BIG_SIDE"] = "1"
    try:
        ext = ORBextractor(2000, 1.2, 8, 20, 7, max_batch=NIMG)
    finally:
        if old is None:
            os.environ.pop("ORBG_BIG_SIDE", None)
        else:
            os.environ["ORBG_BIG_SIDE"] = old
    d = torch.from_numpy(blocks[0]).cuda()
    for rep in range(3):
        ext.extract_batch_device(d.data_ptr(), NIMG, W, H)
        ext.ctx.sync()
        nkp, _, rk, rd, _, _ = out[0]
        for f in range(NIMG):
            k, desc = ext.download_frame(f)
            assert len(k) == nkp[f], (rep, f)
            assert np.array_equal(k.view(np.uint8).reshape(-1), rk[f].view(np.uint8).reshape(-1)), (rep, f)
            assert np.array_equal(desc, rd[f]), (rep, f)
    ext.close()
