"""GPU: the exact step bench.py times, on every frame, bit for bit against the oracle.

bench.py's step is sequence.BenchStep; these tests run that same object at the bench's own
batch sizes, pipelined (orbg_set_pipeline, the bench default), over several consecutive
steps that cycle through distinct resident input blocks as the bench does, and capture each
step's outputs on the match stream while later steps are already in flight
(orbg_batch_acquire / orbg_batch_release).  Every frame of every step is compared with the
oracle (oracle/, the C restatement, threaded over the host's CPU share):

  C3 (mono, B = 1024 + the halo frame): keypoints (all 7 cv::KeyPoint fields), descriptors,
     knn2 {best index, best, second} of every F2 keypoint, vnMatches12 of every pair, and
     the per-frame summary (keypoints, SearchForInitialization matches)
     -- ORBextractor.cc:1330-1397, ORBmatcher.cc:487-631 / 541-556;
  C2 (extract only, B = 1024): keypoints and descriptors;
  C4 (stereo, B = 512 L/R pairs = 1024 images): both images' keypoints and descriptors,
     mvuRight / mvDepth of every pair and the stereo summary -- Frame.cc:619-834.
"""
import ctypes as C
import os

import numpy as np
import pytest
import torch

from orb_slam2_test_amd import ORBextractor, sequence, synthetic as S
from orb_slam2_test_amd import _lib as L

pytestmark = pytest.mark.gpu

W, H = 1241, 376
KP = 28
NBLOCKS = 3
ORDER = [0, 1, 2, 0]  # 4 consecutive steps; slot reuse with new data, then a block again


def _threads():
    n = len(os.sched_getaffinity(0))
    share = os.environ.get("OMP_NUM_THREADS", "")
    if share.isdigit() and int(share) > 0:
        n = min(n, int(share))
    return max(1, min(n, 32))


_hip_lib = None


def _copy(dst, src, nbytes, stream):
    """device -> device hipMemcpyAsync from a raw liborbg pointer on a raw stream."""
    global _hip_lib
    if _hip_lib is None:
        _hip_lib = C.CDLL("libamdhip64.so")
    rc = _hip_lib.hipMemcpyAsync(C.c_void_p(dst), C.c_void_p(src), C.c_size_t(nbytes), 3,
                                 C.c_void_p(stream))
    assert rc == 0, rc


def _runner(B, mode, nimg):
    ext = ORBextractor(2000, 1.2, 8, 20, 7, max_batch=nimg)
    stream = torch.cuda.Stream()  # bench.py: liborbg on a caller (torch) stream
    ext.ctx.set_stream(stream.cuda_stream)
    ext._keep_stream = stream
    ext.ctx.set_pipeline(True)
    assert ext.ctx.pipelined()
    return ext, sequence.BenchStep(ext, B, mode)


def _capture_frames(ext, nimg, ms):
    kp, de, cn, fc = ext.batch_outputs()
    out = {"fc": fc,
           "kps": torch.empty(nimg * fc * KP, dtype=torch.uint8, device="cuda"),
           "desc": torch.empty(nimg * fc * 32, dtype=torch.uint8, device="cuda"),
           "counts": torch.empty(nimg, dtype=torch.int32, device="cuda")}
    for key, src in (("kps", kp), ("desc", de), ("counts", cn)):
        t = out[key]
        _copy(t.data_ptr(), src, t.numel() * t.element_size(), ms)
    return out


def _frames_host(cap, nimg):
    fc = cap["fc"]
    cnt = cap["counts"].cpu().numpy()
    kps = cap["kps"].cpu().numpy().reshape(nimg, fc, KP)
    desc = cap["desc"].cpu().numpy().reshape(nimg, fc, 32)
    return cnt, kps, desc


@pytest.fixture(scope="module")
def mono_blocks():
    n_total, ranges = S.bench_block_ranges(sequence.BENCH_BATCH["mono"], 1, 0, NBLOCKS)
    return S.sequence_blocks(n_total, ranges, H, W)


@pytest.fixture(scope="module")
def mono_ref(oracle, mono_blocks):
    p = oracle.params()
    return [oracle.frames_full(p, b, nthreads=_threads(), window=100, nnratio=0.9)
            for b in mono_blocks]


def test_bench_step_c3_mono_every_frame(mono_blocks, mono_ref):
    B = sequence.BENCH_BATCH["mono"]
    nimg = B + 1
    ext, bstep = _runner(B, "mono", nimg)
    caps = []

    def capture(st):
        ms = st.mstream.cuda_stream
        out = _capture_frames(ext, nimg, ms)
        knn, _, _, fc = ext.match_outputs()
        out["knn"] = torch.empty(B * fc * 3, dtype=torch.int32, device="cuda")
        _copy(out["knn"].data_ptr(), knn, out["knn"].numel() * 4, ms)
        out["summary"] = st.summary.clone()  # on the match stream (capture runs there)
        out["m12"] = st.m12.clone()
        caps.append(out)

    bstep.capture = capture
    dev = [torch.from_numpy(b).cuda() for b in mono_blocks]
    torch.cuda.synchronize()
    for k in ORDER:
        bstep(dev[k].data_ptr(), W, H)
    ext.ctx.sync()
    torch.cuda.synchronize()
    checked = 0
    for step, k in enumerate(ORDER):
        nkp, nm, rk, rd, rknn, rm12 = mono_ref[k]
        cap = caps[step]
        cnt, kps, desc = _frames_host(cap, nimg)
        fc = cap["fc"]
        assert np.array_equal(cnt, nkp), "step %d counts" % step
        assert cnt.min() > 1500, "too few keypoints for a meaningful check"
        for f in range(nimg):
            n = cnt[f]
            assert np.array_equal(kps[f, :n].reshape(-1), rk[f].view(np.uint8).reshape(-1)), \
                "step %d frame %d keypoints" % (step, f)
            assert np.array_equal(desc[f, :n], rd[f]), "step %d frame %d descriptors" % (step, f)
        knn = cap["knn"].cpu().numpy().reshape(B, fc, 3)
        m12 = cap["m12"].cpu().numpy()
        summ = cap["summary"].cpu().numpy()
        assert np.array_equal(summ[:nimg], nkp), "step %d summary counts" % step
        assert np.array_equal(summ[nimg:], nm[1:]), "step %d summary matches" % step
        for pr in range(B):
            f = pr + 1  # pair (pr, pr + 1): oracle row f (frame f against f - 1)
            assert np.array_equal(knn[pr, :cnt[f]], rknn[f]), "step %d pair %d knn2" % (step, pr)
            assert np.array_equal(m12[pr, :cnt[pr]], rm12[f]), \
                "step %d pair %d vnMatches12" % (step, pr)
            assert (m12[pr, cnt[pr]:] == -1).all()
            checked += 1
        # (block 0's halo is the cyclic sequence's last frame, far from frame 0: that pair
        # legitimately finds almost nothing)
        assert np.median(nm[1:]) > 150, "SearchForInitialization found too few matches"
    assert checked == B * len(ORDER)
    # consecutive steps really saw different frames
    assert not np.array_equal(mono_ref[0][0], mono_ref[1][0])
    ext.close()


def test_bench_step_c2_extract_only_every_frame(oracle, mono_blocks, mono_ref):
    B = sequence.BENCH_BATCH["extract"]
    blocks = [np.ascontiguousarray(b[1:]) for b in mono_blocks]  # bench --extract-only
    ext, bstep = _runner(B, "extract", B)
    caps = []
    bstep.capture = lambda st: caps.append(_capture_frames(ext, B, st.mstream.cuda_stream))
    dev = [torch.from_numpy(b).cuda() for b in blocks]
    torch.cuda.synchronize()
    for k in ORDER:
        bstep(dev[k].data_ptr(), W, H)
    ext.ctx.sync()
    torch.cuda.synchronize()
    for step, k in enumerate(ORDER):
        nkp, _, rk, rd, _, _ = mono_ref[k]  # oracle frame f + 1 = block frame f
        cnt, kps, desc = _frames_host(caps[step], B)
        assert np.array_equal(cnt, nkp[1:]), "step %d counts" % step
        for f in range(B):
            n = cnt[f]
            assert np.array_equal(kps[f, :n].reshape(-1), rk[f + 1].view(np.uint8).reshape(-1)), \
                "step %d frame %d keypoints" % (step, f)
            assert np.array_equal(desc[f, :n], rd[f + 1]), "step %d frame %d descriptors" % (step, f)
    ext.close()


def test_bench_step_c4_stereo_every_pair(oracle):
    from concurrent.futures import ThreadPoolExecutor
    B = sequence.BENCH_BATCH["stereo"]
    nb = 2
    lefts, rights, _ = S.stereo_sequence(nb * B, H, W, seed=S.DEFAULT_SEED)  # bench rank 0
    blocks = []
    for k in range(nb):
        fr = np.empty((2 * B, H, W), np.uint8)
        fr[0::2], fr[1::2] = lefts[k * B:(k + 1) * B], rights[k * B:(k + 1) * B]
        blocks.append(fr)
    order = [0, 1, 0]
    ext, bstep = _runner(B, "stereo", 2 * B)
    caps = []

    def capture(st):
        ms = st.mstream.cuda_stream
        out = _capture_frames(ext, 2 * B, ms)
        ur, dp, nv, fc = C.c_void_p(), C.c_void_p(), C.c_void_p(), C.c_int32()
        L.check(L.lib().orbg_stereo_outputs(ext.ctx.handle, C.byref(ur), C.byref(dp),
                                            C.byref(nv), C.byref(fc)), "orbg_stereo_outputs")
        for key, src in (("ur", ur.value), ("dp", dp.value)):
            out[key] = torch.empty(B * fc.value, dtype=torch.float32, device="cuda")
            _copy(out[key].data_ptr(), src, B * fc.value * 4, ms)
        out["ssum"] = st.ssum.clone()
        caps.append(out)

    bstep.capture = capture
    dev = [torch.from_numpy(b).cuda() for b in blocks]
    torch.cuda.synchronize()
    for k in order:
        bstep(dev[k].data_ptr(), W, H)
    ext.ctx.sync()
    torch.cuda.synchronize()
    p = oracle.params()
    bf, min_z = S.KITTI_BF, S.KITTI_BF / S.KITTI_FX

    def one(args):
        lft, rgt = args
        rl = oracle.extract(p, lft, with_pyramid=True)
        rr = oracle.extract(p, rgt, with_pyramid=True)
        ur, dp = oracle.stereo_matches(p, rl, rr, W, H, bf, min_z)
        return rl["kps"], rl["desc"], rr["kps"], rr["desc"], ur, dp

    with ThreadPoolExecutor(_threads()) as pool:
        refs = [list(pool.map(one, [(lefts[k * B + i], rights[k * B + i]) for i in range(B)]))
                for k in range(nb)]
    ndepth = 0
    for step, k in enumerate(order):
        cap = caps[step]
        fc = cap["fc"]
        cnt, kps, desc = _frames_host(cap, 2 * B)
        ur = cap["ur"].cpu().numpy().reshape(B, fc)
        dp = cap["dp"].cpu().numpy().reshape(B, fc)
        ssum = cap["ssum"].cpu().numpy()
        for i in range(B):
            kl, dl, kr, dr, rur, rdp = refs[k][i]
            nl, nr = cnt[2 * i], cnt[2 * i + 1]
            assert nl == len(kl) and nr == len(kr), "step %d pair %d counts" % (step, i)
            assert np.array_equal(kps[2 * i, :nl].reshape(-1), kl.view(np.uint8).reshape(-1))
            assert np.array_equal(desc[2 * i, :nl], dl), "step %d pair %d left desc" % (step, i)
            assert np.array_equal(kps[2 * i + 1, :nr].reshape(-1), kr.view(np.uint8).reshape(-1))
            assert np.array_equal(desc[2 * i + 1, :nr], dr), "step %d pair %d right desc" % (step, i)
            assert np.array_equal(ur[i, :nl], rur), "step %d pair %d mvuRight" % (step, i)
            assert np.array_equal(dp[i, :nl], rdp), "step %d pair %d mvDepth" % (step, i)
            assert ssum[i] == nl and ssum[B + i] == int((rdp > 0).sum()), \
                "step %d pair %d stereo summary" % (step, i)
            ndepth += int((rdp > 0).sum())
    assert ndepth > 100 * B * len(order)
    ext.close()
