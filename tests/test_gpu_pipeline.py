"""GPU: pipelined batches (orbg_set_pipeline) give the outputs of the plain batch path, bit
for bit, for every batch of a run in which the image half of batch k+1 overlaps the keypoint
half of batch k.

Every batch's per-frame outputs (keypoints, descriptors, counts), its vnMatches12 and its
trajectory summary are copied on the match stream while later batches are already in
flight, then compared with a context that runs the same batches one after the other.
"""
import ctypes as C

import numpy as np
import pytest
import torch

from orb_slam2_test_amd import ORBextractor, synthetic as S
from orb_slam2_test_amd import _lib

pytestmark = pytest.mark.gpu

W, H = 1241, 376
KP_BYTES = 28


def _hip():
    return C.CDLL("libamdhip64.so")


def _copy_async(hip, dst, src, nbytes, stream):
    """hipMemcpyAsync device -> device on a raw hipStream_t (test-side capture only)."""
    rc = hip.hipMemcpyAsync(C.c_void_p(dst), C.c_void_p(src), C.c_size_t(nbytes), 3,
                            C.c_void_p(stream))
    assert rc == 0, rc


def _batches(B):
    a = S.sequence(B, H, W, seed=91)
    b = S.sequence(B, H, W, seed=92)
    c = np.ascontiguousarray(a[::-1])
    return [a, b, c, b]


def _run(frames_list, B, pipelined):
    ext = ORBextractor(2000, 1.2, 8, 20, 7, max_batch=B)
    ext.ctx.set_pipeline(pipelined)
    assert ext.ctx.pipelined() == pipelined
    hip = _hip()
    dev = [torch.from_numpy(f).cuda() for f in frames_list]
    torch.cuda.synchronize()
    f1 = np.arange(B - 1, dtype=np.int32)
    f2 = np.arange(1, B, dtype=np.int32)
    caps = []
    for d in dev:
        ext.extract_batch_device(d.data_ptr(), B, W, H)
        ext.match_batch_device(f1, f2, 100, 0.9, True)
        kp, de, cn, fc = ext.batch_outputs()
        _, m12, _, _ = ext.match_outputs()
        out = {
            "kps": torch.zeros(B * fc * KP_BYTES, dtype=torch.uint8, device="cuda"),
            "desc": torch.zeros(B * fc * 32, dtype=torch.uint8, device="cuda"),
            "counts": torch.zeros(B, dtype=torch.int32, device="cuda"),
            "m12": torch.zeros((B - 1) * fc, dtype=torch.int32, device="cuda"),
            "summary": torch.zeros(2 * B, dtype=torch.int32, device="cuda"),
        }
        # the zero fills run on torch's stream, and the context's streams are non-blocking
        # (no implicit order with it): finish them before the match-stream copies
        torch.cuda.current_stream().synchronize()
        ms = ext.ctx.match_stream()
        # on the match stream after this batch's matching, before orbg_batch_summary
        # records the slot's "no longer read" event
        for key, src in (("kps", kp), ("desc", de), ("counts", cn), ("m12", m12)):
            t = out[key]
            _copy_async(hip, t.data_ptr(), src, t.numel() * t.element_size(), ms)
        ext.ctx.batch_summary(out["summary"].data_ptr())
        caps.append((out, fc))
    ext.ctx.sync()
    torch.cuda.synchronize()
    res = []
    for out, fc in caps:
        cnt = out["counts"].cpu().numpy()
        kps = out["kps"].cpu().numpy().reshape(B, fc, KP_BYTES)
        desc = out["desc"].cpu().numpy().reshape(B, fc, 32)
        m12 = out["m12"].cpu().numpy().reshape(B - 1, fc)
        frames = [(kps[f, :cnt[f]].copy(), desc[f, :cnt[f]].copy()) for f in range(B)]
        pairs = [m12[p, :cnt[p]].copy() for p in range(B - 1)]
        res.append((cnt, frames, pairs, out["summary"].cpu().numpy()))
    ext.close()
    return res


def test_pipelined_batches_equal_plain_batches():
    B = 24
    fl = _batches(B)
    ref = _run(fl, B, False)
    got = _run(fl, B, True)
    for k, (r, g) in enumerate(zip(ref, got)):
        assert np.array_equal(r[0], g[0]), "batch %d counts" % k
        assert r[0].min() > 1000, "batch %d: too few keypoints for a meaningful check" % k
        for f in range(B):
            assert np.array_equal(r[1][f][0], g[1][f][0]), "batch %d frame %d keypoints" % (k, f)
            assert np.array_equal(r[1][f][1], g[1][f][1]), "batch %d frame %d descriptors" % (k, f)
        for p in range(B - 1):
            assert np.array_equal(r[2][p], g[2][p]), "batch %d pair %d vnMatches12" % (k, p)
        assert np.array_equal(r[3], g[3]), "batch %d summary" % k
    # consecutive batches really differ (a stale slot would not go unnoticed)
    assert not np.array_equal(ref[0][0], ref[1][0])


def test_pipelined_matches_oracle_last_batch(oracle):
    B = 8
    fl = _batches(B)
    ext = ORBextractor(2000, 1.2, 8, 20, 7, max_batch=B)
    ext.ctx.set_pipeline(True)
    dev = [torch.from_numpy(f).cuda() for f in fl]
    torch.cuda.synchronize()
    for d in dev:
        ext.extract_batch_device(d.data_ptr(), B, W, H)
    p = oracle.params()
    for f in (0, 3, B - 1):
        k, desc = ext.download_frame(f)
        r = oracle.extract(p, fl[-1][f], with_pyramid=True)
        assert np.array_equal(k, r["kps"]) and np.array_equal(desc, r["desc"]), f
        assert np.array_equal(ext.get_level(f, 2), r["pyramid"][2]), f
    ext.close()


def test_pipelined_stereo_equals_plain():
    B = 6
    lefts, rights, _ = S.stereo_sequence(B, H, W, seed=93)
    frames = np.empty((2 * B, H, W), np.uint8)
    frames[0::2], frames[1::2] = lefts, rights
    other = np.ascontiguousarray(frames[::-1])
    sl, sr = np.arange(B) * 2, np.arange(B) * 2 + 1

    def run(pipelined):
        ext = ORBextractor(2000, 1.2, 8, 20, 7, max_batch=2 * B)
        ext.ctx.set_pipeline(pipelined)
        dev = [torch.from_numpy(f).cuda() for f in (other, frames)]
        torch.cuda.synchronize()
        for d in dev:
            ext.extract_batch_device(d.data_ptr(), 2 * B, W, H)
            ext.stereo_batch_device(sl, sr, S.KITTI_BF, S.KITTI_BF / S.KITTI_FX)
        out = []
        for i in range(B):
            n = len(ext.download_frame(2 * i)[0])
            out.append(ext.download_stereo(i, n))
        ext.close()
        return out

    ref, got = run(False), run(True)
    for i, (r, g) in enumerate(zip(ref, got)):
        assert np.array_equal(r[0], g[0]) and np.array_equal(r[1], g[1]) and r[2] == g[2], i
    assert sum(r[2] for r in ref) > 0
