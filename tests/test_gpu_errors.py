"""GPU: device error flags and stale batch outputs surface as error codes, never as silently
short results.

- A quadtree level that overflows a capacity zeroes that level's keypoints on the device.
  The flag is sticky: it survives later batches until orbg_sync / orbg_check_errors /
  orbg_batch_stats / orbg_download_frame reads it, and then the call fails with
  ORBG_ENOTSUP.  The overflow is forced with the fault-injection knob
  ORBG_FAULT_INJECT=octree_overflow (k_octree,
  the fallback for levels past k_octree_lds' 16,384-candidate capacity, is disabled), on a
  pure-noise frame whose level 0 has more candidates than that.
- Match outputs belong to the batch they were computed on: after a new extraction (same or
  another size) orbg_match_outputs / orbg_download_matches fail with ORBG_EINVAL and the
  trajectory summary carries no stale match counts.
"""
import contextlib
import os

import numpy as np
import pytest
import torch

from orb_slam2_test_amd import ORBextractor, synthetic as S
from orb_slam2_test_amd import _lib

pytestmark = pytest.mark.gpu

W, H = 1241, 376


@contextlib.contextmanager
def knob(value):
    """ORBG_FAULT_INJECT is read when a context plans its buffers (its first extraction at a
    size), so the planning call must run inside this block."""
    old = os.environ.get("ORBG_FAULT_INJECT")
    os.environ["ORBG_FAULT_INJECT"] = value
    try:
        yield
    finally:
        if old is None:
            del os.environ["ORBG_FAULT_INJECT"]
        else:
            os.environ["ORBG_FAULT_INJECT"] = old


def test_pure_noise_level0_needs_the_fallback():
    ext = ORBextractor(2000, 1.2, 8, 20, 7)
    kps, _ = ext(S.pure_noise(H, W))
    ncand, _ = ext.ctx.batch_stats()
    assert ncand > 16384, "the fault-injection test below needs a level past OCT_KEY_CAP"
    assert len(kps) >= 2000


def test_batched_overflow_is_sticky_and_fails_loudly():
    frames = np.stack([S.frame(H, W, seed=3), S.pure_noise(H, W), S.frame(H, W, seed=4)])
    d = torch.from_numpy(frames).cuda()
    ext = ORBextractor(2000, 1.2, 8, 20, 7, max_batch=3)
    with knob("octree_overflow"):
        ext.extract_batch_device(d.data_ptr(), 3, W, H)
    # a second, clean batch on top does not wipe the first batch's flag
    clean = torch.from_numpy(np.ascontiguousarray(frames[[0, 2, 0]])).cuda()
    ext.extract_batch_device(clean.data_ptr(), 3, W, H)
    with pytest.raises(_lib.OrbgError) as ei:
        ext.ctx.sync()
    assert ei.value.code == _lib.ORBG_ENOTSUP
    assert "first frame 1" in str(ei.value), str(ei.value)
    # read and cleared: the clean batch alone is fine
    ext.ctx.check_errors()
    ext.extract_batch_device(clean.data_ptr(), 3, W, H)
    ext.ctx.sync()
    # the overflow reaches batch_stats and download_frame too
    ext.extract_batch_device(d.data_ptr(), 3, W, H)
    with pytest.raises(_lib.OrbgError) as ei:
        ext.ctx.batch_stats()
    assert ei.value.code == _lib.ORBG_ENOTSUP
    ext.extract_batch_device(d.data_ptr(), 3, W, H)
    with pytest.raises(_lib.OrbgError):
        ext.download_frame(0)
    # frames 0 and 2 never overflow: after the check their outputs are complete
    ext.extract_batch_device(d.data_ptr(), 3, W, H)
    with pytest.raises(_lib.OrbgError):
        ext.ctx.check_errors()
    k0, _ = ext.download_frame(0)
    assert len(k0) >= 2000


def test_host_entry_overflow_fails():
    ext = ORBextractor(2000, 1.2, 8, 20, 7)
    with knob("octree_overflow"), pytest.raises(_lib.OrbgError) as ei:
        ext(S.pure_noise(H, W))
    assert ei.value.code == _lib.ORBG_ENOTSUP
    # the same context keeps working on frames inside k_octree_lds' capacity
    kps, _ = ext(S.frame(H, W, seed=5))
    assert len(kps) >= 2000


def test_stale_match_outputs_rejected():
    B = 4
    seq = S.sequence(B, H, W, seed=S.DEFAULT_SEED + 77)
    ext = ORBextractor(2000, 1.2, 8, 20, 7, max_batch=B)
    d = torch.from_numpy(seq).cuda()
    ext.extract_batch_device(d.data_ptr(), B, W, H)
    ext.match_batch_device(np.arange(B - 1), np.arange(1, B))
    ext.ctx.sync()
    ext.match_outputs()
    ext.download_matches(0, 16)
    # a new extraction: the match outputs belong to the previous batch
    ext.extract_batch_device(d.data_ptr(), 2, W, H)
    for call in (ext.match_outputs, lambda: ext.download_matches(0, 16)):
        with pytest.raises(_lib.OrbgError) as ei:
            call()
        assert ei.value.code == _lib.ORBG_EINVAL
    summary = torch.full((8,), -7, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()  # the fill (torch's stream) before the summary (context stream)
    ext.ctx.batch_summary(summary.data_ptr())
    ext.ctx.sync()
    s = summary.cpu().numpy()
    assert (s[:2] > 0).all() and (s[2:] == -7).all(), s  # no stale match counts appended
    # a re-plan at another size also invalidates them (buffers were reallocated)
    small = torch.from_numpy(np.stack([S.frame(240, 320, seed=1)] * 2)).cuda()
    ext.extract_batch_device(d.data_ptr(), B, W, H)
    ext.match_batch_device(np.arange(B - 1), np.arange(1, B))
    ext.extract_batch_device(small.data_ptr(), 2, 320, 240)
    with pytest.raises(_lib.OrbgError):
        ext.match_outputs()
    ext.ctx.sync()


def test_widening_entry_points_reject_bad_arguments():
    """the relocalization / loop-closing / RGB-D entry points return ORBG_EINVAL (or
    ORBG_ENOTSUP past the LDS grid's 8192 keypoints) instead of launching on bad input"""
    import ctypes as C
    from orb_slam2_test_amd.orbmatcher import _ctx
    L = _lib
    h = _ctx().handle
    lib = L.lib()
    # batch projection search: unknown mode, RELOC / LOOP without frustum cameras
    d = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    tb = L.TrackBatch()
    tb.kps = tb.desc = tb.counts = tb.bounds = tb.queries = tb.qdesc = tb.qcounts = d.data_ptr()
    tb.match = tb.nmatches = d.data_ptr()
    tb.frame_cap, tb.query_cap = 16, 16
    assert lib.orbg_search_by_projection_batch_device(h, 4, C.byref(tb), 1) == L.ORBG_EINVAL
    for mode in (L.TRACK_RELOC, L.TRACK_LOOP):
        tb.fcams = None
        assert lib.orbg_search_by_projection_batch_device(h, mode, C.byref(tb), 1) == L.ORBG_EINVAL
    # host searches: NULL camera
    kps = np.zeros(8, L.KP_DTYPE)
    desc = np.zeros((8, 32), np.uint8)
    m = np.zeros(8, np.int32)
    n = C.c_int()
    assert lib.orbg_search_by_projection_reloc(h, L.ptr(kps), L.ptr(desc), 8, None, None, None,
                                               None, 0, 10.0, 100, 1, L.ptr(m),
                                               C.byref(n)) == L.ORBG_EINVAL
    assert lib.orbg_search_by_projection_sim3(h, L.ptr(kps), L.ptr(desc), 8, None, None, None,
                                              None, 0, 10, L.ptr(m), C.byref(n)) == L.ORBG_EINVAL
    # RGB-D: unknown depth type, a row pitch below the row
    dep = np.zeros((4, 4), np.uint16)
    ur = np.zeros(8, np.float32)
    dd = np.zeros(8, np.float32)
    assert lib.orbg_rgbd_stereo(h, L.ptr(dep), 7, 1.0, 4, 4, 8, L.ptr(kps), L.ptr(kps), 8, 40.0,
                                L.ptr(ur), L.ptr(dd)) == L.ORBG_EINVAL
    assert lib.orbg_rgbd_stereo(h, L.ptr(dep), L.DEPTH_U16, 1.0, 4, 4, 6, L.ptr(kps), L.ptr(kps),
                                8, 40.0, L.ptr(ur), L.ptr(dd)) == L.ORBG_EINVAL
    # SearchBySim3: NULL pair geometry; more keypoints than the LDS grid holds
    kf = L.KeyFrame(L.ptr(kps), L.ptr(desc), None, None, 8, None, None, None, 0)
    mp = np.zeros(8, L.MAPPOINT_DTYPE)
    assert lib.orbg_search_by_sim3(h, C.byref(kf), L.ptr(mp), L.ptr(desc), None, C.byref(kf),
                                   L.ptr(mp), L.ptr(desc), None, None, 7.5, L.ptr(m),
                                   C.byref(n)) == L.ORBG_EINVAL
    big = np.zeros(9000, L.KP_DTYPE)
    bd = np.zeros((9000, 32), np.uint8)
    bmp = np.zeros(9000, L.MAPPOINT_DTYPE)
    bm = np.zeros(9000, np.int32)
    kb = L.KeyFrame(L.ptr(big), L.ptr(bd), None, None, 9000, None, None, None, 0)
    g = np.zeros(1, L.SIM3_PAIR_DTYPE)
    assert lib.orbg_search_by_sim3(h, C.byref(kb), L.ptr(bmp), L.ptr(bd), None, C.byref(kb),
                                   L.ptr(bmp), L.ptr(bd), None, L.ptr(g), 7.5, L.ptr(bm),
                                   C.byref(n)) == L.ORBG_ENOTSUP


def test_device_matcher_counts_are_clamped_and_flagged():
    """orbg_fuse_batch_device reads the KeyFrame and MapPoint counts from device
    memory.  A count past `cap` / `mcap` is clamped in the kernel (no LDS or output overrun:
    a guard region after the outputs stays untouched) and raises the sticky flag 0x10000,
    which the next orbg_sync reports as ORBG_EINVAL; a pair with sane counts is unaffected,
    and mcap == 0 still writes d_nfused (zero)."""
    import ctypes as C
    import test_oracle_mapping as T
    from orb_slam2_test_amd.orbmatcher import _ctx
    P, cap, mcap, guard = 2, 2048, 1500, 4096
    cases = [T.fuse_case(_lib, 70 + p, n=1800, nmp=1400) for p in range(P)]
    desc = np.zeros((P, cap, 32), np.uint8)
    kps = np.zeros((P, cap), _lib.KP_DTYPE)
    ur = np.zeros((P, cap), np.float32)
    cams = np.zeros(P, _lib.FRUSTUM_DTYPE)
    mps = np.zeros((P, mcap), _lib.MAPPOINT_DTYPE)
    md = np.zeros((P, mcap, 32), np.uint8)
    for p, (kf, fc, mp, mdsc) in enumerate(cases):
        n = len(kf["kps"])
        desc[p, :n], kps[p, :n], ur[p, :n] = kf["desc"], kf["kps"], kf["uright"]
        cams[p] = fc
        mps[p, :len(mp)], md[p, :len(mp)] = mp, mdsc
    cnt = np.array([1800, 1 << 20], np.int32)   # pair 1's KeyFrame count is past cap
    mc = np.array([1400, 1 << 20], np.int32)    # and its MapPoint count past mcap
    t = {k: torch.from_numpy(np.ascontiguousarray(v).view(np.uint8).reshape(-1).copy()).cuda()
         for k, v in dict(desc=desc, kps=kps, ur=ur, cnt=cnt, cams=cams, mps=mps, md=md,
                          mc=mc).items()}
    K = _lib.KeyFrames(t["desc"].data_ptr(), t["kps"].data_ptr(), t["ur"].data_ptr(), None,
                       t["cnt"].data_ptr(), None, None, None, None)
    kfi = torch.arange(P, dtype=torch.int32, device="cuda")
    bi = torch.full((P * mcap + guard,), -9, dtype=torch.int32, device="cuda")
    bd = torch.full((P * mcap + guard,), -9, dtype=torch.int32, device="cuda")
    nf = torch.full((P,), -7, dtype=torch.int32, device="cuda")
    ctx = _ctx()
    torch.cuda.synchronize()
    _lib.check(_lib.lib().orbg_fuse_batch_device(
        ctx.handle, C.byref(K), cap, kfi.data_ptr(), t["cams"].data_ptr(), t["mps"].data_ptr(),
        t["md"].data_ptr(), t["mc"].data_ptr(), mcap, P, 3.0, bi.data_ptr(), bd.data_ptr(),
        nf.data_ptr()), "fuse")
    with pytest.raises(_lib.OrbgError) as ei:
        ctx.sync()
    assert ei.value.code == _lib.ORBG_EINVAL and "capacity" in str(ei.value)
    ctx.sync()  # read and cleared
    torch.cuda.synchronize()
    assert np.all(bi[P * mcap:].cpu().numpy() == -9) and np.all(bd[P * mcap:].cpu().numpy() == -9)
    assert int(nf[0]) > 100  # the sane pair still fuses
    # mcap == 0: nothing to search, d_nfused still written
    nf.fill_(-7)
    _lib.check(_lib.lib().orbg_fuse_batch_device(
        ctx.handle, C.byref(K), cap, kfi.data_ptr(), t["cams"].data_ptr(), t["mps"].data_ptr(),
        t["md"].data_ptr(), t["mc"].data_ptr(), 0, P, 3.0, bi.data_ptr(), bd.data_ptr(),
        nf.data_ptr()), "fuse mcap 0")
    ctx.sync()
    assert np.all(nf.cpu().numpy() == 0)
