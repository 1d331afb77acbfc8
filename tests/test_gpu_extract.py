"""GPU: ORBextractor (HIP, through the C ABI) vs the CPU oracle -- bit-exact.

Keypoints are compared field by field (x, y, size, angle, response, octave, class_id),
descriptors byte by byte, pyramid levels pixel by pixel.  Tolerance: none (integer and
pinned-float arithmetic).
"""
import numpy as np
import pytest

from orb_slam2_test_amd import ORBextractor, synthetic as S
from orb_slam2_test_amd import _lib

pytestmark = pytest.mark.gpu

_EXT = {}


def ext_for(nfeat=2000, nlevels=8, ini=20, mn=7, **pins):
    key = (nfeat, nlevels, ini, mn, tuple(sorted(pins.items())))
    if key not in _EXT:
        _EXT[key] = ORBextractor(nfeat, 1.2, nlevels, ini, mn, **pins)
    return _EXT[key]


def assert_same(oracle, img, nfeat=2000, nlevels=8, ini=20, mn=7, check_pyr=True,
                opins=None, **pins):
    opins = opins or {}
    p = oracle.params(nfeatures=nfeat, nlevels=nlevels, ini_th_fast=ini, min_th_fast=mn, **opins)
    ref = oracle.extract(p, img, with_pyramid=True)
    ext = ext_for(nfeat, nlevels, ini, mn, **pins)
    kps, desc = ext(img)
    if check_pyr:
        for l in range(nlevels):
            assert np.array_equal(ext.mvImagePyramid[l], ref["pyramid"][l]), f"level {l}"
    assert len(kps) == len(ref["kps"])
    for f in _lib.KP_DTYPE.names:
        assert np.array_equal(kps[f], ref["kps"][f]), f
    assert np.array_equal(desc, ref["desc"])
    return kps, desc


def test_c2_kitti_frames(oracle, kitti_seq):
    for t in range(3):
        kps, desc = assert_same(oracle, kitti_seq[t])
        assert 2000 <= len(kps) <= 2000 + 3 * 8


def test_tum_640x480_1000(oracle):
    assert_same(oracle, S.frame(480, 640, seed=31), nfeat=1000)


def test_mono_init_4000(oracle, kitti_seq):
    assert_same(oracle, kitti_seq[3], nfeat=4000)


def test_pure_noise_many_candidates(oracle):
    assert_same(oracle, S.pure_noise(376, 1241))


def test_constant_image_has_no_keypoints(oracle):
    kps, desc = assert_same(oracle, S.constant(376, 1241))
    assert len(kps) == 0 and desc.shape == (0, 32)


def test_threshold_fallback_cells(oracle):
    # low-contrast texture: most cells find nothing at 20 and fall back to 7
    img = (S.frame(376, 1241, seed=9).astype(np.float32) * 0.15 + 100).astype(np.uint8)
    assert_same(oracle, img)


@pytest.mark.parametrize("w,h,L", [(1226, 370, 8), (752, 480, 8), (500, 300, 5), (333, 250, 3)])
def test_odd_sizes(oracle, w, h, L):
    assert_same(oracle, S.frame(h, w, seed=w + h), nlevels=L)


def test_small_golden_fixture():
    g = np.load(__import__("os").path.join(__import__("os").path.dirname(__file__), "golden",
                                           "small_320x240.npz"), allow_pickle=False)
    nf, nl, ini, mn = [int(v) for v in g["params"]]
    ext = ORBextractor(nf, 1.2, nl, ini, mn)
    kps, desc = ext(g["image"])
    assert np.array_equal(np.ascontiguousarray(kps).view(np.uint8).reshape(-1, 28), g["kps"])
    assert np.array_equal(desc, g["desc"])


@pytest.mark.parametrize("mode", [_lib.RESIZE_SCALAR, _lib.RESIZE_SSE2_16_4])
def test_resize_pins(oracle, kitti_seq, mode):
    assert_same(oracle, kitti_seq[1], resize_mode=mode, opins={"resize_mode": mode})


def test_gauss_legacy_table_and_fma_pin(oracle, kitti_seq):
    k = (18, 34, 49, 55, 49, 34, 18)  # OpenCV 3.2 / 3.4.0-3.4.8 rounding table
    assert_same(oracle, kitti_seq[2], gauss_k=k, opins={"gauss_k": k}, check_pyr=False)
    assert_same(oracle, kitti_seq[2], brief_fma=1, opins={"brief_fma": 1}, check_pyr=False)


def test_strided_input_and_empty(oracle, kitti_seq):
    big = np.zeros((376, 1300), np.uint8)
    big[:, :1241] = kitti_seq[4]
    view = big[:, :1241]  # row pitch 1300
    ext = ext_for()
    k1, d1 = ext(np.ascontiguousarray(view))
    ref = oracle.extract(oracle.params(), kitti_seq[4])
    assert np.array_equal(d1, ref["desc"])
    assert ext(np.zeros((0, 0), np.uint8)) == (None, None)


def test_getters_match_oracle_tables(oracle):
    ext = ext_for()
    p = oracle.params()
    assert ext.GetLevels() == 8
    assert np.float32(ext.GetScaleFactor()) == np.float32(1.2)
    assert np.array_equal(np.array(ext.GetScaleFactors(), np.float32), np.array(p.scale[:8], np.float32))
    assert np.array_equal(np.array(ext.GetInverseScaleSigmaSquares(), np.float32),
                          np.array(p.inv_sigma2[:8], np.float32))
    assert list(ext.mnFeaturesPerLevel) == list(p.features_per_level[:8])


def test_batch_equals_single_and_oracle(oracle):
    import torch
    B = 48
    frames = S.sequence(B, 376, 1241, seed=77)
    d = torch.from_numpy(frames).cuda()
    ext = ORBextractor(2000, 1.2, 8, 20, 7, max_batch=B)
    ext.extract_batch_device(d.data_ptr(), B, 1241, 376)
    ext.ctx.sync()
    p = oracle.params()
    for f in (0, 1, 13, 29, B - 1):
        k, desc = ext.download_frame(f)
        r = oracle.extract(p, frames[f])
        assert np.array_equal(k, r["kps"]) and np.array_equal(desc, r["desc"]), f
    # full-size properties for every frame of the batch: determinism + bounds
    outs = [ext.download_frame(f) for f in range(B)]
    ext.extract_batch_device(d.data_ptr(), B, 1241, 376)
    ext.ctx.sync()
    for f in range(B):
        k2, d2 = ext.download_frame(f)
        assert np.array_equal(outs[f][0], k2) and np.array_equal(outs[f][1], d2)
        k = outs[f][0]
        assert np.all((k["x"] >= 16) & (k["x"] < 1241 - 16) & (k["y"] >= 16) & (k["y"] < 376 - 16))
        cnt = np.bincount(k["octave"], minlength=8)
        assert np.all(cnt <= np.array(ext.mnFeaturesPerLevel) + 3)
        assert np.all(np.diff(k["octave"]) >= 0)


def test_batch_level0_kcap_and_fallback(oracle, monkeypatch):
    """Batches (B > 8) split level 0 of k_octree_lds: a first launch at ORBG_OCT_L0_WPC
    workgroups per CU (default 2: a smaller candidate cap), then the frames past its cap at
    one workgroup per CU; a level past that (pure noise) goes to k_octree.  Same outputs as
    the oracle for 2 and 3 (3: most frames take the second launch) and as no split (1)."""
    import torch
    B = 12
    frames = S.sequence(B, 376, 1241, seed=91)
    frames[5] = S.pure_noise(376, 1241)
    d = torch.from_numpy(frames).cuda()
    outs = {}
    for wpc in ("1", "2", "3"):
        monkeypatch.setenv("ORBG_OCT_L0_WPC", wpc)
        ext = ORBextractor(2000, 1.2, 8, 20, 7, max_batch=B)
        ext.extract_batch_device(d.data_ptr(), B, 1241, 376)
        ext.ctx.sync()
        outs[wpc] = [ext.download_frame(f) for f in range(B)]
    p = oracle.params()
    for f in (0, 5, B - 1):
        r = oracle.extract(p, frames[f])
        k, desc = outs["2"][f]
        assert np.array_equal(k, r["kps"]) and np.array_equal(desc, r["desc"]), f
    for w in ("2", "3"):
        for f in range(B):
            assert np.array_equal(outs["1"][f][0], outs[w][f][0]), (w, f)
            assert np.array_equal(outs["1"][f][1], outs[w][f][1]), (w, f)


def test_batch_padded_pitch(oracle):
    import torch
    B, W, H, P = 4, 1241, 376, 1280
    frames = S.sequence(B, H, W, seed=78)
    buf = np.zeros((B, H, P), np.uint8)
    buf[:, :, :W] = frames
    d = torch.from_numpy(buf).cuda()
    ext = ORBextractor(2000, 1.2, 8, 20, 7, max_batch=B)
    ext.extract_batch_device(d.data_ptr(), B, W, H, step=P, frame_stride=P * H)
    ext.ctx.sync()
    p = oracle.params()
    for f in range(B):
        k, desc = ext.download_frame(f)
        r = oracle.extract(p, frames[f])
        assert np.array_equal(k, r["kps"]) and np.array_equal(desc, r["desc"])
        assert np.array_equal(ext.get_level(f, 0), frames[f])


def _extract_with(oracle, img, sf, nl, nfeat=2000, env=None):
    """ORBextractor(nfeat, sf, nl, 20, 7) vs the oracle; returns the kernel names that ran."""
    import os
    old = {k: os.environ.get(k) for k in (env or {})}
    os.environ.update(env or {})
    try:
        ext = ORBextractor(nfeat, sf, nl, 20, 7)
        ext.ctx.profile(True)
        kps, desc = ext(img)
        names = set(ext.ctx.profile_read())
        pyr = ext.mvImagePyramid
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    p = oracle.params(nfeatures=nfeat, scale_factor=sf, nlevels=nl)
    ref = oracle.extract(p, img, with_pyramid=True)
    for l in range(nl):
        assert np.array_equal(pyr[l], ref["pyramid"][l]), f"level {l}"
    assert np.array_equal(kps, ref["kps"]) and np.array_equal(desc, ref["desc"])
    ext.close()
    return names


@pytest.mark.parametrize("sf,nl", [(1.5, 5), (1.7, 4)])
def test_resize_chain_scale_factors(oracle, kitti_seq, sf, nl):
    """Scale factors past k_pyramid's band plan (> 11 source rows per 8 output rows) build the
    pyramid with the k_resize chain (one launch per level); bit-exact all the same."""
    names = _extract_with(oracle, kitti_seq[0], sf, nl)
    assert "resize_chain" in names and "resize" not in names


@pytest.mark.parametrize("sf,nl", [(1.1, 8), (1.25, 8), (1.3, 6)])
def test_other_scale_factors(oracle, kitti_seq, sf, nl):
    """ORBextractor.scaleFactor / nLevels other than the shipped 1.2 / 8 (ORBextractor.cc:
    432-470 tables, :1400-1443 pyramid): bit-exact whichever pyramid kernel the plan takes."""
    names = _extract_with(oracle, kitti_seq[1], sf, nl)
    assert ("resize" in names) != ("resize_chain" in names)


def test_euroc_752x480_1200(oracle):
    """EuRoC's settings (Examples/Monocular/EuRoC.yaml: 752 x 480, 1200 features)."""
    assert_same(oracle, S.frame(480, 752, seed=77), nfeat=1200)


def test_resize_chain_forced_at_1_2(oracle, kitti_seq):
    """ORBG_PYR=0 forces the k_resize chain at the reference's 1.2 (KITTI and TUM shapes)."""
    names = _extract_with(oracle, kitti_seq[2], 1.2, 8, env={"ORBG_PYR": "0"})
    assert "resize_chain" in names and "resize" not in names
    names = _extract_with(oracle, S.frame(480, 640, seed=5), 1.2, 8, nfeat=1000,
                          env={"ORBG_PYR": "0"})
    assert "resize_chain" in names
    names = _extract_with(oracle, kitti_seq[2], 1.2, 8)
    assert "resize" in names and "resize_chain" not in names
