"""GPU: the blurred pyramid (k_blur2, ORBextractor.cc:1375-1377 GaussianBlur 7x7 sigma 2
REFLECT_101) pixel by pixel against the oracle's cv::GaussianBlur restatement
(oracle/orb_oracle.c orc_gauss7_u8) of the same pyramid level.

The widths sweep the row-end cases of k_blur2's tiles (244 columns per wave; the left lane
and the last 1..7 columns rebuild their windows by byte permutes): every level width mod 4
and mod 244 near the tile edges, single-tile levels (both row ends in one wave), odd level-0
pitches (per-row byte shifts), and the legacy 257-sum weight table (saturating path).
Tolerance: none.
"""
import numpy as np
import pytest

from orb_slam2_test_amd import ORBextractor, synthetic as S

pytestmark = pytest.mark.gpu


def _image(h, w, seed):
    rng = np.random.default_rng(seed)
    img = S.sequence(1, h, w, seed=seed)[0].astype(np.int32)
    img += rng.integers(-40, 40, img.shape)  # texture up to the borders
    return np.clip(img, 0, 255).astype(np.uint8)


def _levels_for(h, w):
    n = 1
    while n < 8 and min(h, w) / 1.2 ** n >= 72:
        n += 1
    return n


def _check(oracle, ext, img, nlevels, k=None):
    ext(img)
    for l in range(nlevels):
        pyr = ext.get_level(0, l)
        got = ext.get_blurred_level(0, l)
        ref = oracle.gauss7(pyr) if k is None else oracle.gauss7(pyr, k)
        assert got.shape == ref.shape
        bad = np.argwhere(got != ref)
        assert bad.size == 0, f"level {l} ({pyr.shape[1]}x{pyr.shape[0]}): first diffs {bad[:5]}"


@pytest.mark.parametrize("w", list(range(250, 263)) + [243, 244, 245, 487, 488, 489, 493])
def test_blur_widths(oracle, w):
    h = 90
    nl = _levels_for(h, w)
    _check(oracle, ORBextractor(300, 1.2, nl, 20, 7), _image(h, w, 100 + w), nl)


def test_blur_kitti_all_levels(oracle, kitti_seq):
    _check(oracle, ORBextractor(2000, 1.2, 8, 20, 7), kitti_seq[1], 8)


def test_blur_single_tile_levels(oracle):
    # every level narrower than one 244-column tile: both row ends in the same wave
    h, w = 120, 200
    nl = _levels_for(h, w)
    _check(oracle, ORBextractor(300, 1.2, nl, 20, 7), _image(h, w, 7), nl)


def test_blur_legacy_weights(oracle):
    k = (18, 34, 49, 55, 49, 34, 18)  # sums to 257: the saturating path
    h, w = 100, 259
    nl = _levels_for(h, w)
    _check(oracle, ORBextractor(300, 1.2, nl, 20, 7, gauss_k=k), _image(h, w, 3), nl, k=k)


def test_blur_batch_padded_pitch(oracle):
    # level 0 read in place with a pitch that is not a multiple of 4 (per-row byte shifts)
    import torch
    B, h, w, pitch = 3, 96, 301, 307
    frames = np.zeros((B, h, pitch), np.uint8)
    for b in range(B):
        frames[b, :, :w] = _image(h, w, 40 + b)
    d = torch.from_numpy(frames).cuda()
    nl = _levels_for(h, w)
    ext = ORBextractor(300, 1.2, nl, 20, 7, max_batch=B)
    ext.extract_batch_device(d.data_ptr(), B, w, h, step=pitch, frame_stride=h * pitch)
    ext.ctx.sync()
    for b in range(B):
        for l in range(nl):
            pyr = ext.get_level(b, l)
            if l == 0:
                assert np.array_equal(pyr, frames[b, :, :w])
            assert np.array_equal(ext.get_blurred_level(b, l), oracle.gauss7(pyr)), (b, l)


def _with_env(env, fn):
    import os
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return fn()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.mark.parametrize("h,w", [(376, 1241), (90, 257), (120, 200), (480, 640)])
def test_blur_fused_into_fast_cells(oracle, h, w):
    """ORBG_FAST_BLUR=1 (opt-in): the FAST cells blur their detection regions from
    their window tiles (k_fast2<P4, true>) and k_blur_border the rest of every level: the same
    bytes as the oracle's GaussianBlur, and the same keypoints / descriptors."""
    nl = _levels_for(h, w)
    img = _image(h, w, 900 + w)
    ext = _with_env({"ORBG_FAST_BLUR": "1"}, lambda: ORBextractor(300, 1.2, nl, 20, 7))
    _check(oracle, ext, img, nl)
    fused, inner, border = ext.ctx.blur_plan()
    assert fused and inner > 0 and border > 0
    k, d = ext(img)
    p = oracle.params(nfeatures=300, nlevels=nl)
    r = oracle.extract(p, img)
    assert np.array_equal(k, r["kps"]) and np.array_equal(d, r["desc"])


def test_blur_fused_batch_padded_pitch(oracle):
    import torch
    B, h, w, pitch = 3, 160, 301, 307
    frames = np.zeros((B, h, pitch), np.uint8)
    for b in range(B):
        frames[b, :, :w] = _image(h, w, 60 + b)
    d = torch.from_numpy(frames).cuda()
    nl = _levels_for(h, w)
    ext = _with_env({"ORBG_FAST_BLUR": "1"}, lambda: ORBextractor(300, 1.2, nl, 20, 7, max_batch=B))
    ext.extract_batch_device(d.data_ptr(), B, w, h, step=pitch, frame_stride=h * pitch)
    ext.ctx.sync()
    assert ext.ctx.blur_plan()[0]
    for b in range(B):
        for l in range(nl):
            assert np.array_equal(ext.get_blurred_level(b, l), oracle.gauss7(ext.get_level(b, l))), (b, l)


@pytest.mark.parametrize("h,w", [(376, 1241), (90, 257), (121, 333), (480, 640), (97, 250)])
def test_blur_tiled_layout_equals_rows(oracle, h, w):
    """The default tiled blurred levels (k_blur2 stores 16 x 8-px tiles through its LDS stage,
    the rBRIEF phase reads tile rows; heights and widths off the tile grid) against
    ORBG_BLUR_TILED=0 (rows): the same blurred bytes (the oracle's GaussianBlur) and the same
    keypoints and descriptors as the oracle, in both layouts."""
    nl = _levels_for(h, w)
    img = _image(h, w, 1300 + w)
    p = oracle.params(nfeatures=300, nlevels=nl)
    r = oracle.extract(p, img)
    for tiled in (True, False):
        ext = _with_env({"ORBG_BLUR_TILED": "1" if tiled else "0"},
                        lambda: ORBextractor(300, 1.2, nl, 20, 7))
        _check(oracle, ext, img, nl)
        assert ext.ctx.blur_tiled() == tiled
        k, d = ext(img)
        assert np.array_equal(k, r["kps"]) and np.array_equal(d, r["desc"]), tiled
        ext.close()


@pytest.mark.parametrize("tiled", [True, False])
def test_blur_batch_unaligned_frames(oracle, tiled):
    """A batch read in place with an odd pitch AND an odd height: the frames start at every
    byte offset mod 4, so the dword holding a frame's first pixels straddles the frame start
    (k_blur2's bounds-checked range starts at that dword).  Both blurred layouts."""
    import torch
    B, h, w, pitch = 4, 131, 389, 395
    frames = np.zeros((B, h, pitch), np.uint8)
    for b in range(B):
        frames[b, :, :w] = _image(h, w, 80 + b)
    d = torch.from_numpy(frames).cuda()
    nl = _levels_for(h, w)
    ext = _with_env({"ORBG_BLUR_TILED": "1" if tiled else "0"},
                    lambda: ORBextractor(300, 1.2, nl, 20, 7, max_batch=B))
    ext.extract_batch_device(d.data_ptr(), B, w, h, step=pitch, frame_stride=h * pitch)
    ext.ctx.sync()
    assert ext.ctx.blur_tiled() == tiled
    for b in range(B):
        for l in range(nl):
            assert np.array_equal(ext.get_blurred_level(b, l), oracle.gauss7(ext.get_level(b, l))), (b, l)
    ext.close()


def test_blur_fused_unaligned_frames(oracle):
    """The fused blur's border pass (k_blur_border) on frames starting at every byte mod 4."""
    import torch
    B, h, w, pitch = 4, 163, 301, 307
    frames = np.zeros((B, h, pitch), np.uint8)
    for b in range(B):
        frames[b, :, :w] = _image(h, w, 90 + b)
    d = torch.from_numpy(frames).cuda()
    nl = _levels_for(h, w)
    ext = _with_env({"ORBG_FAST_BLUR": "1"}, lambda: ORBextractor(300, 1.2, nl, 20, 7, max_batch=B))
    ext.extract_batch_device(d.data_ptr(), B, w, h, step=pitch, frame_stride=h * pitch)
    ext.ctx.sync()
    assert ext.ctx.blur_plan()[0]
    for b in range(B):
        for l in range(nl):
            assert np.array_equal(ext.get_blurred_level(b, l), oracle.gauss7(ext.get_level(b, l))), (b, l)
    ext.close()
