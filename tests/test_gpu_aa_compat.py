"""GPU: the C++ host layer (compat/orbg_compat.hpp) driven like Tracking.cc -- two KITTI-
shaped frames through ORBextractor, SearchForInitialization(0.9, checkOri, window 100),
brute-force knn2 and a StereoFrame -- bit-exact against the oracle.

The selftest binary is started as a child process from this module, which sorts first among
the GPU tests, before this pytest process has initialised the GPU (device_count() does not).
"""
import os
import subprocess

import numpy as np
import pytest

from orb_slam2_test_amd import synthetic as S
from orb_slam2_test_amd import _lib

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "orb_slam2_test_amd", "lib", "compat_selftest")


# the single-frame launch-sequence switches: each must give the same bytes
LAUNCH_ENV = {
    "dma": {"ORBG_IMG_PULL": "0"},    # the image by SDMA instead of k_copy16 from host memory
    "notag": {"ORBG_SF_TAG": "0"},    # the fallback note cleared by a memset, not tagged
    "nopf": {"ORBG_PYR_FIRST": "0"},  # the batch launch order
}


@pytest.mark.parametrize("zc", ["1", "0", "1-nohc", "1-dma", "1-notag", "1-nopf", "1-noise",
                                "1-noise-notag"])
def test_cpp_compat_layer_matches_oracle(oracle, tmp_path, zc):
    """zc: ORBG_ZC, the zero-copy output block / SearchForInitialization staging (default 1)
    or the DMA path it replaced; "1-nohc": zero-copy with the block filled by k_pack_frame
    (ORBG_HC=0) instead of by k_orient_desc itself; "1-dma" / "1-notag" / "1-nopf": the
    default with one launch-sequence switch off (LAUNCH_ENV); "-noise": the second frame is
    pure noise, whose level 0 overflows k_octree_lds, so the single-frame path extracts it
    again with k_octree (the fallback note: per-call tag, or the memset under notag)"""
    import torch
    if torch.cuda.device_count() == 0:
        pytest.skip("no GPU")
    assert os.path.exists(EXE), "build() must produce the compat selftest"
    w, h, nfeat = 1241, 376, 2000
    seq = S.sequence(2, h, w, seed=S.DEFAULT_SEED + 77)
    if "noise" in zc:
        seq[1] = S.pure_noise(h, w)
    for t in range(2):
        seq[t].tofile(tmp_path / f"f{t}.raw")
    r = subprocess.run([EXE, "run", str(w), str(h), str(tmp_path / "f0.raw"),
                        str(tmp_path / "f1.raw"), str(tmp_path), str(nfeat)],
                       capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, ORBG_ZC=zc[0], ORBG_HC="0" if "nohc" in zc else "1",
                                **LAUNCH_ENV.get(zc.split("-")[-1], {})))
    assert r.returncode == 0, r.stdout + r.stderr
    p = oracle.params(nfeatures=nfeat)
    ref = [oracle.extract(p, seq[t]) for t in range(2)]
    for t in range(2):
        kps = np.fromfile(tmp_path / f"kps{t}", dtype=_lib.KP_DTYPE)
        desc = np.fromfile(tmp_path / f"desc{t}", dtype=np.uint8).reshape(-1, 32)
        assert len(kps) == len(ref[t]["kps"])
        for f in _lib.KP_DTYPE.names:
            assert np.array_equal(kps[f], ref[t]["kps"][f]), f
        assert np.array_equal(desc, ref[t]["desc"])
    prev = np.ascontiguousarray(np.stack([ref[0]["kps"]["x"], ref[0]["kps"]["y"]], 1))
    rn, rm12, _ = oracle.search_for_initialization(ref[0]["kps"], ref[0]["desc"], ref[1]["kps"],
                                                   ref[1]["desc"], prev, (0, w, 0, h), 100, 0.9,
                                                   True)
    m12 = np.fromfile(tmp_path / "m12", dtype=np.int32)
    assert int(open(tmp_path / "nm.txt").read()) == rn
    assert np.array_equal(m12, rm12)
    # StereoFrame (frame0 left, frame1 right)
    pl = oracle.extract(p, seq[0], with_pyramid=True)
    pr = oracle.extract(p, seq[1], with_pyramid=True)
    bf = np.float32(386.1448)
    rur, rdp = oracle.stereo_matches(p, pl, pr, w, h, float(bf), float(bf / np.float32(718.856)))
    assert np.array_equal(np.fromfile(tmp_path / "stereo_ur", dtype=np.float32), rur)
    assert np.array_equal(np.fromfile(tmp_path / "stereo_depth", dtype=np.float32), rdp)
    knn = np.fromfile(tmp_path / "knn", dtype=np.int32).reshape(-1, 3)
    rbi, rbd, rsd = oracle.knn2(ref[1]["desc"], ref[0]["desc"])
    assert np.array_equal(knn[:, 0], rbi)
    assert np.array_equal(knn[:, 1], rbd)
    assert np.array_equal(knn[:, 2], rsd)
