"""GPU: Optimizer::PoseOptimization (Optimizer.cc:356-631) on the GPU (one workgroup per
frame, fp64) vs the oracle restatement (oracle/pose_oracle.c), bit for bit: the optimised
SE3Quat, its float matrix, mvbOutlier and the inlier count.  Both sum the edges in the same
pinned order and run the same LM / LDLT / exp-map arithmetic without FMA contraction.

Frames: synthetic.pose_frame (map points at 4-60 m, octave-scaled pixel noise, stereo and
mono edges, gross outliers, a perturbed motion-model pose).
"""
import ctypes as C

import numpy as np
import pytest

from orb_slam2_test_amd import PoseOptimization, synthetic as S
from orb_slam2_test_amd import _lib as L

pytestmark = pytest.mark.gpu

CAM = (S.KITTI_FX, S.KITTI_FY, S.KITTI_CX, S.KITTI_CY, S.KITTI_BF)


def check(oracle, edges, T0):
    n, To, q, t, out = PoseOptimization(edges, T0, *CAM)
    rn, rq, rt, rTo, rout = oracle.pose_optimization(edges, CAM, T0)
    assert n == rn
    assert np.array_equal(out, rout)
    assert np.array_equal(q, rq) and np.array_equal(t, rt)
    assert np.array_equal(To, rTo)
    return n, To, out


@pytest.mark.parametrize("seed,stereo_frac,outlier_frac", [(1, 0.5, 0.1), (2, 0.0, 0.2),
                                                           (3, 1.0, 0.05), (4, 0.3, 0.4)])
def test_pose_optimization_matches_oracle(oracle, seed, stereo_frac, outlier_frac):
    edges, Tt, T0 = S.pose_frame(seed=seed, stereo_frac=stereo_frac, outlier_frac=outlier_frac)
    n, To, out = check(oracle, edges, T0)
    assert n > 0.4 * len(edges)
    # and it converges: the optimised pose is far closer to the truth than the prediction
    assert np.abs(To[:, 3] - Tt[:, 3]).max() < 0.3 * np.abs(T0[:, 3] - Tt[:, 3]).max()


def test_small_and_degenerate(oracle):
    edges, Tt, T0 = S.pose_frame(n=200, seed=5)
    for m in (0, 2, 3, 9, 10, 40):          # < 3: untouched, < 10: one round only
        check(oracle, edges[:m], T0)
    # every observation an outlier except a handful
    e2 = edges.copy()
    e2["obs"][10:, 0] += 300.0
    check(oracle, e2, T0)


def test_batch_device(oracle):
    import torch
    frames = [S.pose_frame(n=n, seed=10 + i) for i, n in enumerate((1500, 800, 3, 2000))]
    B = len(frames)
    cap = max(len(f[0]) for f in frames)
    e = np.zeros((B, cap), L.PEDGE_DTYPE)
    cnt = np.zeros(B, np.int32)
    tin = np.zeros((B, 12), np.float32)
    cams = (L.PoseCamera * B)()
    for i, (ed, Tt, T0) in enumerate(frames):
        e[i, :len(ed)] = ed
        cnt[i] = len(ed)
        tin[i] = T0.reshape(12)
        cams[i] = L.PoseCamera(*[float(np.float32(v)) for v in CAM], 0.0)
    dev = "cuda"
    d_e = torch.from_numpy(e.view(np.uint8).reshape(-1)).to(dev)
    d_cnt = torch.from_numpy(cnt).to(dev)
    d_cam = torch.from_numpy(np.frombuffer(bytes(cams), np.uint8).copy()).to(dev)
    d_tin = torch.from_numpy(tin).to(dev)
    d_q = torch.zeros(B * 4, dtype=torch.float64, device=dev)
    d_t = torch.zeros(B * 3, dtype=torch.float64, device=dev)
    d_to = torch.zeros(B * 12, dtype=torch.float32, device=dev)
    d_out = torch.zeros(B * cap, dtype=torch.uint8, device=dev)
    d_ni = torch.zeros(B, dtype=torch.int32, device=dev)
    from orb_slam2_test_amd.orbmatcher import _ctx
    ctx = _ctx(0)
    torch.cuda.synchronize()
    L.check(L.lib().orbg_pose_optimization_batch_device(
        ctx.handle, d_e.data_ptr(), d_cnt.data_ptr(), cap, d_cam.data_ptr(), d_tin.data_ptr(),
        d_q.data_ptr(), d_t.data_ptr(), d_to.data_ptr(), d_out.data_ptr(), d_ni.data_ptr(), B),
        "pose batch")
    ctx.sync()
    q = d_q.cpu().numpy().reshape(B, 4)
    t = d_t.cpu().numpy().reshape(B, 3)
    out = d_out.cpu().numpy().reshape(B, cap)
    ni = d_ni.cpu().numpy()
    for i, (ed, Tt, T0) in enumerate(frames):
        rn, rq, rt, rTo, rout = oracle.pose_optimization(ed, CAM, T0)
        assert ni[i] == rn
        assert np.array_equal(q[i], rq) and np.array_equal(t[i], rt)
        assert np.array_equal(out[i, :len(ed)].astype(bool), rout)
