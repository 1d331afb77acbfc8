"""CPU: the oracle's Levenberg-Marquardt loop for LocalBundleAdjustment (oracle/ba_oracle.c
orc_ba_optimize: OptimizationAlgorithmLevenberg::solve, optimization_algorithm_levenberg.cpp:
61-164, over orc_ba_linearize / orc_ba_schur_solve / orc_ba_errors / orc_ba_update).  The
device loop (orbg_ba_graph_optimize) is compared with it in tests/test_gpu_ba.py."""
import numpy as np

from orb_slam2_test_amd import synthetic as S


def _perturbed(seed, n_points, s_pose=2e-3, s_point=5e-2):
    poses, pts, edges = S.ba_window(seed=seed, n_points=n_points)
    rng = np.random.default_rng(seed)
    poses = poses.copy()
    free = poses["fixed"] == 0
    poses["t"][free] += rng.normal(0, s_pose, (free.sum(), 3))
    pts = pts + rng.normal(0, s_point, pts.shape)
    return poses, pts, edges


def test_lm_decreases_the_robust_chi2(oracle):
    poses, pts, edges = _perturbed(60, 1500)
    p, q, rep = oracle.ba_optimize(poses, pts, edges, 10)
    assert rep["iterations"] >= 3 and rep["trials"] >= rep["iterations"]
    assert rep["final_chi2"] < 0.5 * rep["initial_chi2"]
    # the reported chi2 is the active robust chi2 of the returned estimates
    tot = oracle.ba_errors(p, q, edges)[4]
    assert tot == rep["final_chi2"]
    # fixed poses never move
    fx = poses["fixed"] != 0
    assert fx.any() and p[fx].tobytes() == poses[fx].tobytes()


def test_lm_steps_are_deterministic_and_resumable(oracle):
    poses, pts, edges = _perturbed(61, 800)
    a = oracle.ba_optimize(poses, pts, edges, 4)
    b = oracle.ba_optimize(poses, pts, edges, 4)
    assert a[0].tobytes() == b[0].tobytes() and a[1].tobytes() == b[1].tobytes()
    assert a[2] == b[2]
    z = oracle.ba_optimize(poses, pts, edges, 0)
    assert z[2]["iterations"] == 0 and z[2]["initial_chi2"] == z[2]["final_chi2"]
    assert z[0].tobytes() == np.asarray(poses).tobytes()


def test_update_small_angle_branch(oracle):
    """VertexSE3Expmap::oplusImpl below |omega| = 1e-5 takes SE3Quat::exp's first-order
    branch (R = I + W + W^2, V = R): a pure translation update moves t by exactly dx."""
    poses, pts, edges = S.ba_window(seed=62, n_points=50)
    dxp = np.zeros((len(poses), 6))
    dxp[:, 3:] = [0.25, -0.5, 1.0]
    dxq = np.zeros((len(pts), 3))
    p, q = oracle.ba_update(poses, pts, dxp, dxq)
    free = poses["fixed"] == 0
    assert np.array_equal(q, pts)
    np.testing.assert_allclose(p["t"][free], poses["t"][free] + [0.25, -0.5, 1.0], rtol=0,
                               atol=1e-12)
