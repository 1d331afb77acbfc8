"""Optimizer -- the per-edge arithmetic of Optimizer::LocalBundleAdjustment on the GPU.

Reference: src/Optimizer.cc:633-979 builds a g2o graph with EdgeSE3ProjectXYZ /
EdgeStereoSE3ProjectXYZ edges (Huber delta sqrt(5.991) / sqrt(7.815), information
invSigma2 * I) and runs Levenberg-Marquardt.  The LM driver, Schur solve and map
write-back stay on the host (they are sequential); this module replaces the
arithmetic g2o performs per edge in computeActiveErrors + BlockSolver::buildSystem:
residual, analytic Jacobians, chi2, Huber weight and the J^T W J / J^T W r blocks.

Arrays use the dtypes of ``_lib`` (POSE_DTYPE, EDGE_DTYPE, EDGE_OUT_DTYPE).
"""
import ctypes
import math

import numpy as np

from . import _lib as L
from .orbmatcher import _ctx

TH_HUBER_MONO = float(np.float32(math.sqrt(5.991)))     # const float thHuberMono (Optimizer.cc:758)
TH_HUBER_STEREO = float(np.float32(math.sqrt(7.815)))   # const float thHuberStereo (:759)
CHI2_MONO = 5.991                                       # outlier cut (:879)
CHI2_STEREO = 7.815                                     # (:895)


def linearize_local_ba(poses, points, edges, device=0, with_edges=True):
    """Returns (edge_out | None, H_pose[np,6,6], b_pose[np,6], H_point[nq,3,3], b_point[nq,3])."""
    poses = np.ascontiguousarray(poses, L.POSE_DTYPE)
    points = np.ascontiguousarray(points, np.float64).reshape(-1, 3)
    edges = np.ascontiguousarray(edges, L.EDGE_DTYPE)
    npose, npoint, nedge = len(poses), len(points), len(edges)
    eout = np.zeros(nedge, L.EDGE_OUT_DTYPE) if with_edges else None
    hpose = np.zeros((npose, 6, 6))
    bpose = np.zeros((npose, 6))
    hpoint = np.zeros((npoint, 3, 3))
    bpoint = np.zeros((npoint, 3))
    L.check(L.lib().orbg_ba_linearize(_ctx(device).handle, L.ptr(poses), npose, L.ptr(points),
                                      npoint, L.ptr(edges), nedge, L.ptr(eout), L.ptr(hpose),
                                      L.ptr(bpose), L.ptr(hpoint), L.ptr(bpoint)),
            "orbg_ba_linearize")
    return eout, hpose, bpose, hpoint, bpoint


def ba_errors(poses, points, edges, device=0):
    """g2o's per-trial error pass (computeActiveErrors + activeRobustChi2 terms +
    isDepthPositive, sparse_optimizer.cpp:61-114, orbg_ba_errors) for the LBA edges.
    Returns (err (n, 3), chi2 (n,), rho0 (n,), depth_ok (n,) bool, active robust chi2 sum in
    edge order)."""
    poses = np.ascontiguousarray(poses, L.POSE_DTYPE)
    points = np.ascontiguousarray(points, np.float64).reshape(-1, 3)
    edges = np.ascontiguousarray(edges, L.EDGE_DTYPE)
    n = len(edges)
    err = np.zeros((max(n, 1), 3))
    chi2 = np.zeros(max(n, 1))
    rho0 = np.zeros(max(n, 1))
    dok = np.zeros(max(n, 1), np.uint8)
    tot = ctypes.c_double()
    L.check(L.lib().orbg_ba_errors(_ctx(device).handle, L.ptr(poses), len(poses), L.ptr(points),
                                   len(points), L.ptr(edges), n, L.ptr(err), L.ptr(chi2),
                                   L.ptr(rho0), L.ptr(dok), ctypes.byref(tot)), "orbg_ba_errors")
    return err[:n], chi2[:n], rho0[:n], dok[:n].astype(bool), tot.value


def ba_schur_solve(poses, npoint, edges, eout, hpose, bpose, hpoint, bpoint, lam, device=0):
    """g2o BlockSolver<6,3>::solve (block_solver.hpp:354-486) after setLambda(lam), on
    linearize_local_ba's outputs.  Returns (ok, dx_pose (npose, 6), dx_point (npoint, 3))."""
    poses = np.ascontiguousarray(poses, L.POSE_DTYPE)
    edges = np.ascontiguousarray(edges, L.EDGE_DTYPE)
    eout = np.ascontiguousarray(eout, L.EDGE_OUT_DTYPE)
    arrs = [np.ascontiguousarray(a, np.float64) for a in (hpose, bpose, hpoint, bpoint)]
    dp = np.zeros((max(len(poses), 1), 6))
    dq = np.zeros((max(npoint, 1), 3))
    ok = ctypes.c_int()
    L.check(L.lib().orbg_ba_schur_solve(_ctx(device).handle, L.ptr(poses), len(poses), npoint,
                                        L.ptr(edges), len(edges), L.ptr(eout), *[L.ptr(a) for a in arrs],
                                        float(lam), L.ptr(dp), L.ptr(dq), ctypes.byref(ok)),
            "orbg_ba_schur_solve")
    return bool(ok.value), dp[:len(poses)], dq[:npoint]


def PoseOptimization(edges, Tcw, fx, fy, cx, cy, bf, device=0):
    """Optimizer::PoseOptimization (Optimizer.cc:356-631) on one frame.

    edges: PEDGE_DTYPE records, one per keypoint with a MapPoint in index order (obs =
    kpUn.pt.x, kpUn.pt.y, mvuRight; xw = world position; inv_sigma2 = mvInvLevelSigma2
    [octave]; stereo = mvuRight >= 0).  Tcw: pFrame->mTcw (3x4 or 4x4).  Returns
    (nInliers, Tcw_out (3, 4) float32 = SetPose's matrix, q (x, y, z, w), t, mvbOutlier)."""
    e = np.ascontiguousarray(edges, L.PEDGE_DTYPE)
    T = np.ascontiguousarray(np.asarray(Tcw, np.float32)[:3, :4].reshape(12))
    cam = L.PoseCamera(*[float(np.float32(v)) for v in (fx, fy, cx, cy, bf)], 0.0)
    q = np.zeros(4)
    t = np.zeros(3)
    To = np.zeros(12, np.float32)
    out = np.zeros(max(len(e), 1), np.uint8)
    ni = ctypes.c_int()
    L.check(L.lib().orbg_pose_optimization(_ctx(device).handle, L.ptr(e), len(e), ctypes.byref(cam),
                                           L.ptr(T), L.ptr(q), L.ptr(t), L.ptr(To), L.ptr(out),
                                           ctypes.byref(ni)), "orbg_pose_optimization")
    return ni.value, To.reshape(3, 4), q, t, out[:len(e)].astype(bool)


def vertex_csr(edges, field, nvert):
    """Edge lists per vertex (CSR): (off[nvert+1], edge ids[nedge]) int32, edges in input
    order within a vertex -- the layout orbg_ba_linearize_device reduces blocks over."""
    v = np.asarray(edges[field], np.int64)
    order = np.argsort(v, kind="stable").astype(np.int32)
    off = np.zeros(nvert + 1, np.int64)
    np.add.at(off, v + 1, 1)
    return np.cumsum(off).astype(np.int32), order


class DeviceLBA:
    """Device-resident batch of LBA windows (one graph; windows are independent blocks of
    it): uploads once, then linearize() runs orbg_ba_linearize_device on the context stream
    with every array in HBM -- the per-iteration work of g2o's computeActiveErrors +
    buildSystem."""

    def __init__(self, poses, points, edges, device=0, jacobians=True, edge_errors=True,
                 graph=False):
        import torch
        self.ctx = _ctx(device)
        self.graph = None  # orbg_ba_graph (packed edges in HBM): build_system / errors use it
        if graph:
            e = np.ascontiguousarray(edges, L.EDGE_DTYPE)
            h = L.C.c_void_p()
            L.check(L.lib().orbg_ba_graph_create(self.ctx.handle, e.ctypes.data, len(e), len(poses),
                                                 len(points), L.C.byref(h)),
                    "orbg_ba_graph_create")
            self.graph = h
        self.jacobians = bool(jacobians)  # eout.jp / jt stored (orbg_ba_set_jacobians)
        self.edge_errors = bool(edge_errors)  # eout.err / chi2 / rho1 (orbg_ba_set_edge_errors)
        self.np, self.nq, self.ne = len(poses), len(points), len(edges)
        off, pe = vertex_csr(edges, "pose", self.np)
        qoff, qe = vertex_csr(edges, "point", self.nq)
        dev = torch.device("cuda", device)

        def up(a):
            return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8)).to(dev)

        self.d_poses = up(np.ascontiguousarray(poses, L.POSE_DTYPE))
        self.d_points = up(np.ascontiguousarray(points, np.float64))
        self.d_edges = up(np.ascontiguousarray(edges, L.EDGE_DTYPE))
        self.d_off, self.d_pe = up(off), up(pe)
        self.d_qoff, self.d_qe = up(qoff), up(qe)
        self.d_eout = torch.zeros(self.ne * L.EDGE_OUT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
        self.d_hpose = torch.zeros((self.np, 6, 6), dtype=torch.float64, device=dev)
        self.d_bpose = torch.zeros((self.np, 6), dtype=torch.float64, device=dev)
        self.d_hpoint = torch.zeros((self.nq, 3, 3), dtype=torch.float64, device=dev)
        self.d_bpoint = torch.zeros((self.nq, 3), dtype=torch.float64, device=dev)
        self.d_chi2 = torch.zeros(max(self.ne, 1), dtype=torch.float64, device=dev)
        self.d_rho0 = torch.zeros(max(self.ne, 1), dtype=torch.float64, device=dev)
        torch.cuda.synchronize(dev)

    def linearize(self):
        p = lambda t: L.C.c_void_p(t.data_ptr())  # noqa: E731
        L.check(L.lib().orbg_ba_set_jacobians(self.ctx.handle, 1 if self.jacobians else 0),
                "orbg_ba_set_jacobians")
        L.check(L.lib().orbg_ba_set_edge_errors(self.ctx.handle, 1 if self.edge_errors else 0),
                "orbg_ba_set_edge_errors")
        L.check(L.lib().orbg_ba_linearize_device(
            self.ctx.handle, p(self.d_poses), self.np, p(self.d_points), self.nq, p(self.d_edges),
            self.ne, p(self.d_off), p(self.d_pe), p(self.d_qoff), p(self.d_qe), p(self.d_eout),
            p(self.d_hpose),
            p(self.d_bpose), p(self.d_hpoint), p(self.d_bpoint)), "orbg_ba_linearize_device")

    def build_system(self):
        """buildSystem alone (orbg_ba_build_system_device): the vertex blocks and H_pl into the
        compact self.d_hpl [nedge][3][6], no per-edge Jacobian / error record (the error pass
        supplies those): the per-iteration pair of a device-resident LM is build_system() +
        errors()."""
        import torch
        if getattr(self, "d_hpl", None) is None:
            self.d_hpl = torch.zeros((max(self.ne, 1), 3, 6), dtype=torch.float64,
                                     device=self.d_hpose.device)
        p = lambda t: L.C.c_void_p(t.data_ptr())  # noqa: E731
        if self.graph is not None:
            L.check(L.lib().orbg_ba_graph_build_system(
                self.ctx.handle, self.graph, p(self.d_poses), p(self.d_points), p(self.d_hpl),
                p(self.d_hpose), p(self.d_bpose), p(self.d_hpoint), p(self.d_bpoint)),
                "orbg_ba_graph_build_system")
            return
        L.check(L.lib().orbg_ba_build_system_device(
            self.ctx.handle, p(self.d_poses), self.np, p(self.d_points), self.nq, p(self.d_edges),
            self.ne, p(self.d_off), p(self.d_pe), p(self.d_qoff), p(self.d_qe), p(self.d_hpl),
            p(self.d_hpose), p(self.d_bpose), p(self.d_hpoint), p(self.d_bpoint)),
            "orbg_ba_build_system_device")

    def errors(self):
        """The per-trial error pass (orbg_ba_errors_device): chi2 and the robust term of every
        edge into self.d_chi2 / self.d_rho0."""
        p = lambda t: L.C.c_void_p(t.data_ptr())  # noqa: E731
        if self.graph is not None:
            L.check(L.lib().orbg_ba_graph_errors(self.ctx.handle, self.graph, p(self.d_poses),
                                                 p(self.d_points), None, p(self.d_chi2),
                                                 p(self.d_rho0), None), "orbg_ba_graph_errors")
            return
        L.check(L.lib().orbg_ba_errors_device(self.ctx.handle, p(self.d_poses), p(self.d_points),
                                              p(self.d_edges), self.ne, None, p(self.d_chi2),
                                              p(self.d_rho0), None), "orbg_ba_errors_device")

    def set_active(self, active):
        """The outlier pass's setLevel (Optimizer.cc:871-901) on the graph: active[e] per edge."""
        a = np.ascontiguousarray(np.asarray(active) != 0, np.uint8)
        if self.graph is None:
            raise ValueError("set_active needs a DeviceLBA built with graph=True")
        L.check(L.lib().orbg_ba_graph_set_active(self.ctx.handle, self.graph, a.ctypes.data),
                "orbg_ba_graph_set_active")

    def schur_plan(self, fixed):
        """orbg_ba_graph_schur_plan: the Schur structure of the graph for the free poses
        (fixed[i] != 0: g2o's fixed vertex), built once; set_active rebuilds it."""
        import torch
        if self.graph is None:
            raise ValueError("schur_plan needs a DeviceLBA built with graph=True")
        f = np.ascontiguousarray(np.asarray(fixed) != 0, np.uint8)
        L.check(L.lib().orbg_ba_graph_schur_plan(self.ctx.handle, self.graph, f.ctypes.data),
                "orbg_ba_graph_schur_plan")
        dev = self.d_hpose.device
        self.d_dx_pose = torch.zeros((self.np, 6), dtype=torch.float64, device=dev)
        self.d_dx_point = torch.zeros((self.nq, 3), dtype=torch.float64, device=dev)
        self.d_ok = torch.zeros(1, dtype=torch.int32, device=dev)

    def schur_solve(self, lam):
        """BlockSolver<6,3>::solve on the device blocks of the last build_system()
        (orbg_ba_graph_schur_solve): increments into self.d_dx_pose / self.d_dx_point,
        self.d_ok, on the context stream with no host copy."""
        p = lambda t: L.C.c_void_p(t.data_ptr())  # noqa: E731
        L.check(L.lib().orbg_ba_graph_schur_solve(
            self.ctx.handle, self.graph, float(lam), p(self.d_hpl), p(self.d_hpose),
            p(self.d_bpose), p(self.d_hpoint), p(self.d_bpoint), p(self.d_dx_pose),
            p(self.d_dx_point), p(self.d_ok)), "orbg_ba_graph_schur_solve")

    def set_robust(self, robust):
        """setRobustKernel per edge (orbg_ba_graph_set_robust): robust[e] != 0 keeps Huber."""
        r = np.ascontiguousarray(np.asarray(robust) != 0, np.uint8)
        L.check(L.lib().orbg_ba_graph_set_robust(self.ctx.handle, self.graph, r.ctypes.data),
                "orbg_ba_graph_set_robust")

    def update(self):
        """SparseOptimizer::update with the last schur_solve's increments, in place on the
        device estimates (orbg_ba_update_device; fixed poses untouched)."""
        p = lambda t: L.C.c_void_p(t.data_ptr())  # noqa: E731
        L.check(L.lib().orbg_ba_update_device(
            self.ctx.handle, p(self.d_poses), self.np, p(self.d_points), self.nq,
            p(self.d_dx_pose), p(self.d_dx_point), p(self.d_poses), p(self.d_points)),
            "orbg_ba_update_device")

    def optimize(self, iterations):
        """optimizer.optimize(iterations) (Optimizer.cc:857, :905) with g2o's
        Levenberg-Marquardt on the device estimates (orbg_ba_graph_optimize): build, Schur
        solve, update and error pass per trial on the context stream, three scalars read
        back per trial.  Needs schur_plan(fixed).  Returns the orbg_lm_report as a dict."""
        if self.graph is None:
            raise ValueError("optimize needs a DeviceLBA built with graph=True")
        return self.optimize_ctl(iterations)

    def optimize_ctl(self, iterations, stop_flag=None, post_iteration=None, post_trial=None,
                     last_chi2=None):
        """optimize(iterations) with g2o's force-stop flag (orbg_ba_graph_optimize_ctl):
        `stop_flag` a one-byte host buffer (e.g. numpy uint8 [1], or ctypes c_bool) polled
        before every iteration and after every trial as SparseOptimizer::terminate()
        (sparse_optimizer.cpp:376, optimization_algorithm_levenberg.cpp:149);
        `post_iteration(it)` / `post_trial(it, trial)` Python callbacks (they may raise the
        flag); `last_chi2` a float64 CUDA tensor [nedge] that receives the chi2 g2o's edges
        hold afterwards (the last trial's).  Returns the report as a dict (terminated 3 =
        stopped by the flag)."""
        if self.graph is None:
            raise ValueError("optimize needs a DeviceLBA built with graph=True")
        rep = L.LmReport()
        ctl = L.LmControl()
        if stop_flag is not None:
            if isinstance(stop_flag, np.ndarray):
                assert stop_flag.dtype == np.uint8 and stop_flag.size >= 1
                ctl.force_stop = stop_flag.ctypes.data
            else:
                ctl.force_stop = L.C.addressof(stop_flag)
        # keep the thunks alive for the call
        pi = L.LM_POST_ITERATION((lambda u, it: post_iteration(it)) if post_iteration else 0)
        pt = L.LM_POST_TRIAL((lambda u, it, tr: post_trial(it, tr)) if post_trial else 0)
        ctl.post_iteration, ctl.post_trial = pi, pt
        if last_chi2 is not None:
            import torch
            assert last_chi2.dtype == torch.float64 and last_chi2.is_cuda
            assert last_chi2.numel() == self.ne
            ctl.d_last_chi2 = last_chi2.data_ptr()
        p = lambda t: L.C.c_void_p(t.data_ptr())  # noqa: E731
        L.check(L.lib().orbg_ba_graph_optimize_ctl(self.ctx.handle, self.graph, p(self.d_poses),
                                                   p(self.d_points), int(iterations),
                                                   L.C.byref(ctl), L.C.byref(rep)),
                "orbg_ba_graph_optimize_ctl")
        return dict(iterations=rep.iterations, trials=rep.trials, terminated=rep.terminated,
                    initial_chi2=rep.initial_chi2, final_chi2=rep.final_chi2,
                    **{"lambda": rep.lam})

    def estimates(self):
        """(poses, points) of the device estimates, host copies."""
        self.ctx.sync()
        poses = np.frombuffer(self.d_poses.cpu().numpy().tobytes(), L.POSE_DTYPE).copy()
        points = np.frombuffer(self.d_points.cpu().numpy().tobytes(), np.float64).reshape(-1, 3).copy()
        return poses, points

    def __del__(self):
        if getattr(self, "graph", None) is not None:
            L.lib().orbg_ba_graph_destroy(self.graph)
            self.graph = None

    def download(self):
        self.ctx.sync()
        eo = np.frombuffer(self.d_eout.cpu().numpy().tobytes(), L.EDGE_OUT_DTYPE)
        return (eo, self.d_hpose.cpu().numpy(), self.d_bpose.cpu().numpy(),
                self.d_hpoint.cpu().numpy(), self.d_bpoint.cpu().numpy())
