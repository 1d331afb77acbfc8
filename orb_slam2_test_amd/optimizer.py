"""Optimizer -- the per-edge arithmetic of Optimizer::LocalBundleAdjustment on the GPU.

Reference: src/Optimizer.cc:633-979 builds a g2o graph with EdgeSE3ProjectXYZ /
EdgeStereoSE3ProjectXYZ edges (Huber delta sqrt(5.991) / sqrt(7.815), information
invSigma2 * I) and runs Levenberg-Marquardt.  The LM driver, Schur solve and map
write-back stay on the host (they are sequential); this module replaces the
arithmetic g2o performs per edge in computeActiveErrors + BlockSolver::buildSystem:
residual, analytic Jacobians, chi2, Huber weight and the J^T W J / J^T W r blocks.

Arrays use the dtypes of ``_lib`` (POSE_DTYPE, EDGE_DTYPE, EDGE_OUT_DTYPE).
"""
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
