"""LocalMapping -- mirror of ORB_SLAM2::LocalMapping::CreateNewMapPoints' per-pair work over
liborbg (the geometry and the triangulation either side of ORBmatcher.SearchForTriangulation).

Reference: src/LocalMapping.cc:293-560 (CreateNewMapPoints), :690-707 (ComputeF12),
src/KeyFrame.cc:798-814 (UnprojectStereo).

    cam1 = kf_camera(Tcw1, fx, fy, cx, cy, mb, mbf)          # pKF1 = mpCurrentKeyFrame
    cam2 = kf_camera(Tcw2, ...)                               # pKF2 = a covisible neighbour
    lm = LocalMapping()
    geom = lm.ComputeF12(cam1, cam2)                          # F12 + the epipole inputs
    n, vMatches12 = ORBmatcher(0.6, False).SearchForTriangulation(pKF1, pKF2, geom)
    nnew, x3D, status = lm.Triangulate(pKF1, pKF2, cam1, cam2, vMatches12)

The reference's per-neighbour loop (GetBestCovisibilityKeyFrames, the baseline test, the
MapPoint creation for every status == TRI_NEW in feature order) is host control flow and stays
the caller's; batches of pairs go through orbg_triangulation_geometry_batch_device /
orbg_triangulate_batch_device (include/orbg.h).  ``pKF`` here is any object with mvKeysUn and,
for stereo, mvuRight / mvDepth (mvKeys: the distorted keypoints UnprojectStereo reads; None:
mvKeysUn).  There is no CPU path: without liborbg the calls raise.
"""
import ctypes as C

import numpy as np

from . import _lib as L
from .orbmatcher import _ctx


def kf_camera(Tcw, fx, fy, cx, cy, mb=0.0, mbf=0.0):
    """orbg_kf_camera of a KeyFrame: mTcw rows 0..2 (3x4 float32), intrinsics, invfx = 1/fx
    as Frame.cc computes it (float division), mb, mbf."""
    c = np.zeros((), L.KF_CAMERA_DTYPE)
    c["Tcw"] = np.asarray(Tcw, np.float32).reshape(-1)[:12]
    c["fx"], c["fy"], c["cx"], c["cy"] = fx, fy, cx, cy
    c["invfx"] = np.float32(1.0) / np.float32(fx)
    c["invfy"] = np.float32(1.0) / np.float32(fy)
    c["mb"], c["mbf"] = mb, mbf
    return c


class LocalMapping:
    def __init__(self, device=0):
        self.device = device

    def ComputeF12(self, cam1, cam2):
        """LocalMapping::ComputeF12(pKF1, pKF2) -> TRI_GEOM_DTYPE record (F12, pKF1's camera
        centre, pKF2's pose and intrinsics), as SearchForTriangulation takes it."""
        a = np.ascontiguousarray(cam1, L.KF_CAMERA_DTYPE)
        b = np.ascontiguousarray(cam2, L.KF_CAMERA_DTYPE)
        g = np.zeros((), L.TRI_GEOM_DTYPE)
        L.check(L.lib().orbg_triangulation_geometry(_ctx(self.device).handle, L.ptr(a), L.ptr(b),
                                                    L.ptr(g)), "orbg_triangulation_geometry")
        return g

    def Triangulate(self, pKF1, pKF2, cam1, cam2, vMatches12):
        """The triangulation loop of CreateNewMapPoints over one neighbour's vMatchedPairs
        (given as vMatches12, SearchForTriangulation's per-feature form) -> (nnew, x3D[N1, 3],
        status[N1]): status[i] == TRI_NEW where the reference creates a MapPoint at x3D[i];
        the other TRI_* codes name the test that rejected the pair."""
        keep = []

        def side(fr):
            kps = np.ascontiguousarray(fr.mvKeysUn, L.KP_DTYPE)
            raw = getattr(fr, "mvKeys", None)
            raw = None if raw is None else np.ascontiguousarray(raw, L.KP_DTYPE)
            ur = getattr(fr, "mvuRight", None)
            ur = None if ur is None else np.ascontiguousarray(ur, np.float32)
            dp = getattr(fr, "mvDepth", None)
            dp = None if dp is None else np.ascontiguousarray(dp, np.float32)
            keep.extend([kps, raw, ur, dp])
            return L.KeyFrameGeo(L.ptr(kps), L.ptr(raw), L.ptr(ur), L.ptr(dp), len(kps))

        a, b = side(pKF1), side(pKF2)
        ca = np.ascontiguousarray(cam1, L.KF_CAMERA_DTYPE)
        cb = np.ascontiguousarray(cam2, L.KF_CAMERA_DTYPE)
        m = np.ascontiguousarray(vMatches12, np.int32)
        if len(m) != a.n:
            raise ValueError("vMatches12 must have one entry per pKF1 feature")
        x = np.zeros((max(a.n, 1), 3), np.float32)
        st = np.zeros(max(a.n, 1), np.int8)
        n = C.c_int()
        L.check(L.lib().orbg_triangulate(_ctx(self.device).handle, C.byref(a), C.byref(b),
                                         L.ptr(ca), L.ptr(cb), L.ptr(m), L.ptr(x), L.ptr(st),
                                         C.byref(n)), "orbg_triangulate")
        return n.value, x[:a.n].copy(), st[:a.n].copy()
