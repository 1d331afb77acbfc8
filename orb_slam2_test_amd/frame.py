"""Frame geometry and the stereo constructor of ORB_SLAM2::Frame over liborbg.

    cam = camera(fx, fy, cx, cy, k1, k2, p1, p2, k3)      # Frame::mK + mDistCoef
    mvKeysUn = undistort_keypoints(cam, mvKeys)           # Frame::UndistortKeyPoints
    mnMinX, mnMaxX, mnMinY, mnMaxY = compute_image_bounds(cam, w, h)  # ComputeImageBounds
    proj, n = is_in_frustum(frustum_camera(...), map_points, 0.5)      # Frame::isInFrustum

References: src/Frame.cc:542-572 (UndistortKeyPoints), :575-611 (ComputeImageBounds),
:342-409 (isInFrustum, MapPoint::PredictScale src/MapPoint.cc:575-590).

Reference: src/Frame.cc:86-161 (two ORBextractor calls on the left/right images, Frame.cc
:110-113, then ComputeStereoMatches, :619-834).  The fields mirror Frame's:

    F = StereoFrame(imLeft, imRight, ext, bf)       # ext: an ORBextractor (the context)
    F.mvKeys, F.mDescriptors, F.mvKeysRight, F.mDescriptorsRight, F.mvuRight, F.mvDepth, F.N

``mb`` (minZ of the disparity search) is read uninitialised by the reference
(Frame.cc:661 vs :148); the default here is bf / fx, the value assigned right after.
"""
import ctypes as C

import numpy as np

from . import _lib as L


def _default_ctx(device=0):
    from .orbmatcher import _ctx
    return _ctx(device)


def camera(fx, fy, cx, cy, k1=0.0, k2=0.0, p1=0.0, p2=0.0, k3=0.0):
    """orbg_camera: Frame::mK (fx, fy, cx, cy) and mDistCoef (k1, k2, p1, p2[, k3])."""
    c = np.zeros((), L.CAMERA_DTYPE)
    for k, v in zip(L.CAMERA_DTYPE.names, (fx, fy, cx, cy, k1, k2, p1, p2, k3)):
        c[k] = v
    return c


def undistort_keypoints(cam, mvKeys, ctx=None):
    """Frame::UndistortKeyPoints: mvKeysUn (a copy when k1 == 0)."""
    cam = np.ascontiguousarray(cam, L.CAMERA_DTYPE)
    kps = np.ascontiguousarray(mvKeys, L.KP_DTYPE)
    out = np.zeros_like(kps)
    ctx = ctx or _default_ctx()
    L.check(L.lib().orbg_undistort_keypoints(ctx.handle, L.ptr(cam), L.ptr(kps), len(kps),
                                             L.ptr(out)), "orbg_undistort_keypoints")
    return out


def compute_stereo_from_rgbd(depth, depth_map_factor, mvKeys, mvKeysUn, mbf, ctx=None):
    """Frame::ComputeStereoFromRGBD (src/Frame.cc:837-858) with Tracking::GrabImageRGBD's
    depth conversion (Tracking.cc:233-234): depth the (h, w) uint16 or float32 image as
    GrabImageRGBD receives it, depth_map_factor = mDepthMapFactor (1 / the settings'
    DepthMapFactor).  Returns (mvuRight, mvDepth), -1 where there is no depth."""
    depth = np.ascontiguousarray(depth)
    if depth.dtype not in (np.uint16, np.float32):
        raise ValueError("depth must be uint16 or float32")
    kps = np.ascontiguousarray(mvKeys, L.KP_DTYPE)
    kun = np.ascontiguousarray(mvKeysUn, L.KP_DTYPE)
    if len(kps) != len(kun):
        raise ValueError("mvKeys and mvKeysUn differ in length")
    ur = np.zeros(max(len(kps), 1), np.float32)
    dd = np.zeros(max(len(kps), 1), np.float32)
    h, w = depth.shape
    c = ctx or _default_ctx()
    L.check(L.lib().orbg_rgbd_stereo(c.handle, L.ptr(depth),
                                     L.DEPTH_U16 if depth.dtype == np.uint16 else L.DEPTH_F32,
                                     float(np.float32(depth_map_factor)), w, h, depth.strides[0],
                                     L.ptr(kps), L.ptr(kun), len(kps), float(np.float32(mbf)),
                                     L.ptr(ur), L.ptr(dd)), "orbg_rgbd_stereo")
    return ur[:len(kps)].copy(), dd[:len(kps)].copy()


def compute_image_bounds(cam, width, height):
    """Frame::ComputeImageBounds: (mnMinX, mnMaxX, mnMinY, mnMaxY)."""
    cam = np.ascontiguousarray(cam, L.CAMERA_DTYPE)
    b = L.Bounds()
    L.check(L.lib().orbg_compute_image_bounds(L.ptr(cam), int(width), int(height), C.byref(b)),
            "orbg_compute_image_bounds")
    return b.min_x, b.max_x, b.min_y, b.max_y


def frustum_camera(Tcw, fx, fy, cx, cy, bf, log_scale_factor, nlevels, bounds):
    """orbg_frustum_camera: the Frame state isInFrustum reads (mTcw rows 0..2, intrinsics,
    mbf, mfLogScaleFactor, mnScaleLevels, mnMinX/mnMaxX/mnMinY/mnMaxY)."""
    c = np.zeros((), L.FRUSTUM_DTYPE)
    c["Tcw"] = np.asarray(Tcw, np.float32).reshape(12)
    for k, v in zip(("fx", "fy", "cx", "cy", "bf", "log_scale_factor"),
                    (fx, fy, cx, cy, bf, log_scale_factor)):
        c[k] = v
    c["nlevels"] = nlevels
    c["min_x"], c["max_x"], c["min_y"], c["max_y"] = bounds
    return c


def is_in_frustum(fcam, map_points, viewingCosLimit=0.5, proj=None, ctx=None):
    """Frame::isInFrustum(pMP, viewingCosLimit) for MAPPOINT_DTYPE records: the mTrack*
    members as MP_DTYPE records (flags MP_VALID = mbTrackInView) and the number in view.
    proj: the records before the call (a point out of view keeps all but its flags)."""
    fcam = np.ascontiguousarray(fcam, L.FRUSTUM_DTYPE)
    mps = np.ascontiguousarray(map_points, L.MAPPOINT_DTYPE)
    out = np.zeros(len(mps), L.MP_DTYPE) if proj is None else np.array(proj, L.MP_DTYPE)
    nv = C.c_int()
    ctx = ctx or _default_ctx()
    L.check(L.lib().orbg_is_in_frustum(ctx.handle, L.ptr(fcam), L.ptr(mps), len(mps),
                                       float(viewingCosLimit), L.ptr(out), C.byref(nv)),
            "orbg_is_in_frustum")
    return out, nv.value


class StereoFrame:
    def __init__(self, imLeft, imRight, extractor, bf, fx=None, mb=None):
        imLeft = np.ascontiguousarray(imLeft, np.uint8)
        imRight = np.ascontiguousarray(imRight, np.uint8)
        if imLeft.shape != imRight.shape or imLeft.ndim != 2:
            raise ValueError("left and right must be 2-D u8 images of one size")
        h, w = imLeft.shape
        self.mbf = float(bf)
        if mb is None:
            if fx is None:
                raise ValueError("give fx (mb = bf / fx) or mb")
            mb = float(np.float32(bf) / np.float32(fx))
        self.mb = float(mb)
        cap = 8192  # grown on ORBG_ERANGE
        while True:
            kl = np.zeros(cap, L.KP_DTYPE)
            dl = np.zeros((cap, 32), np.uint8)
            kr = np.zeros(cap, L.KP_DTYPE)
            dr = np.zeros((cap, 32), np.uint8)
            ur = np.zeros(cap, np.float32)
            dp = np.zeros(cap, np.float32)
            nl, nr = C.c_int(), C.c_int()
            rc = L.lib().orbg_stereo_frame(extractor.ctx.handle, L.ptr(imLeft), L.ptr(imRight), w,
                                           h, w, float(bf), float(mb), L.ptr(kl), L.ptr(dl), cap,
                                           C.byref(nl), L.ptr(kr), L.ptr(dr), cap, C.byref(nr),
                                           L.ptr(ur), L.ptr(dp))
            if rc == L.ORBG_ERANGE:
                cap = max(nl.value, nr.value)
                continue
            L.check(rc, "orbg_stereo_frame")
            break
        n, m = nl.value, nr.value
        self.mvKeys, self.mDescriptors = kl[:n].copy(), dl[:n].copy()
        self.mvKeysRight, self.mDescriptorsRight = kr[:m].copy(), dr[:m].copy()
        self.mvuRight, self.mvDepth = ur[:n].copy(), dp[:n].copy()
        self.N = n
