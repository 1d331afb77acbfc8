"""StereoFrame -- the stereo constructor of ORB_SLAM2::Frame over liborbg.

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
