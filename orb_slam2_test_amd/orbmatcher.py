"""ORBmatcher -- mirror of ORB_SLAM2::ORBmatcher's frame-to-frame path over liborbg.

Reference: include/ORBmatcher.h:40-193, src/ORBmatcher.cc.

    m = ORBmatcher(nnratio=0.9, checkOri=True)
    nmatches, vnMatches12 = m.SearchForInitialization(F1, F2, vbPrevMatched, windowSize=100)
    d = ORBmatcher.DescriptorDistance(a, b)

``Frame`` here carries just what the matcher reads from ORB_SLAM2::Frame
(mvKeysUn, mDescriptors and the image bounds mnMinX/mnMaxX/mnMinY/mnMaxY that define
the 64x48 keypoint grid, Frame.cc:292-307, 421-520, 580-610).  vbPrevMatched is an
(N1, 2) float32 array updated in place, as the reference updates its vector.
"""
import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib as L

_ctx_by_device = {}


def _ctx(device=0):
    c = _ctx_by_device.get(device)
    if c is None:
        c = L.Context(device)
        _ctx_by_device[device] = c
    return c


@dataclass
class Frame:
    """The subset of ORB_SLAM2::Frame the matcher reads."""
    mvKeysUn: np.ndarray          # KP_DTYPE structured array
    mDescriptors: np.ndarray      # (N, 32) uint8
    mnMinX: float = 0.0
    mnMaxX: float = 0.0
    mnMinY: float = 0.0
    mnMaxY: float = 0.0

    @classmethod
    def from_extraction(cls, keypoints, descriptors, width, height):
        # undistorted KITTI-style images: mvKeysUn = mvKeys, bounds = image (Frame.cc:603-609)
        return cls(np.ascontiguousarray(keypoints, L.KP_DTYPE),
                   np.ascontiguousarray(descriptors, np.uint8), 0.0, float(width), 0.0,
                   float(height))

    @property
    def N(self):
        return len(self.mvKeysUn)


class ORBmatcher:
    TH_HIGH = 100
    TH_LOW = 50
    HISTO_LENGTH = 30

    def __init__(self, nnratio=0.6, checkOri=True, device=0):
        self.mfNNratio = float(nnratio)
        self.mbCheckOrientation = bool(checkOri)
        self.device = device

    @staticmethod
    def DescriptorDistance(a, b):
        a = np.ascontiguousarray(a, np.uint8).reshape(32)
        b = np.ascontiguousarray(b, np.uint8).reshape(32)
        return L.lib().orbg_descriptor_distance(L.ptr(a), L.ptr(b))

    def SearchForInitialization(self, F1, F2, vbPrevMatched, windowSize=10):
        k1 = np.ascontiguousarray(F1.mvKeysUn, L.KP_DTYPE)
        k2 = np.ascontiguousarray(F2.mvKeysUn, L.KP_DTYPE)
        d1 = np.ascontiguousarray(F1.mDescriptors, np.uint8)
        d2 = np.ascontiguousarray(F2.mDescriptors, np.uint8)
        if vbPrevMatched.dtype != np.float32 or not vbPrevMatched.flags.c_contiguous:
            raise ValueError("vbPrevMatched must be a C-contiguous float32 (N1, 2) array")
        m12 = np.full(len(k1), -1, np.int32)
        nm = C.c_int()
        b = L.Bounds(F2.mnMinX, F2.mnMaxX, F2.mnMinY, F2.mnMaxY)
        L.check(L.lib().orbg_search_for_initialization(
            _ctx(self.device).handle, L.ptr(k1), L.ptr(d1), len(k1), L.ptr(k2), L.ptr(d2),
            len(k2), C.byref(b), L.ptr(vbPrevMatched), L.ptr(m12), int(windowSize),
            self.mfNNratio, 1 if self.mbCheckOrientation else 0, C.byref(nm)),
            "orbg_search_for_initialization")
        return nm.value, m12

    def hamming_knn2(self, query_desc, train_desc):
        """Brute-force 2-NN: (best_idx, best_dist, second_dist) per query row."""
        q = np.ascontiguousarray(query_desc, np.uint8)
        t = np.ascontiguousarray(train_desc, np.uint8)
        bi = np.zeros(len(q), np.int32)
        bd = np.zeros(len(q), np.int32)
        sd = np.zeros(len(q), np.int32)
        L.check(L.lib().orbg_hamming_knn2(_ctx(self.device).handle, L.ptr(q), len(q), L.ptr(t),
                                          len(t), L.ptr(bi), L.ptr(bd), L.ptr(sd)),
                "orbg_hamming_knn2")
        return bi, bd, sd
