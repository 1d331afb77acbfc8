"""ORBmatcher -- mirror of ORB_SLAM2::ORBmatcher's frame-to-frame path over liborbg.

Reference: include/ORBmatcher.h:40-193, src/ORBmatcher.cc.

    m = ORBmatcher(nnratio=0.9, checkOri=True)
    nmatches, vnMatches12 = m.SearchForInitialization(F1, F2, vbPrevMatched, windowSize=100)
    d = ORBmatcher.DescriptorDistance(a, b)
    n, match = m.SearchByProjection(CurrentFrame, LastFrame, th, bMono)   # motion model
    n, match = m.SearchByProjection(F, vpMapPoints, th)                   # local map
    n, match = m.SearchByBoW(pKF, F)                                      # reference KF / reloc
    n, match12 = m.SearchByBoW_KF(pKF1, pKF2)                             # loop closing
    n, vMatches12 = m.SearchForTriangulation(pKF1, pKF2, F12, bOnlyStereo) # LocalMapping
    n, best_idx, best_dist = m.Fuse(pKF, fcam, map_points, map_desc, th)   # its search

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
    """The subset of ORB_SLAM2::Frame the matchers read."""
    mvKeysUn: np.ndarray          # KP_DTYPE structured array
    mDescriptors: np.ndarray      # (N, 32) uint8
    mnMinX: float = 0.0
    mnMaxX: float = 0.0
    mnMinY: float = 0.0
    mnMaxY: float = 0.0
    # tracking state (SearchByProjection)
    mvuRight: np.ndarray = None   # (N,) float32, None = monocular
    mTcw: np.ndarray = None       # (3, 4) float32 rows of the pose
    fx: float = 0.0
    fy: float = 0.0
    cx: float = 0.0
    cy: float = 0.0
    mbf: float = 0.0
    mb: float = 0.0
    # mvpMapPoints[i] && mvpMapPoints[i]->Observations() > 0 on entry, (N,) uint8 or None
    taken: np.ndarray = None
    # LastFrame.mvpMapPoints as LF_DTYPE records (+ their descriptors), one per keypoint
    points: np.ndarray = None
    point_desc: np.ndarray = None
    # SearchByBoW: mvKeys (distorted keypoints; None = mvKeysUn), mFeatVec as the
    # (fv_nodes, fv_off, fv_feats) arrays Vocabulary.transform_arrays returns, and on a
    # KeyFrame map_valid[i] = "mvpMapPoints[i] && !mvpMapPoints[i]->isBad()" (None = all)
    mvKeys: np.ndarray = None
    mFeatVec: tuple = None
    map_valid: np.ndarray = None
    # SearchForTriangulation: GetMapPoint(i) != NULL, (N,) uint8 or None (none)
    has_mp: np.ndarray = None

    @classmethod
    def from_extraction(cls, keypoints, descriptors, width, height):
        # undistorted KITTI-style images: mvKeysUn = mvKeys, bounds = image (Frame.cc:603-609)
        return cls(np.ascontiguousarray(keypoints, L.KP_DTYPE),
                   np.ascontiguousarray(descriptors, np.uint8), 0.0, float(width), 0.0,
                   float(height))

    @property
    def N(self):
        return len(self.mvKeysUn)


@dataclass
class MapPointProjections:
    """vpMapPoints after Frame::isInFrustum: MP_DTYPE records (mTrackProjX/Y/XR,
    mnTrackScaleLevel, mTrackViewCos, flags) and pMP->GetDescriptor() rows."""
    records: np.ndarray
    descriptors: np.ndarray


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

    def SearchByBoW(self, pKF, F):
        """SearchByBoW(KeyFrame *pKF, Frame &F, vector<MapPoint*> &vpMapPointMatches)
        (ORBmatcher.cc:195-348).  pKF and F are Frames carrying mFeatVec (pKF also map_valid).
        Returns (nmatches, match): match[i] = the KeyFrame feature whose MapPoint is
        vpMapPointMatches[i], -1 for NULL."""
        def side(fr, keys):
            d = np.ascontiguousarray(fr.mDescriptors, np.uint8).reshape(-1, 32)
            a = np.ascontiguousarray(keys["angle"], np.float32)
            nodes, off, feats = [np.ascontiguousarray(x, np.int32) for x in fr.mFeatVec]
            return d, a, nodes, off, feats
        kd, ka, kn, ko, kf = side(pKF, pKF.mvKeysUn)
        fd, fa, fn, fo, ff = side(F, F.mvKeys if F.mvKeys is not None else F.mvKeysUn)
        kv = None if pKF.map_valid is None else np.ascontiguousarray(pKF.map_valid, np.uint8)
        match = np.full(max(len(fd), 1), -1, np.int32)
        nm = C.c_int()
        L.check(L.lib().orbg_search_by_bow(
            _ctx(self.device).handle, L.ptr(kd), L.ptr(ka), L.ptr(kv), len(kd), L.ptr(kn),
            L.ptr(ko), L.ptr(kf), len(kn), L.ptr(fd), L.ptr(fa), len(fd), L.ptr(fn), L.ptr(fo),
            L.ptr(ff), len(fn), self.mfNNratio, 1 if self.mbCheckOrientation else 0,
            L.ptr(match), C.byref(nm)), "orbg_search_by_bow")
        return nm.value, match[:len(fd)]

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

    def SearchByProjection(self, F, second, th, bMono=True):
        """SearchByProjection(CurrentFrame, LastFrame, th, bMono) (ORBmatcher.cc:1503-1667)
        when `second` is a Frame carrying `points`, SearchByProjection(F, vpMapPoints, th)
        (:59-146) when it is a MapPointProjections.  Returns (nmatches, match): match[i] is
        the LastFrame keypoint / map point index written to F.mvpMapPoints[i], -1 where the
        call wrote nothing, -2 where the rotation filter set the slot to NULL."""
        kps = np.ascontiguousarray(F.mvKeysUn, L.KP_DTYPE)
        desc = np.ascontiguousarray(F.mDescriptors, np.uint8)
        ur = None if F.mvuRight is None else np.ascontiguousarray(F.mvuRight, np.float32)
        tk = None if F.taken is None else np.ascontiguousarray(F.taken, np.uint8)
        b = L.Bounds(F.mnMinX, F.mnMaxX, F.mnMinY, F.mnMaxY)
        match = np.full(len(kps), -1, np.int32)
        nm = C.c_int()
        h = _ctx(self.device).handle
        if isinstance(second, MapPointProjections):
            rec = np.ascontiguousarray(second.records, L.MP_DTYPE)
            md = np.ascontiguousarray(second.descriptors, np.uint8)
            L.check(L.lib().orbg_search_by_projection_local(
                h, L.ptr(kps), L.ptr(desc), L.ptr(ur), len(kps), L.ptr(tk), C.byref(b),
                L.ptr(rec), L.ptr(md), len(rec), float(th), self.mfNNratio, L.ptr(match),
                C.byref(nm)), "orbg_search_by_projection_local")
        else:
            pts = np.ascontiguousarray(second.points, L.LF_DTYPE)
            pd = np.ascontiguousarray(second.point_desc, np.uint8)
            cam = L.track_camera(F.mTcw, second.mTcw, F.fx, F.fy, F.cx, F.cy, F.mbf, F.mb, bMono)
            L.check(L.lib().orbg_search_by_projection_lastframe(
                h, L.ptr(kps), L.ptr(desc), L.ptr(ur), len(kps), L.ptr(tk), C.byref(b),
                L.ptr(pts), L.ptr(pd), len(pts), C.byref(cam), float(th),
                1 if self.mbCheckOrientation else 0, L.ptr(match), C.byref(nm)),
                "orbg_search_by_projection_lastframe")
        return nm.value, match

    def SearchByProjection_Reloc(self, F, fcam, kf_points, kf_point_desc, th, ORBdist):
        """SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist)
        (ORBmatcher.cc:1670-1798; Tracking::Relocalization): F with mvKeysUn, mDescriptors and
        taken (mvpMapPoints[i] != NULL, None: none); fcam its FRUSTUM_DTYPE state; kf_points
        RELOC_DTYPE records of pKF->GetMapPointMatches() (flags MP_VALID = pMP && !isBad() &&
        not in sAlreadyFound; angle = pKF->mvKeysUn[i].angle).  Returns (nmatches, match):
        match[i2] = the pKF index written to mvpMapPoints[i2], -1, or -2 (rotation filter)."""
        kps = np.ascontiguousarray(F.mvKeysUn, L.KP_DTYPE)
        desc = np.ascontiguousarray(F.mDescriptors, np.uint8)
        tk = None if F.taken is None else np.ascontiguousarray(F.taken, np.uint8)
        fc = np.ascontiguousarray(fcam, L.FRUSTUM_DTYPE)
        pts = np.ascontiguousarray(kf_points, L.RELOC_DTYPE)
        pd = np.ascontiguousarray(kf_point_desc, np.uint8).reshape(-1, 32)
        match = np.full(max(len(kps), 1), -1, np.int32)
        nm = C.c_int()
        L.check(L.lib().orbg_search_by_projection_reloc(
            _ctx(self.device).handle, L.ptr(kps), L.ptr(desc), len(kps), L.ptr(tk), L.ptr(fc),
            L.ptr(pts), L.ptr(pd), len(pts), float(th), int(ORBdist),
            1 if self.mbCheckOrientation else 0, L.ptr(match), C.byref(nm)),
            "orbg_search_by_projection_reloc")
        return nm.value, match[:len(kps)].copy()

    def SearchByProjection_Sim3(self, pKF, fcam, points, points_desc, th=10):
        """SearchByProjection(pKF, Scw, vpPoints, vpMatched, th) (ORBmatcher.cc:353-470;
        LoopClosing::ComputeSim3): pKF with mvKeysUn, mDescriptors and taken (vpMatched[i] !=
        NULL, None: none); fcam["Tcw"] = Scw rows 0..2 (decomposed on the device), bounds the
        Frame's; points MAPPOINT_DTYPE (flags MP_VALID = !isBad() and not in vpMatched).
        Returns (nmatches, match): match[idx] = the vpPoints index written to vpMatched[idx]."""
        kps = np.ascontiguousarray(pKF.mvKeysUn, L.KP_DTYPE)
        desc = np.ascontiguousarray(pKF.mDescriptors, np.uint8)
        tk = None if pKF.taken is None else np.ascontiguousarray(pKF.taken, np.uint8)
        fc = np.ascontiguousarray(fcam, L.FRUSTUM_DTYPE)
        mps = np.ascontiguousarray(points, L.MAPPOINT_DTYPE)
        md = np.ascontiguousarray(points_desc, np.uint8).reshape(-1, 32)
        match = np.full(max(len(kps), 1), -1, np.int32)
        nm = C.c_int()
        L.check(L.lib().orbg_search_by_projection_sim3(
            _ctx(self.device).handle, L.ptr(kps), L.ptr(desc), len(kps), L.ptr(tk), L.ptr(fc),
            L.ptr(mps), L.ptr(md), len(mps), int(th), L.ptr(match), C.byref(nm)),
            "orbg_search_by_projection_sim3")
        return nm.value, match[:len(kps)].copy()

    def SearchBySim3(self, pKF1, pKF2, mp1, md1, mp2, md2, g, th=7.5, matched1=None,
                     matched2=None):
        """ORBmatcher::SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th)
        (ORBmatcher.cc:1262-1470; LoopClosing::ComputeSim3): pKF1 / pKF2 with mvKeysUn and
        mDescriptors; mp1 / md1 MAPPOINT_DTYPE records + descriptors of
        pKF1->GetMapPointMatches() (flags MP_VALID = pMP && !isBad()), likewise mp2 / md2;
        g a SIM3_PAIR_DTYPE record (poses, s12 / R12 / t12, pKF1's intrinsics, bounds);
        matched1[i] = vpMatches12[i] != NULL, matched2 their indices in pKF2.  Returns
        (nFound, matches12): vpMatches12[i] = pKF2's MapPoint at matches12[i] (>= 0)."""
        def side(fr):
            k = np.ascontiguousarray(fr.mvKeysUn, L.KP_DTYPE)
            d = np.ascontiguousarray(fr.mDescriptors, np.uint8)
            return k, d, L.KeyFrame(L.ptr(k), L.ptr(d), None, None, len(k), None, None, None, 0)
        k1, d1, K1 = side(pKF1)
        k2, d2, K2 = side(pKF2)
        a = [np.ascontiguousarray(x, L.MAPPOINT_DTYPE) for x in (mp1, mp2)]
        b = [np.ascontiguousarray(x, np.uint8).reshape(-1, 32) for x in (md1, md2)]
        m1 = None if matched1 is None else np.ascontiguousarray(matched1, np.uint8)
        m2 = None if matched2 is None else np.ascontiguousarray(matched2, np.uint8)
        gg = np.ascontiguousarray(g, L.SIM3_PAIR_DTYPE)
        out = np.full(max(len(k1), 1), -1, np.int32)
        n = C.c_int()
        L.check(L.lib().orbg_search_by_sim3(
            _ctx(self.device).handle, C.byref(K1), L.ptr(a[0]), L.ptr(b[0]), L.ptr(m1),
            C.byref(K2), L.ptr(a[1]), L.ptr(b[1]), L.ptr(m2), L.ptr(gg), float(th), L.ptr(out),
            C.byref(n)), "orbg_search_by_sim3")
        return n.value, out[:len(k1)].copy()

    def SearchForTriangulation(self, pKF1, pKF2, geom, bOnlyStereo=False):
        """ORBmatcher::SearchForTriangulation(pKF1, pKF2, F12, vMatchedPairs, bOnlyStereo)
        (src/ORBmatcher.cc:779-957).  pKF1 / pKF2: Frames with mvKeysUn, mDescriptors,
        mFeatVec, mvuRight (None: monocular) and has_mp (GetMapPoint(i) != NULL, None: none);
        geom: a TRI_GEOM_DTYPE record (F12, pKF1's camera centre, pKF2's pose and
        intrinsics).  Returns (nmatches, vMatches12); vMatchedPairs = the (i, vMatches12[i])
        with vMatches12[i] >= 0."""
        keep = []

        def side(fr):
            kps = np.ascontiguousarray(fr.mvKeysUn, L.KP_DTYPE)
            desc = np.ascontiguousarray(fr.mDescriptors, np.uint8)
            ur = None if fr.mvuRight is None else np.ascontiguousarray(fr.mvuRight, np.float32)
            mp = None if fr.has_mp is None else np.ascontiguousarray(fr.has_mp, np.uint8)
            nodes, off, feats = (np.ascontiguousarray(a, np.int32) for a in fr.mFeatVec)
            keep.extend([kps, desc, ur, mp, nodes, off, feats])
            return L.KeyFrame(L.ptr(kps), L.ptr(desc), L.ptr(ur), L.ptr(mp), len(kps),
                              L.ptr(nodes), L.ptr(off), L.ptr(feats), len(nodes))

        a, b = side(pKF1), side(pKF2)
        g = np.ascontiguousarray(geom, L.TRI_GEOM_DTYPE)
        m = np.zeros(max(a.n, 1), np.int32)
        n = C.c_int()
        L.check(L.lib().orbg_search_for_triangulation(_ctx(self.device).handle, C.byref(a),
                                                      C.byref(b), L.ptr(g),
                                                      1 if bOnlyStereo else 0,
                                                      1 if self.mbCheckOrientation else 0,
                                                      L.ptr(m), C.byref(n)),
                "orbg_search_for_triangulation")
        return n.value, m[:a.n].copy()

    def Fuse(self, pKF, fcam, map_points, map_desc, th=3.0):
        """ORBmatcher::Fuse(pKF, vpMapPoints, th)'s search (src/ORBmatcher.cc:968-1069):
        pKF a Frame with mvKeysUn / mDescriptors / mvuRight, fcam its FRUSTUM_DTYPE state
        (pose, intrinsics, mbf, mfLogScaleFactor, mnScaleLevels, bounds), map_points
        MAPPOINT_DTYPE records (flags MP_VALID = pMP && !isBad() && !IsInKeyFrame(pKF)) with
        map_desc their descriptors.  Returns (nfused, best_idx, best_dist): the reference
        fuses point i with pKF's feature best_idx[i] (>= 0); the Replace / AddObservation
        update is the caller's, in vpMapPoints order."""
        kps = np.ascontiguousarray(pKF.mvKeysUn, L.KP_DTYPE)
        desc = np.ascontiguousarray(pKF.mDescriptors, np.uint8)
        ur = None if pKF.mvuRight is None else np.ascontiguousarray(pKF.mvuRight, np.float32)
        kf = L.KeyFrame(L.ptr(kps), L.ptr(desc), L.ptr(ur), None, len(kps), None, None, None, 0)
        fc = np.ascontiguousarray(fcam, L.FRUSTUM_DTYPE)
        mps = np.ascontiguousarray(map_points, L.MAPPOINT_DTYPE)
        md = np.ascontiguousarray(map_desc, np.uint8).reshape(-1, 32)
        bi = np.zeros(max(len(mps), 1), np.int32)
        bd = np.zeros(max(len(mps), 1), np.int32)
        n = C.c_int()
        L.check(L.lib().orbg_fuse(_ctx(self.device).handle, C.byref(kf), L.ptr(fc), L.ptr(mps),
                                  L.ptr(md), len(mps), float(th), L.ptr(bi), L.ptr(bd),
                                  C.byref(n)), "orbg_fuse")
        return n.value, bi[:len(mps)].copy(), bd[:len(mps)].copy()

    def FuseSim3(self, pKF, fcam, points, points_desc, th=4.0):
        """ORBmatcher::Fuse(pKF, Scw, vpPoints, th, vpReplacePoint)'s search
        (src/ORBmatcher.cc:1133-1238; LoopClosing::SearchAndFuse, th 4): fcam["Tcw"] holds
        Scw's rows 0..2 (decomposed on the device as the reference does), points
        MAPPOINT_DTYPE records (flags MP_VALID = !isBad() and not already in pKF), no
        reprojection gate.  Returns (nfused, best_idx, best_dist); the caller fills
        vpReplacePoint / adds observations in vpPoints order."""
        kps = np.ascontiguousarray(pKF.mvKeysUn, L.KP_DTYPE)
        desc = np.ascontiguousarray(pKF.mDescriptors, np.uint8)
        kf = L.KeyFrame(L.ptr(kps), L.ptr(desc), None, None, len(kps), None, None, None, 0)
        fc = np.ascontiguousarray(fcam, L.FRUSTUM_DTYPE)
        mps = np.ascontiguousarray(points, L.MAPPOINT_DTYPE)
        md = np.ascontiguousarray(points_desc, np.uint8).reshape(-1, 32)
        bi = np.zeros(max(len(mps), 1), np.int32)
        bd = np.zeros(max(len(mps), 1), np.int32)
        n = C.c_int()
        L.check(L.lib().orbg_fuse_sim3(_ctx(self.device).handle, C.byref(kf), L.ptr(fc),
                                       L.ptr(mps), L.ptr(md), len(mps), float(th), L.ptr(bi),
                                       L.ptr(bd), C.byref(n)), "orbg_fuse_sim3")
        return n.value, bi[:len(mps)].copy(), bd[:len(mps)].copy()

    def SearchByBoW_KF(self, pKF1, pKF2):
        """ORBmatcher::SearchByBoW(KeyFrame *pKF1, KeyFrame *pKF2, vpMatches12)
        (src/ORBmatcher.cc:634-769): both KeyFrames with mvKeysUn, mDescriptors, mFeatVec and
        map_valid (pMP && !isBad(), None: all).  Returns (nmatches, match12) with match12[i]
        the pKF2 feature matched to pKF1's feature i (vpMatches12[i] = its MapPoint), -1."""
        def side(fr):
            d = np.ascontiguousarray(fr.mDescriptors, np.uint8)
            a = np.ascontiguousarray(fr.mvKeysUn["angle"], np.float32)
            v = None if fr.map_valid is None else np.ascontiguousarray(fr.map_valid, np.uint8)
            nodes, off, feats = (np.ascontiguousarray(x, np.int32) for x in fr.mFeatVec)
            return d, a, v, nodes, off, feats
        d1, a1, v1, n1, o1, f1 = side(pKF1)
        d2, a2, v2, n2, o2, f2 = side(pKF2)
        m = np.zeros(max(len(d1), 1), np.int32)
        n = C.c_int()
        L.check(L.lib().orbg_search_by_bow_kf(
            _ctx(self.device).handle, L.ptr(d1), L.ptr(a1), L.ptr(v1), len(d1), L.ptr(n1),
            L.ptr(o1), L.ptr(f1), len(n1), L.ptr(d2), L.ptr(a2), L.ptr(v2), len(d2), L.ptr(n2),
            L.ptr(o2), L.ptr(f2), len(n2), float(self.mfNNratio),
            1 if self.mbCheckOrientation else 0, L.ptr(m), C.byref(n)), "orbg_search_by_bow_kf")
        return n.value, m[:len(d1)].copy()
