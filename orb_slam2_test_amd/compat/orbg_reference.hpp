// orbg_reference.hpp -- the reference-facing drop-in layer: the ORB_SLAM2 call sites of the
// hot path (ORBmatcher, Optimizer) over liborbg's C ABI, written against the reference's
// own classes.
//
// Every function is a template over the reference types (ORB_SLAM2::Frame, KeyFrame,
// MapPoint) and touches only the members the reference functions it replaces touch, with
// the same names, so ORBmatcher.cc / Optimizer.cc keep their signatures and forward to it
// (INTEGRATION.md 3-4):
//
//   int ORBmatcher::SearchForInitialization(Frame &F1, Frame &F2,
//           vector<cv::Point2f> &vbPrevMatched, vector<int> &vnMatches12, int windowSize)
//   { return orbg_compat::ref::SearchForInitialization(ctx, mfNNratio, mbCheckOrientation,
//                                                      F1, F2, vbPrevMatched, vnMatches12,
//                                                      windowSize); }
//
// The cv:: surface used is the stable OpenCV core subset (Mat::rows/cols/at/ptr/eye/clone,
// KeyPoint, Point2f); tests/compat_stub/ holds a test-only stand-in of exactly that subset so
// this header is compiled and run in this repository's tests (tests/test_compat_ref.py),
// where OpenCV is absent.
//
//   SearchForInitialization ......... ORBmatcher.cc:487-631 (include/ORBmatcher.h:47)
//   SearchByProjection (last frame) .. ORBmatcher.cc:1503-1667 (ORBmatcher.h:62)
//   SearchByProjection (local map) ... ORBmatcher.cc:59-154 (ORBmatcher.h:51)
//   SearchByBoW (KeyFrame, Frame) .... ORBmatcher.cc:195-348 (ORBmatcher.h:57)
//   SearchByBoW (KeyFrame, KeyFrame) . ORBmatcher.cc:634-769 (ORBmatcher.h:58)
//   DescriptorDistance ............... ORBmatcher.cc:1846-1862 (ORBmatcher.h:128)
//   PoseOptimization ................. Optimizer.cc:356-631 (include/Optimizer.h:49)
//   UndistortKeyPoints .............. Frame.cc:542-572 (Frame.h:142)
//   ComputeImageBounds .............. Frame.cc:575-611
//   isInFrustum (SearchLocalPoints) . Frame.cc:342-409, Tracking.cc:1676-1691
//   SearchForTriangulation .......... ORBmatcher.cc:779-957 (ORBmatcher.h:72)
//   Fuse(pKF, vpMapPoints, th) ...... ORBmatcher.cc:968-1107 (ORBmatcher.h:153)
//   Fuse(pKF, Scw, vpPoints, th, vpReplacePoint) ORBmatcher.cc:1133-1258 (ORBmatcher.h:162)
//   SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist) ORBmatcher.cc:1670-1798
//   SearchByProjection(pKF, Scw, vpPoints, vpMatched, th) ORBmatcher.cc:353-470
//   SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th) ORBmatcher.cc:1262-1470
//   Frame::ComputeStereoFromRGBD ...... Frame.cc:837-858 (+ Tracking.cc:233-234)
//   ComputeDistinctiveDescriptors ... MapPoint.cc:342-420 (the BestIdx over vDescriptors)
//   LocalBundleAdjustment window ..... Optimizer.cc:633-851: the vertex / edge set g2o builds
//                                      (LbaWindow), and BlockSolver<6,3>::buildSystem's block
//                                      layout of the linearised system (block_solver.hpp:
//                                      502-560, G2oBlockSystem)
//   LocalBundleAdjustment ............ Optimizer.cc:633-979 (include/Optimizer.h:45): the
//                                      whole function, its LM on the device
//                                      (orbg_local_ba_optimize), pbStopFlag honoured
#pragma once

#include <algorithm>
#include <cmath>
#include <cstring>
#include <list>
#include <map>
#include <mutex>
#include <set>
#include <type_traits>
#include <vector>

#include "orbg_compat.hpp"

namespace orbg_compat {
namespace ref {

// The context behind ORBmatcher / Optimizer call sites, which the reference constructs
// freely (ORBmatcher matcher(0.9, true) on the stack): ONE PER CALLING THREAD, device 0,
// default parameters (scale factor 1.2, 8 levels: the ORBextractor settings the tracking
// matchers' scale tables must agree with), created on the thread's first use and destroyed
// at its exit.  The reference calls the matchers and PoseOptimization on the Tracking thread
// while LocalMapping runs LocalBundleAdjustment (System.cc:117, LocalMapping.cc:99), and a
// liborbg context is not thread-safe (include/orbg.h), so each thread gets its own context
// (its own streams, planning state and scratch); distinct contexts run concurrently.
//
// ctx_for_scale(sf, nl) is the calling thread's context for other pyramid settings (created
// on first use per (sf, nl), kept until thread exit); default_ctx() is ctx_for_scale(1.2, 8).
inline orbg_ctx *ctx_for_scale(float scale_factor, int nlevels)
{
    struct Holder {
        float sf;
        int nl;
        orbg_ctx *c = nullptr;
        Holder(float sf_, int nl_) : sf(sf_), nl(nl_)
        {
            orbg_params p;
            orbg_params_default(&p);
            p.scale_factor = sf;
            p.nlevels = nl;
            check(orbg_create(0, &p, &c), "orbg_create");
        }
        ~Holder() { orbg_destroy(c); }
        Holder(const Holder &) = delete;
        Holder &operator=(const Holder &) = delete;
    };
    static thread_local std::list<Holder> held;  // list: a context's address never moves
    for (const Holder &h : held)
        if (h.sf == scale_factor && h.nl == nlevels) return h.c;
    held.emplace_back(scale_factor, nlevels);
    return held.back().c;
}

inline orbg_ctx *default_ctx() { return ctx_for_scale(1.2f, 8); }

// The calling thread's context for a Frame's / KeyFrame's own pyramid (mfScaleFactor,
// mnScaleLevels): the matchers size their search radii from the frame's mvScaleFactors
// (ORBmatcher.cc:86,117,1570,1724), which the context's scale tables restate.
template <class FrameT>
inline orbg_ctx *ctx_for(const FrameT &F)
{
    return ctx_for_scale(F.mfScaleFactor, F.mnScaleLevels);
}

// cv::KeyPoint -> orbg_keypoint (field by field, the ABI's layout is its own)
template <class KP>
inline orbg_keypoint to_orbg(const KP &k)
{
    orbg_keypoint o;
    o.x = k.pt.x;
    o.y = k.pt.y;
    o.size = k.size;
    o.angle = k.angle;
    o.response = k.response;
    o.octave = k.octave;
    o.class_id = k.class_id;
    return o;
}

template <class KPV>
inline std::vector<orbg_keypoint> keys_of(const KPV &v)
{
    std::vector<orbg_keypoint> out(v.size());
    for (size_t i = 0; i < v.size(); i++) out[i] = to_orbg(v[i]);
    return out;
}

// N x 32 CV_8U descriptor matrix (any row step) -> contiguous rows
template <class Mat>
inline std::vector<uint8_t> rows32(const Mat &m, int n)
{
    std::vector<uint8_t> out((size_t)n * 32);
    for (int i = 0; i < n; i++) std::memcpy(&out[(size_t)i * 32], m.template ptr<uint8_t>(i), 32);
    return out;
}

// Frame::mnMinX .. mnMaxY (static members of the reference's Frame)
template <class FrameT>
inline orbg_bounds bounds_of(const FrameT &)
{
    return orbg_bounds{FrameT::mnMinX, FrameT::mnMaxX, FrameT::mnMinY, FrameT::mnMaxY};
}

// rows 0..2 of a 4x4 CV_32F pose (Frame::mTcw, KeyFrame::GetPose())
template <class Mat>
inline void pose12(const Mat &T, float out[12])
{
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 4; c++) out[4 * r + c] = T.template at<float>(r, c);
}

inline int DescriptorDistance(const uint8_t *a, const uint8_t *b)
{
    return orbg_descriptor_distance(a, b);
}

// ORBmatcher(nnratio, checkOri).SearchForInitialization(F1, F2, vbPrevMatched,
// vnMatches12, windowSize): vbPrevMatched is updated for the matched keypoints of F1 and
// vnMatches12 resized to F1's keypoints, as the reference does.
template <class FrameT, class Point2fT>
int SearchForInitialization(orbg_ctx *ctx, float nnratio, bool checkOri, FrameT &F1, FrameT &F2,
                            std::vector<Point2fT> &vbPrevMatched, std::vector<int> &vnMatches12,
                            int windowSize = 10)
{
    const int n1 = (int)F1.mvKeysUn.size(), n2 = (int)F2.mvKeysUn.size();
    const std::vector<orbg_keypoint> k1 = keys_of(F1.mvKeysUn), k2 = keys_of(F2.mvKeysUn);
    const std::vector<uint8_t> d1 = rows32(F1.mDescriptors, n1), d2 = rows32(F2.mDescriptors, n2);
    std::vector<float> prev((size_t)2 * n1);
    for (int i = 0; i < n1; i++) {
        prev[2 * i] = vbPrevMatched[i].x;
        prev[2 * i + 1] = vbPrevMatched[i].y;
    }
    const orbg_bounds b = bounds_of(F2);
    std::vector<int32_t> m12(n1 > 0 ? n1 : 1);
    int nm = 0;
    check(orbg_search_for_initialization(ctx, k1.data(), d1.data(), n1, k2.data(), d2.data(), n2,
                                         &b, prev.data(), m12.data(), windowSize, nnratio,
                                         checkOri ? 1 : 0, &nm),
          "orbg_search_for_initialization");
    vnMatches12.assign(m12.begin(), m12.begin() + n1);
    for (int i = 0; i < n1; i++) {
        vbPrevMatched[i].x = prev[2 * i];
        vbPrevMatched[i].y = prev[2 * i + 1];
    }
    return nm;
}

// mvpMapPoints[i] && mvpMapPoints[i]->Observations() > 0, the "taken" test both
// SearchByProjection loops apply to the current frame's slots on entry
template <class FrameT>
inline std::vector<uint8_t> taken_of(const FrameT &F)
{
    std::vector<uint8_t> t(F.mvpMapPoints.size());
    for (size_t i = 0; i < t.size(); i++)
        t[i] = F.mvpMapPoints[i] && F.mvpMapPoints[i]->Observations() > 0;
    return t;
}

template <class MapPointT>
inline void mp_desc(const MapPointT *pMP, uint8_t out[32])
{
    std::memcpy(out, pMP->GetDescriptor().template ptr<uint8_t>(0), 32);
}

// ORBmatcher(nnratio, checkOri).SearchByProjection(CurrentFrame, LastFrame, th, bMono)
// (Tracking::TrackWithMotionModel): writes CurrentFrame.mvpMapPoints.
template <class FrameT>
int SearchByProjection(orbg_ctx *ctx, bool checkOri, FrameT &CurrentFrame, const FrameT &LastFrame,
                       float th, bool bMono)
{
    const int n = (int)CurrentFrame.mvKeysUn.size(), np = (int)LastFrame.mvpMapPoints.size();
    const std::vector<orbg_keypoint> k = keys_of(CurrentFrame.mvKeysUn);
    const std::vector<uint8_t> d = rows32(CurrentFrame.mDescriptors, n);
    const std::vector<uint8_t> taken = taken_of(CurrentFrame);
    std::vector<orbg_lastframe_point> pts(np > 0 ? np : 1);
    std::vector<uint8_t> pdesc((size_t)(np > 0 ? np : 1) * 32, 0);
    for (int i = 0; i < np; i++) {
        orbg_lastframe_point &p = pts[i];
        std::memset(&p, 0, sizeof(p));
        const auto *pMP = LastFrame.mvpMapPoints[i];
        p.octave = LastFrame.mvKeys[i].octave;
        p.angle = LastFrame.mvKeysUn[i].angle;
        if (!pMP) continue;
        const auto X = pMP->GetWorldPos();
        p.x = X.template at<float>(0);
        p.y = X.template at<float>(1);
        p.z = X.template at<float>(2);
        p.flags = (!LastFrame.mvbOutlier[i] ? ORBG_MP_VALID : 0) |
                  (pMP->Observations() > 0 ? ORBG_MP_HAS_OBS : 0);
        mp_desc(pMP, &pdesc[(size_t)i * 32]);
    }
    orbg_track_camera cam;
    std::memset(&cam, 0, sizeof(cam));
    pose12(CurrentFrame.mTcw, cam.Tcw);
    pose12(LastFrame.mTcw, cam.Tlw);
    cam.fx = FrameT::fx;
    cam.fy = FrameT::fy;
    cam.cx = FrameT::cx;
    cam.cy = FrameT::cy;
    cam.bf = CurrentFrame.mbf;
    cam.b = CurrentFrame.mb;
    cam.mono = bMono ? 1 : 0;
    const orbg_bounds b = bounds_of(CurrentFrame);
    std::vector<int32_t> match(n > 0 ? n : 1);
    int nm = 0;
    check(orbg_search_by_projection_lastframe(ctx, k.data(), d.data(), CurrentFrame.mvuRight.data(),
                                              n, taken.data(), &b, pts.data(), pdesc.data(), np,
                                              &cam, th, checkOri ? 1 : 0, match.data(), &nm),
          "orbg_search_by_projection_lastframe");
    for (int i = 0; i < n; i++) {
        if (match[i] >= 0)
            CurrentFrame.mvpMapPoints[i] = LastFrame.mvpMapPoints[match[i]];
        else if (match[i] == -2)
            CurrentFrame.mvpMapPoints[i] = nullptr;  // rotation-consistency filter
    }
    return nm;
}

// ORBmatcher(nnratio).SearchByProjection(F, vpMapPoints, th) (Tracking::SearchLocalPoints;
// the projections come from Frame::isInFrustum's mTrackProj* fields): writes
// F.mvpMapPoints.
template <class FrameT, class MapPointT>
int SearchByProjection(orbg_ctx *ctx, float nnratio, FrameT &F,
                       const std::vector<MapPointT *> &vpMapPoints, float th = 3)
{
    const int n = (int)F.mvKeysUn.size(), nm_in = (int)vpMapPoints.size();
    const std::vector<orbg_keypoint> k = keys_of(F.mvKeysUn);
    const std::vector<uint8_t> d = rows32(F.mDescriptors, n);
    const std::vector<uint8_t> taken = taken_of(F);
    std::vector<orbg_map_projection> mps(nm_in > 0 ? nm_in : 1);
    std::vector<uint8_t> mdesc((size_t)(nm_in > 0 ? nm_in : 1) * 32, 0);
    for (int j = 0; j < nm_in; j++) {
        const MapPointT *pMP = vpMapPoints[j];
        orbg_map_projection &m = mps[j];
        std::memset(&m, 0, sizeof(m));
        if (!pMP) continue;
        m.u = pMP->mTrackProjX;
        m.v = pMP->mTrackProjY;
        m.ur = pMP->mTrackProjXR;
        m.level = pMP->mnTrackScaleLevel;
        m.view_cos = pMP->mTrackViewCos;
        m.flags = (pMP->mbTrackInView && !pMP->isBad() ? ORBG_MP_VALID : 0) |
                  (pMP->Observations() > 0 ? ORBG_MP_HAS_OBS : 0);
        if (m.flags & ORBG_MP_VALID) mp_desc(pMP, &mdesc[(size_t)j * 32]);
    }
    const orbg_bounds b = bounds_of(F);
    std::vector<int32_t> match(n > 0 ? n : 1);
    int nm = 0;
    check(orbg_search_by_projection_local(ctx, k.data(), d.data(), F.mvuRight.data(), n,
                                          taken.data(), &b, mps.data(), mdesc.data(), nm_in, th,
                                          nnratio, match.data(), &nm),
          "orbg_search_by_projection_local");
    for (int i = 0; i < n; i++)
        if (match[i] >= 0) F.mvpMapPoints[i] = vpMapPoints[match[i]];
    return nm;
}

// ORBmatcher(0.75, checkOri).SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th,
// ORBdist) (Tracking::Relocalization): pKF's map points projected into CurrentFrame with its
// pose; writes CurrentFrame.mvpMapPoints (a slot NULL on entry only: the reference skips any
// non-NULL one).
template <class FrameT, class KeyFrameT, class MapPointT>
int SearchByProjection(orbg_ctx *ctx, bool checkOri, FrameT &CurrentFrame, KeyFrameT *pKF,
                       const std::set<MapPointT *> &sAlreadyFound, const float th,
                       const int ORBdist)
{
    const int n = (int)CurrentFrame.mvKeysUn.size();
    const std::vector<orbg_keypoint> k = keys_of(CurrentFrame.mvKeysUn);
    const std::vector<uint8_t> d = rows32(CurrentFrame.mDescriptors, n);
    std::vector<uint8_t> taken(n > 0 ? n : 1, 0);
    for (int i = 0; i < n; i++) taken[i] = CurrentFrame.mvpMapPoints[i] != nullptr;
    const std::vector<MapPointT *> vpMPs = pKF->GetMapPointMatches();
    const int np = (int)vpMPs.size();
    std::vector<orbg_reloc_point> pts(np > 0 ? np : 1);
    std::vector<uint8_t> pdesc((size_t)(np > 0 ? np : 1) * 32, 0);
    for (int i = 0; i < np; i++) {
        orbg_reloc_point &p = pts[i];
        std::memset(&p, 0, sizeof(p));
        MapPointT *pMP = vpMPs[i];
        if (!pMP || pMP->isBad() || sAlreadyFound.count(pMP)) continue;
        const auto X = pMP->GetWorldPos();
        p.x = X.template at<float>(0);
        p.y = X.template at<float>(1);
        p.z = X.template at<float>(2);
        p.min_dist = pMP->GetMinDistance();
        p.max_dist = pMP->GetMaxDistance();
        p.angle = pKF->mvKeysUn[i].angle;
        p.flags = ORBG_MP_VALID;
        mp_desc(pMP, &pdesc[(size_t)i * 32]);
    }
    orbg_frustum_camera cam;
    std::memset(&cam, 0, sizeof(cam));
    pose12(CurrentFrame.mTcw, cam.Tcw);
    cam.fx = FrameT::fx;
    cam.fy = FrameT::fy;
    cam.cx = FrameT::cx;
    cam.cy = FrameT::cy;
    cam.bf = CurrentFrame.mbf;
    cam.log_scale_factor = CurrentFrame.mfLogScaleFactor;
    cam.nlevels = CurrentFrame.mnScaleLevels;
    cam.bounds = bounds_of(CurrentFrame);
    std::vector<int32_t> match(n > 0 ? n : 1);
    int nm = 0;
    check(orbg_search_by_projection_reloc(ctx, k.data(), d.data(), n, taken.data(), &cam,
                                          pts.data(), pdesc.data(), np, th, ORBdist,
                                          checkOri ? 1 : 0, match.data(), &nm),
          "orbg_search_by_projection_reloc");
    for (int i = 0; i < n; i++)  // -2: written, then set to NULL by the rotation filter
        if (match[i] >= 0) CurrentFrame.mvpMapPoints[i] = vpMPs[match[i]];
    return nm;
}

// ORBmatcher::SearchByProjection(pKF, Scw, vpPoints, vpMatched, th) (LoopClosing::
// ComputeSim3): writes vpMatched (the Scw decomposition happens on the device).  FrameT gives
// the Frame's float bounds the KeyFrame's grid was built with.
template <class FrameT, class KeyFrameT, class MapPointT, class Mat>
int SearchByProjection(orbg_ctx *ctx, KeyFrameT *pKF, const Mat &Scw,
                       const std::vector<MapPointT *> &vpPoints,
                       std::vector<MapPointT *> &vpMatched, int th)
{
    const int n = (int)pKF->mvKeysUn.size(), nm_in = (int)vpPoints.size();
    const std::vector<orbg_keypoint> k = keys_of(pKF->mvKeysUn);
    const std::vector<uint8_t> d = rows32(pKF->mDescriptors, n);
    std::set<MapPointT *> spAlreadyFound(vpMatched.begin(), vpMatched.end());
    spAlreadyFound.erase(static_cast<MapPointT *>(nullptr));
    std::vector<uint8_t> taken(n > 0 ? n : 1, 0);
    for (int i = 0; i < n; i++) taken[i] = vpMatched[i] != nullptr;
    std::vector<orbg_map_point> mps(nm_in > 0 ? nm_in : 1);
    std::vector<uint8_t> mdesc((size_t)(nm_in > 0 ? nm_in : 1) * 32, 0);
    for (int i = 0; i < nm_in; i++) {
        MapPointT *p = vpPoints[i];
        orbg_map_point &m = mps[i];
        std::memset(&m, 0, sizeof(m));
        if (p->isBad() || spAlreadyFound.count(p)) continue;
        const auto X = p->GetWorldPos(), Pn = p->GetNormal();
        m.x = X.template at<float>(0);
        m.y = X.template at<float>(1);
        m.z = X.template at<float>(2);
        m.nx = Pn.template at<float>(0);
        m.ny = Pn.template at<float>(1);
        m.nz = Pn.template at<float>(2);
        m.min_dist = p->GetMinDistance();
        m.max_dist = p->GetMaxDistance();
        m.flags = ORBG_MP_VALID;
        mp_desc(p, &mdesc[(size_t)i * 32]);
    }
    orbg_frustum_camera cam;
    std::memset(&cam, 0, sizeof(cam));
    pose12(Scw, cam.Tcw);
    cam.fx = pKF->fx;
    cam.fy = pKF->fy;
    cam.cx = pKF->cx;
    cam.cy = pKF->cy;
    cam.log_scale_factor = pKF->mfLogScaleFactor;
    cam.nlevels = pKF->mnScaleLevels;
    cam.bounds = orbg_bounds{FrameT::mnMinX, FrameT::mnMaxX, FrameT::mnMinY, FrameT::mnMaxY};
    std::vector<int32_t> match(n > 0 ? n : 1);
    int nm = 0;
    check(orbg_search_by_projection_sim3(ctx, k.data(), d.data(), n, taken.data(), &cam,
                                         mps.data(), mdesc.data(), nm_in, th, match.data(), &nm),
          "orbg_search_by_projection_sim3");
    for (int i = 0; i < n; i++)
        if (match[i] >= 0) vpMatched[i] = vpPoints[match[i]];
    return nm;
}

// DBoW2::FeatureVector (std::map<NodeId, std::vector<unsigned int>>, ascending ids and
// indices) -> the ABI's CSR arrays (nodes, off[nodes + 1], feats)
template <class FeatVecT>
inline void flatten_fv(const FeatVecT &fv, std::vector<int32_t> &nodes, std::vector<int32_t> &off,
                       std::vector<int32_t> &feats)
{
    nodes.clear();
    feats.clear();
    off.assign(1, 0);
    for (const auto &e : fv) {
        nodes.push_back((int32_t)e.first);
        for (auto f : e.second) feats.push_back((int32_t)f);
        off.push_back((int32_t)feats.size());
    }
}

// ORBmatcher(nnratio, checkOri).SearchByBoW(pKF, F, vpMapPointMatches)
// (Tracking::TrackReferenceKeyFrame Tracking.cc:1069, Relocalization :2009): both frames'
// mFeatVec after ComputeBoW; vpMapPointMatches = F.N entries, the KeyFrame's MapPoint per
// matched Frame feature or NULL (ORBmatcher.cc:197, 276).
template <class KeyFrameT, class FrameT, class MapPointT>
int SearchByBoW(orbg_ctx *ctx, float nnratio, bool checkOri, KeyFrameT *pKF, FrameT &F,
                std::vector<MapPointT *> &vpMapPointMatches)
{
    const std::vector<MapPointT *> vpMPs = pKF->GetMapPointMatches();
    const int nk = (int)pKF->mvKeysUn.size(), nf = F.N;
    std::vector<uint8_t> valid(nk > 0 ? nk : 1, 0);
    std::vector<float> ak(nk > 0 ? nk : 1), af(nf > 0 ? nf : 1);
    for (int i = 0; i < nk; i++) {
        valid[i] = vpMPs[i] && !vpMPs[i]->isBad();
        ak[i] = pKF->mvKeysUn[i].angle;
    }
    for (int i = 0; i < nf; i++) af[i] = F.mvKeys[i].angle;
    std::vector<int32_t> kn, ko, kf, fn, fo, ff;
    flatten_fv(pKF->mFeatVec, kn, ko, kf);
    flatten_fv(F.mFeatVec, fn, fo, ff);
    const std::vector<uint8_t> kd = rows32(pKF->mDescriptors, nk), fd = rows32(F.mDescriptors, nf);
    std::vector<int32_t> match(nf > 0 ? nf : 1);
    int nm = 0;
    check(orbg_search_by_bow(ctx, kd.data(), ak.data(), valid.data(), nk, kn.data(), ko.data(),
                             kf.data(), (int)kn.size(), fd.data(), af.data(), nf, fn.data(),
                             fo.data(), ff.data(), (int)fn.size(), nnratio, checkOri ? 1 : 0,
                             match.data(), &nm),
          "orbg_search_by_bow");
    vpMapPointMatches.assign(nf, static_cast<MapPointT *>(nullptr));
    for (int i = 0; i < nf; i++)
        if (match[i] >= 0) vpMapPointMatches[i] = vpMPs[match[i]];
    return nm;
}

// ORBmatcher(nnratio, checkOri).SearchByBoW(pKF1, pKF2, vpMatches12) (LoopClosing::
// ComputeSim3, LoopClosing.cc:485): vpMatches12 = pKF1's N entries, pKF2's MapPoint per
// matched pKF1 feature or NULL.
template <class KeyFrameT, class MapPointT>
int SearchByBoW(orbg_ctx *ctx, float nnratio, bool checkOri, KeyFrameT *pKF1, KeyFrameT *pKF2,
                std::vector<MapPointT *> &vpMatches12)
{
    const std::vector<MapPointT *> vp1 = pKF1->GetMapPointMatches(), vp2 = pKF2->GetMapPointMatches();
    const int n1 = (int)pKF1->mvKeysUn.size(), n2 = (int)pKF2->mvKeysUn.size();
    std::vector<uint8_t> v1(n1 > 0 ? n1 : 1, 0), v2(n2 > 0 ? n2 : 1, 0);
    std::vector<float> a1(n1 > 0 ? n1 : 1), a2(n2 > 0 ? n2 : 1);
    for (int i = 0; i < n1; i++) {
        v1[i] = vp1[i] && !vp1[i]->isBad();
        a1[i] = pKF1->mvKeysUn[i].angle;
    }
    for (int i = 0; i < n2; i++) {
        v2[i] = vp2[i] && !vp2[i]->isBad();
        a2[i] = pKF2->mvKeysUn[i].angle;
    }
    std::vector<int32_t> n1v, o1, f1, n2v, o2, f2;
    flatten_fv(pKF1->mFeatVec, n1v, o1, f1);
    flatten_fv(pKF2->mFeatVec, n2v, o2, f2);
    const std::vector<uint8_t> d1 = rows32(pKF1->mDescriptors, n1), d2 = rows32(pKF2->mDescriptors, n2);
    std::vector<int32_t> m12(n1 > 0 ? n1 : 1);
    int nm = 0;
    check(orbg_search_by_bow_kf(ctx, d1.data(), a1.data(), v1.data(), n1, n1v.data(), o1.data(),
                                f1.data(), (int)n1v.size(), d2.data(), a2.data(), v2.data(), n2,
                                n2v.data(), o2.data(), f2.data(), (int)n2v.size(), nnratio,
                                checkOri ? 1 : 0, m12.data(), &nm),
          "orbg_search_by_bow_kf");
    vpMatches12.assign(n1, static_cast<MapPointT *>(nullptr));
    for (int i = 0; i < n1; i++)
        if (m12[i] >= 0) vpMatches12[i] = vp2[m12[i]];
    return nm;
}

// Optimizer::PoseOptimization(pFrame): one edge per keypoint with a MapPoint (index order),
// stereo when mvuRight[i] >= 0 (Optimizer.cc:381-460); writes pFrame->SetPose(Tcw) and
// pFrame->mvbOutlier, returns nInitialCorrespondences - nBad.
template <class FrameT>
int PoseOptimization(orbg_ctx *ctx, FrameT *pFrame)
{
    typedef typename std::decay<decltype(pFrame->mTcw)>::type MatT;
    const int N = (int)pFrame->mvpMapPoints.size();
    std::vector<orbg_pose_edge> edges;
    std::vector<int> idx;
    edges.reserve(N);
    for (int i = 0; i < N; i++) {
        const auto *pMP = pFrame->mvpMapPoints[i];
        if (!pMP) continue;
        pFrame->mvbOutlier[i] = false;
        const auto &kpUn = pFrame->mvKeysUn[i];
        const auto X = pMP->GetWorldPos();
        orbg_pose_edge e;
        e.obs[0] = kpUn.pt.x;
        e.obs[1] = kpUn.pt.y;
        e.obs[2] = pFrame->mvuRight[i];
        e.xw[0] = X.template at<float>(0);
        e.xw[1] = X.template at<float>(1);
        e.xw[2] = X.template at<float>(2);
        e.inv_sigma2 = pFrame->mvInvLevelSigma2[kpUn.octave];
        e.stereo = pFrame->mvuRight[i] >= 0 ? 1 : 0;
        edges.push_back(e);
        idx.push_back(i);
    }
    orbg_pose_camera cam{FrameT::fx, FrameT::fy, FrameT::cx, FrameT::cy, pFrame->mbf, 0.f};
    float tcw[12], tout[12];
    pose12(pFrame->mTcw, tcw);
    double q[4], t[3];
    std::vector<uint8_t> outl(edges.size() + 1);
    int ninl = 0;
    check(orbg_pose_optimization(ctx, edges.data(), (int)edges.size(), &cam, tcw, q, t, tout,
                                 outl.data(), &ninl),
          "orbg_pose_optimization");
    if ((int)edges.size() < 3) return 0;  // Optimizer.cc:463-464: pose untouched
    MatT pose = MatT::eye(4, 4, 5 /* CV_32F */);
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 4; c++) pose.template at<float>(r, c) = tout[4 * r + c];
    pFrame->SetPose(pose);
    for (size_t k = 0; k < idx.size(); k++) pFrame->mvbOutlier[idx[k]] = outl[k] != 0;
    return ninl;
}

// ---------------------------------------------------------------------------------------
// Local bundle adjustment
// ---------------------------------------------------------------------------------------

// Converter::toSE3Quat (Converter.cc:47-60): SE3Quat(Matrix3d R, Vector3d t), i.e. Eigen's
// Quaterniond(R) (trace branch, else the largest diagonal) then normalizeRotation
// (se3quat.h:280-285).  Host arithmetic, the same as oracle/pose_oracle.c's pin.
inline orbg_pose se3quat_of(const float T[12], int fixed)
{
    double R[3][3], q[4];
    orbg_pose p;
    std::memset(&p, 0, sizeof(p));
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) R[i][j] = T[4 * i + j];
        p.t[i] = T[4 * i + 3];
    }
    const double tr = R[0][0] + R[1][1] + R[2][2];
    if (tr > 0) {
        double s = std::sqrt(tr + 1.0);
        q[3] = 0.5 * s;
        s = 0.5 / s;
        q[0] = (R[2][1] - R[1][2]) * s;
        q[1] = (R[0][2] - R[2][0]) * s;
        q[2] = (R[1][0] - R[0][1]) * s;
    } else {
        int i = 0;
        if (R[1][1] > R[0][0]) i = 1;
        if (R[2][2] > R[i][i]) i = 2;
        const int j = (i + 1) % 3, k = (j + 1) % 3;
        double s = std::sqrt(R[i][i] - R[j][j] - R[k][k] + 1.0);
        q[i] = 0.5 * s;
        s = 0.5 / s;
        q[3] = (R[k][j] - R[j][k]) * s;
        q[j] = (R[j][i] + R[i][j]) * s;
        q[k] = (R[k][i] + R[i][k]) * s;
    }
    if (q[3] < 0)
        for (double &v : q) v = -v;
    const double nq = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    for (int c = 0; c < 4; c++) p.q[c] = q[c] / nq;
    p.fixed = fixed;
    return p;
}

// The vertices and edges Optimizer::LocalBundleAdjustment puts into g2o (Optimizer.cc:
// 662-851) as liborbg's SoA: poses = lLocalKeyFrames (fixed iff mnId == 0) then
// lFixedCameras (fixed); points = lLocalMapPoints (xyz); one edge per observation of a local
// map point by a local or fixed key frame that is not bad, in the map point's observation
// order (std::map<KeyFrame*, size_t>), mono when mvuRight < 0 (Huber delta (float)sqrt(5.991))
// else stereo ((float)sqrt(7.815)), information = mvInvLevelSigma2[octave].  (The reference
// adds an edge for every observing key frame that is not bad, Optimizer.cc:783-848; its
// lFixedCameras hold all of them, :672-686, so the "in the window" test never drops one there.)
template <class KeyFrameT, class MapPointT>
struct LbaWindow {
    std::vector<orbg_pose> poses;
    std::vector<double> points;  // 3 per point
    std::vector<orbg_edge> edges;
    std::vector<KeyFrameT *> kfs;   // pose index -> key frame
    std::vector<MapPointT *> mps;   // point index -> map point
    std::vector<size_t> edge_obs;   // edge -> keypoint index in its key frame
};

template <class KeyFrameT, class MapPointT>
LbaWindow<KeyFrameT, MapPointT> build_lba_window(const std::list<KeyFrameT *> &lLocalKeyFrames,
                                                 const std::list<KeyFrameT *> &lFixedCameras,
                                                 const std::list<MapPointT *> &lLocalMapPoints)
{
    LbaWindow<KeyFrameT, MapPointT> w;
    std::map<const KeyFrameT *, int> pose_of;
    auto add_kf = [&](KeyFrameT *pKF, int fixed) {
        float T[12];
        pose12(pKF->GetPose(), T);
        pose_of[pKF] = (int)w.poses.size();
        w.poses.push_back(se3quat_of(T, fixed));
        w.kfs.push_back(pKF);
    };
    for (KeyFrameT *pKFi : lLocalKeyFrames) add_kf(pKFi, pKFi->mnId == 0 ? 1 : 0);
    for (KeyFrameT *pKFi : lFixedCameras) add_kf(pKFi, 1);
    // float in the reference (Optimizer.cc:758-759), then RobustKernelHuber::setDelta(double)
    const float thHuberMono = std::sqrt(5.991), thHuberStereo = std::sqrt(7.815);
    for (MapPointT *pMP : lLocalMapPoints) {
        const int pt = (int)w.mps.size();
        const auto X = pMP->GetWorldPos();
        for (int c = 0; c < 3; c++) w.points.push_back(X.template at<float>(c));
        w.mps.push_back(pMP);
        const auto observations = pMP->GetObservations();
        for (const auto &obs : observations) {
            KeyFrameT *pKFi = obs.first;
            if (pKFi->isBad()) continue;
            auto it = pose_of.find(pKFi);
            if (it == pose_of.end()) continue;
            const size_t k = obs.second;
            const auto &kpUn = pKFi->mvKeysUn[k];
            orbg_edge e;
            std::memset(&e, 0, sizeof(e));
            e.point = pt;
            e.pose = it->second;
            e.stereo = pKFi->mvuRight[k] < 0 ? 0 : 1;
            e.robust = 1;
            e.active = 1;
            e.obs[0] = kpUn.pt.x;
            e.obs[1] = kpUn.pt.y;
            e.obs[2] = e.stereo ? pKFi->mvuRight[k] : 0.0;
            e.inv_sigma2 = pKFi->mvInvLevelSigma2[kpUn.octave];
            e.fx = pKFi->fx;
            e.fy = pKFi->fy;
            e.cx = pKFi->cx;
            e.cy = pKFi->cy;
            e.bf = pKFi->mbf;
            e.huber_delta = e.stereo ? thHuberStereo : thHuberMono;
            w.edges.push_back(e);
            w.edge_obs.push_back(k);
        }
    }
    return w;
}

// BlockSolver<6,3>::buildSystem's layout (block_solver.hpp:502-560).  g2o numbers the
// hessian blocks in vertex-id order (SparseOptimizer::buildIndexMapping sorts the active
// vertices by id): key frames are vertex mnId, map points mnId + maxKFid + 1, so the free
// poses come first by KeyFrame::mnId, then the points by MapPoint::mnId.  Blocks are Eigen's
// column-major 6x6 / 3x3 / 6x3; b = [b_pose (6 each) | b_point (3 each)] in hessian order
// with g2o's sign (b -= J^T Omega e).  Hpl holds one 6x3 block per (pose, point) hessian
// pair with an active edge, the sum of its edges' J_pose^T W J_point.  active_robust_chi2
// is SparseOptimizer::activeRobustChi2 after computeActiveErrors (sparse_optimizer.cpp:
// 100-112).
struct G2oBlockSystem {
    std::vector<int> pose_hidx;          // pose -> hessian index, -1 for fixed poses
    std::vector<int> point_hidx;         // point -> hessian index (counted from the points)
    std::vector<double> Hpp;             // [free pose][36] column-major, hessian order
    std::vector<double> Hll;             // [point][9] column-major, hessian order
    std::map<std::pair<int, int>, std::vector<double>> Hpl;  // (pose hidx, point hidx) -> 18
    std::vector<double> b;               // 6 * free poses + 3 * points
    double active_robust_chi2 = 0;
};

template <class Window>
G2oBlockSystem linearize_lba_window(orbg_ctx *ctx, const Window &w)
{
    const int np = (int)w.poses.size(), nx = (int)(w.points.size() / 3);
    BASystem s = linearize_local_ba(ctx, w.poses, w.points, w.edges);
    G2oBlockSystem g;
    g.pose_hidx.assign(np, -1);
    g.point_hidx.assign(nx, -1);
    {
        std::vector<std::pair<decltype(w.kfs[0]->mnId), int>> ids;
        for (int i = 0; i < np; i++)
            if (!w.poses[i].fixed) ids.emplace_back(w.kfs[i]->mnId, i);
        std::sort(ids.begin(), ids.end());
        for (size_t k = 0; k < ids.size(); k++) g.pose_hidx[ids[k].second] = (int)k;
    }
    {
        std::vector<std::pair<decltype(w.mps[0]->mnId), int>> ids;
        for (int j = 0; j < nx; j++) ids.emplace_back(w.mps[j]->mnId, j);
        std::sort(ids.begin(), ids.end());
        for (size_t k = 0; k < ids.size(); k++) g.point_hidx[ids[k].second] = (int)k;
    }
    int nfree = 0;
    for (int i = 0; i < np; i++) nfree += g.pose_hidx[i] >= 0;
    g.Hpp.assign((size_t)nfree * 36, 0.0);
    g.Hll.assign((size_t)nx * 9, 0.0);
    g.b.assign((size_t)6 * nfree + 3 * nx, 0.0);
    for (int i = 0; i < np; i++) {
        const int h = g.pose_hidx[i];
        if (h < 0) continue;
        for (int r = 0; r < 6; r++) {
            for (int c = 0; c < 6; c++)
                g.Hpp[(size_t)h * 36 + c * 6 + r] = s.hpose[(size_t)i * 36 + r * 6 + c];
            g.b[(size_t)6 * h + r] = s.bpose[(size_t)i * 6 + r];
        }
    }
    for (int j = 0; j < nx; j++) {
        const int h = g.point_hidx[j];
        for (int r = 0; r < 3; r++) {
            for (int c = 0; c < 3; c++)
                g.Hll[(size_t)h * 9 + c * 3 + r] = s.hpoint[(size_t)j * 9 + r * 3 + c];
            g.b[(size_t)6 * nfree + 3 * h + r] = s.bpoint[(size_t)j * 3 + r];
        }
    }
    for (size_t e = 0; e < w.edges.size(); e++) {
        const orbg_edge &E = w.edges[e];
        if (!E.active) continue;
        const orbg_edge_out &o = s.edges[e];
        // RobustKernelHuber::robustify (robust_kernel_impl.cpp:78-91); dsqr is a float
        // member there, so delta^2 is rounded to float
        if (E.robust) {
            const double dsqr = (float)(E.huber_delta * E.huber_delta);
            g.active_robust_chi2 +=
                o.chi2 <= dsqr ? o.chi2 : 2 * std::sqrt(o.chi2) * E.huber_delta - dsqr;
        } else {
            g.active_robust_chi2 += o.chi2;
        }
        const int h = g.pose_hidx[E.pose];
        if (h < 0) continue;
        std::vector<double> &blk = g.Hpl[std::make_pair(h, g.point_hidx[E.point])];
        if (blk.empty()) blk.assign(18, 0.0);
        for (int r = 0; r < 6; r++)  // (pose row r, point col c) = hpl[c][r]
            for (int c = 0; c < 3; c++) blk[c * 6 + r] += o.hpl[c][r];
    }
    return g;
}

// Converter::toCvMat(SE3Quat) (Converter.cc:49-53, 63-71): to_homogeneous_matrix (Eigen's
// QuaternionBase::toRotationMatrix, se3quat.h:270-278), every element cast to float -- the
// arithmetic of oracle/pose_oracle.c orc_se3_to_tcw
inline void tcw_of(const orbg_pose &p, float T[12])
{
    const double *q = p.q;
    const double tx = 2 * q[0], ty = 2 * q[1], tz = 2 * q[2];
    const double twx = tx * q[3], twy = ty * q[3], twz = tz * q[3];
    const double txx = tx * q[0], txy = ty * q[0], txz = tz * q[0];
    const double tyy = ty * q[1], tyz = tz * q[1], tzz = tz * q[2];
    const double R[3][3] = {{1 - (tyy + tzz), txy - twz, txz + twy},
                            {txy + twz, 1 - (txx + tzz), tyz - twx},
                            {txz - twy, tyz + twx, 1 - (txx + tyy)}};
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) T[4 * i + j] = (float)R[i][j];
        T[4 * i + 3] = (float)p.t[i];
    }
}

// Optimizer::LocalBundleAdjustment(pKF, pbStopFlag, pMap) (Optimizer.cc:633-979) with the
// optimisation on the device:
//   the local key frames (pKF + its not-bad covisible key frames, mnBALocalForKF), local map
//   points (mnBALocalForKF) and fixed cameras (mnBAFixedForKF) exactly as :635-683;
//   the window (build_lba_window, :687-851); the stop check (:853-855: return, nothing
//   written);
//   optimize(5), the outlier pass, optimize(10) and the vToErase test in one call
//   (orbg_local_ba_optimize: pbStopFlag polled where g2o polls terminate(), pMP->isBad()
//   asked where the reference asks it);
//   under pMap->mMutexMapUpdate: EraseMapPointMatch / EraseObservation of the erased
//   observations (mono edges first, then stereo, as vToErase is filled :909-937), the local
//   key frames' SetPose(Converter::toCvMat(SE3quat)) and the local map points' SetWorldPos +
//   UpdateNormalAndDepth (:939-978).
// hooks (tests: deterministic stops) are merged with pbStopFlag; report (may be NULL).
template <class KeyFrameT, class MapT>
void LocalBundleAdjustment(orbg_ctx *ctx, KeyFrameT *pKF, bool *pbStopFlag, MapT *pMap,
                           const orbg_lm_control *hooks = nullptr,
                           orbg_lba_report *report = nullptr)
{
    typedef typename std::remove_pointer<
        typename decltype(pKF->GetMapPointMatches())::value_type>::type MapPointT;
    typedef typename std::decay<decltype(pKF->GetPose())>::type MatT;
    std::list<KeyFrameT *> lLocalKeyFrames;
    lLocalKeyFrames.push_back(pKF);
    pKF->mnBALocalForKF = pKF->mnId;
    const std::vector<KeyFrameT *> vNeighKFs = pKF->GetVectorCovisibleKeyFrames();
    for (KeyFrameT *pKFi : vNeighKFs) {
        pKFi->mnBALocalForKF = pKF->mnId;
        if (!pKFi->isBad()) lLocalKeyFrames.push_back(pKFi);
    }
    std::list<MapPointT *> lLocalMapPoints;
    for (KeyFrameT *pKFi : lLocalKeyFrames) {
        const std::vector<MapPointT *> vpMPs = pKFi->GetMapPointMatches();
        for (MapPointT *pMP : vpMPs)
            if (pMP && !pMP->isBad() && pMP->mnBALocalForKF != pKF->mnId) {
                lLocalMapPoints.push_back(pMP);
                pMP->mnBALocalForKF = pKF->mnId;
            }
    }
    std::list<KeyFrameT *> lFixedCameras;
    for (MapPointT *pMP : lLocalMapPoints) {
        const auto observations = pMP->GetObservations();
        for (const auto &obs : observations) {
            KeyFrameT *pKFi = obs.first;
            if (pKFi->mnBALocalForKF != pKF->mnId && pKFi->mnBAFixedForKF != pKF->mnId) {
                pKFi->mnBAFixedForKF = pKF->mnId;
                if (!pKFi->isBad()) lFixedCameras.push_back(pKFi);
            }
        }
    }
    auto w = build_lba_window(lLocalKeyFrames, lFixedCameras, lLocalMapPoints);
    if (pbStopFlag && *pbStopFlag) return;
    orbg_lm_control K;
    std::memset(&K, 0, sizeof(K));
    if (hooks) K = *hooks;
    K.force_stop = reinterpret_cast<const volatile uint8_t *>(pbStopFlag);
    K.d_last_chi2 = nullptr;
    const size_t ne = w.edges.size();
    std::vector<uint8_t> erase(ne + 1, 0);
    struct Bad {
        static int point(void *u, int pt)
        {
            return (*static_cast<const std::vector<MapPointT *> *>(u))[pt]->isBad() ? 1 : 0;
        }
    };
    orbg_lba_report rep;
    check(orbg_local_ba_optimize(ctx, w.poses.data(), (int)w.poses.size(), w.points.data(),
                                 (int)(w.points.size() / 3), w.edges.data(), (int)ne, &K,
                                 &Bad::point, &w.mps, erase.data(), &rep),
          "orbg_local_ba_optimize");
    if (report) *report = rep;
    std::unique_lock<std::mutex> lock(pMap->mMutexMapUpdate);
    for (int pass = 0; pass < 2; pass++)  // vpEdgesMono, then vpEdgesStereo
        for (size_t e = 0; e < ne; e++) {
            if (w.edges[e].stereo != pass || !erase[e]) continue;
            KeyFrameT *pKFi = w.kfs[w.edges[e].pose];
            MapPointT *pMPi = w.mps[w.edges[e].point];
            pKFi->EraseMapPointMatch(pMPi);
            pMPi->EraseObservation(pKFi);
        }
    const size_t nlocal = lLocalKeyFrames.size();  // the window's first poses
    for (size_t i = 0; i < nlocal; i++) {
        float T[12];
        tcw_of(w.poses[i], T);
        MatT pose = MatT::eye(4, 4, 5 /* CV_32F */);
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 4; c++) pose.template at<float>(r, c) = T[4 * r + c];
        w.kfs[i]->SetPose(pose);
    }
    for (size_t j = 0; j < w.mps.size(); j++) {
        MatT X(3, 1, 5 /* CV_32F */);
        for (int c = 0; c < 3; c++) X.template at<float>(c) = (float)w.points[3 * j + c];
        w.mps[j]->SetWorldPos(X);
        w.mps[j]->UpdateNormalAndDepth();
    }
}

// ---------------------------------------------------------------------------
// Frame geometry
// ---------------------------------------------------------------------------
// Frame::mK (3x3 CV_32F) + mDistCoef (4x1 or 5x1 CV_32F) -> orbg_camera
template <class Mat>
inline orbg_camera camera_of(const Mat &K, const Mat &D)
{
    orbg_camera c;
    c.fx = K.template at<float>(0, 0);
    c.fy = K.template at<float>(1, 1);
    c.cx = K.template at<float>(0, 2);
    c.cy = K.template at<float>(1, 2);
    c.k1 = D.template at<float>(0);
    c.k2 = D.template at<float>(1);
    c.p1 = D.template at<float>(2);
    c.p2 = D.template at<float>(3);
    c.k3 = D.rows * D.cols > 4 ? D.template at<float>(4) : 0.f;
    return c;
}

// Frame::UndistortKeyPoints(): F.mvKeysUn from F.mvKeys (k1 == 0: a copy)
template <class FrameT>
void UndistortKeyPoints(orbg_ctx *ctx, FrameT &F)
{
    if (F.mDistCoef.template at<float>(0) == 0.0) {
        F.mvKeysUn = F.mvKeys;
        return;
    }
    const orbg_camera cam = camera_of(F.mK, F.mDistCoef);
    const int n = (int)F.mvKeys.size();
    std::vector<orbg_keypoint> k = keys_of(F.mvKeys), u(n > 0 ? n : 1);
    check(orbg_undistort_keypoints(ctx, &cam, k.data(), n, u.data()), "orbg_undistort_keypoints");
    F.mvKeysUn.resize(n);
    for (int i = 0; i < n; i++) {
        auto kp = F.mvKeys[i];
        kp.pt.x = u[i].x;
        kp.pt.y = u[i].y;
        F.mvKeysUn[i] = kp;
    }
}

// Frame::ComputeImageBounds(imLeft): the static mnMinX .. mnMaxY
template <class FrameT, class Mat>
void ComputeImageBounds(FrameT &F, const Mat &imLeft)
{
    const orbg_camera cam = camera_of(F.mK, F.mDistCoef);
    orbg_bounds b;
    check(orbg_compute_image_bounds(&cam, imLeft.cols, imLeft.rows, &b), "orbg_compute_image_bounds");
    FrameT::mnMinX = b.min_x;
    FrameT::mnMaxX = b.max_x;
    FrameT::mnMinY = b.min_y;
    FrameT::mnMaxY = b.max_y;
}

// The isInFrustum loop of Tracking::SearchLocalPoints (Tracking.cc:1676-1691) over
// Frame::isInFrustum(pMP, viewingCosLimit): the points not seen by this frame and not bad are
// tested; mbTrackInView / mTrack* are written as isInFrustum writes them (a point out of view
// gets mbTrackInView = false only) and IncreaseVisible() is called for those in view.  Returns
// nToMatch.  PredictScale needs MapPoint::mfMinDistance / mfMaxDistance (protected in
// MapPoint.h): the drop-in reads them through two getters a maintainer adds beside
// GetMinDistanceInvariance (GetMinDistance / GetMaxDistance).
template <class FrameT, class MapPointT>
int SearchLocalPointsInFrustum(orbg_ctx *ctx, FrameT &F, const std::vector<MapPointT *> &vpLocal,
                               float viewingCosLimit = 0.5f)
{
    const int n = (int)vpLocal.size();
    std::vector<orbg_map_point> mp(n > 0 ? n : 1);
    std::vector<orbg_map_projection> pr(n > 0 ? n : 1);
    for (int i = 0; i < n; i++) {
        MapPointT *p = vpLocal[i];
        orbg_map_point &m = mp[i];
        std::memset(&m, 0, sizeof(m));
        const bool test = p->mnLastFrameSeen != F.mnId && !p->isBad();
        if (test) {
            const auto X = p->GetWorldPos(), Pn = p->GetNormal();
            m.x = X.template at<float>(0);
            m.y = X.template at<float>(1);
            m.z = X.template at<float>(2);
            m.nx = Pn.template at<float>(0);
            m.ny = Pn.template at<float>(1);
            m.nz = Pn.template at<float>(2);
            m.min_dist = p->GetMinDistance();
            m.max_dist = p->GetMaxDistance();
            m.flags = ORBG_MP_VALID;
        }
        pr[i] = orbg_map_projection{p->mTrackProjX, p->mTrackProjY, p->mTrackProjXR,
                                    p->mnTrackScaleLevel, p->mTrackViewCos, 0};
    }
    orbg_frustum_camera fc;
    std::memset(&fc, 0, sizeof(fc));
    pose12(F.mTcw, fc.Tcw);
    fc.fx = FrameT::fx;
    fc.fy = FrameT::fy;
    fc.cx = FrameT::cx;
    fc.cy = FrameT::cy;
    fc.bf = F.mbf;
    fc.log_scale_factor = F.mfLogScaleFactor;
    fc.nlevels = F.mnScaleLevels;
    fc.bounds = bounds_of(F);
    int nvis = 0;
    check(orbg_is_in_frustum(ctx, &fc, mp.data(), n, viewingCosLimit, pr.data(), &nvis),
          "orbg_is_in_frustum");
    for (int i = 0; i < n; i++) {
        if (!(mp[i].flags & ORBG_MP_VALID)) continue;  // not tested: untouched
        MapPointT *p = vpLocal[i];
        p->mbTrackInView = (pr[i].flags & ORBG_MP_VALID) != 0;
        if (!p->mbTrackInView) continue;
        p->mTrackProjX = pr[i].u;
        p->mTrackProjY = pr[i].v;
        p->mTrackProjXR = pr[i].ur;
        p->mnTrackScaleLevel = pr[i].level;
        p->mTrackViewCos = pr[i].view_cos;
        p->IncreaseVisible();
    }
    return nvis;
}

// ---------------------------------------------------------------------------
// LocalMapping matchers
// ---------------------------------------------------------------------------
template <class KeyFrameT>
struct KfArrays {  // one KeyFrame flattened for orbg_keyframe (kept alive by the caller)
    std::vector<orbg_keypoint> k;
    std::vector<uint8_t> d, mp;
    std::vector<float> ur;
    std::vector<int32_t> nodes, off, feats;
    orbg_keyframe view(bool with_fv) const
    {
        orbg_keyframe v;
        v.kps = k.data();
        v.desc = d.data();
        v.uright = ur.data();
        v.has_mp = mp.data();
        v.n = (int32_t)k.size();
        v.fv_nodes = with_fv ? nodes.data() : nullptr;
        v.fv_off = with_fv ? off.data() : nullptr;
        v.fv_feats = with_fv ? feats.data() : nullptr;
        v.nfv = with_fv ? (int32_t)nodes.size() : 0;
        return v;
    }
};

template <class KeyFrameT>
KfArrays<KeyFrameT> kf_arrays(KeyFrameT *pKF, bool with_fv)
{
    KfArrays<KeyFrameT> a;
    const int n = (int)pKF->mvKeysUn.size();
    a.k = keys_of(pKF->mvKeysUn);
    a.d = rows32(pKF->mDescriptors, n);
    a.ur.assign(pKF->mvuRight.begin(), pKF->mvuRight.end());
    a.mp.resize(n);
    for (int i = 0; i < n; i++) a.mp[i] = pKF->GetMapPoint((size_t)i) != nullptr;
    if (with_fv) flatten_fv(pKF->mFeatVec, a.nodes, a.off, a.feats);
    return a;
}

// ORBmatcher(nnratio, checkOri).SearchForTriangulation(pKF1, pKF2, F12, vMatchedPairs,
// bOnlyStereo) (LocalMapping::CreateNewMapPoints): both mFeatVec after ComputeBoW.
template <class KeyFrameT, class Mat>
int SearchForTriangulation(orbg_ctx *ctx, bool checkOri, KeyFrameT *pKF1, KeyFrameT *pKF2,
                           const Mat &F12, std::vector<std::pair<size_t, size_t>> &vMatchedPairs,
                           const bool bOnlyStereo)
{
    const KfArrays<KeyFrameT> a1 = kf_arrays(pKF1, true), a2 = kf_arrays(pKF2, true);
    const orbg_keyframe k1 = a1.view(true), k2 = a2.view(true);
    orbg_triangulation_pair g;
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) g.F12[3 * r + c] = F12.template at<float>(r, c);
    const auto Cw = pKF1->GetCameraCenter(), R2w = pKF2->GetRotation(), t2w = pKF2->GetTranslation();
    for (int r = 0; r < 3; r++) {
        g.Cw1[r] = Cw.template at<float>(r);
        for (int c = 0; c < 3; c++) g.Tcw2[4 * r + c] = R2w.template at<float>(r, c);
        g.Tcw2[4 * r + 3] = t2w.template at<float>(r);
    }
    g.fx2 = pKF2->fx;
    g.fy2 = pKF2->fy;
    g.cx2 = pKF2->cx;
    g.cy2 = pKF2->cy;
    std::vector<int32_t> m12(k1.n > 0 ? k1.n : 1);
    int n = 0;
    check(orbg_search_for_triangulation(ctx, &k1, &k2, &g, bOnlyStereo ? 1 : 0, checkOri ? 1 : 0,
                                        m12.data(), &n),
          "orbg_search_for_triangulation");
    vMatchedPairs.clear();
    vMatchedPairs.reserve(n);
    for (int i = 0; i < k1.n; i++)
        if (m12[i] >= 0) vMatchedPairs.push_back(std::make_pair((size_t)i, (size_t)m12[i]));
    return n;
}

// ORBmatcher::Fuse(pKF, vpMapPoints, th) (LocalMapping::SearchInNeighbors): the per-point
// search on the device, then the reference's map update in vpMapPoints order, each point
// re-checked as the reference's loop checks it at that moment (ORBmatcher.cc:986-987) -- an
// earlier Replace can make a later point bad or put it in pKF.  Returns nFused.  FrameT gives
// the Frame's static (float) image bounds the KeyFrame's grid was built with (KeyFrame.cc:
// 35-67 copies mGrid and mfGridElementWidthInv; its int mnMinX .. are their truncation).
template <class FrameT, class KeyFrameT, class MapPointT>
int Fuse(orbg_ctx *ctx, KeyFrameT *pKF, const std::vector<MapPointT *> &vpMapPoints,
         const float th = 3.0f)
{
    const int n = (int)vpMapPoints.size();
    const KfArrays<KeyFrameT> a = kf_arrays(pKF, false);
    const orbg_keyframe kf = a.view(false);
    std::vector<orbg_map_point> mp(n > 0 ? n : 1);
    std::vector<uint8_t> md((size_t)(n > 0 ? n : 1) * 32, 0);
    for (int i = 0; i < n; i++) {
        MapPointT *p = vpMapPoints[i];
        orbg_map_point &m = mp[i];
        std::memset(&m, 0, sizeof(m));
        if (!p || p->isBad() || p->IsInKeyFrame(pKF)) continue;
        const auto X = p->GetWorldPos(), Pn = p->GetNormal();
        m.x = X.template at<float>(0);
        m.y = X.template at<float>(1);
        m.z = X.template at<float>(2);
        m.nx = Pn.template at<float>(0);
        m.ny = Pn.template at<float>(1);
        m.nz = Pn.template at<float>(2);
        m.min_dist = p->GetMinDistance();
        m.max_dist = p->GetMaxDistance();
        m.flags = ORBG_MP_VALID;
        mp_desc(p, &md[(size_t)i * 32]);
    }
    orbg_frustum_camera fc;
    std::memset(&fc, 0, sizeof(fc));
    const auto R = pKF->GetRotation(), t = pKF->GetTranslation();
    for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) fc.Tcw[4 * r + c] = R.template at<float>(r, c);
        fc.Tcw[4 * r + 3] = t.template at<float>(r);
    }
    fc.fx = pKF->fx;
    fc.fy = pKF->fy;
    fc.cx = pKF->cx;
    fc.cy = pKF->cy;
    fc.bf = pKF->mbf;
    fc.log_scale_factor = pKF->mfLogScaleFactor;
    fc.nlevels = pKF->mnScaleLevels;
    fc.bounds = orbg_bounds{FrameT::mnMinX, FrameT::mnMaxX, FrameT::mnMinY, FrameT::mnMaxY};
    std::vector<int32_t> best(n > 0 ? n : 1), dist(n > 0 ? n : 1);
    int ncand = 0;
    check(orbg_fuse(ctx, &kf, &fc, mp.data(), md.data(), n, th, best.data(), dist.data(), &ncand),
          "orbg_fuse");
    int nFused = 0;
    for (int i = 0; i < n; i++) {
        MapPointT *pMP = vpMapPoints[i];
        if (best[i] < 0 || !pMP || pMP->isBad() || pMP->IsInKeyFrame(pKF)) continue;
        MapPointT *pMPinKF = pKF->GetMapPoint((size_t)best[i]);
        if (pMPinKF) {
            if (!pMPinKF->isBad()) {
                if (pMPinKF->Observations() > pMP->Observations())
                    pMP->Replace(pMPinKF);
                else
                    pMPinKF->Replace(pMP);
            }
        } else {
            pMP->AddObservation(pKF, (size_t)best[i]);
            pKF->AddMapPoint(pMP, (size_t)best[i]);
        }
        nFused++;
    }
    return nFused;
}

// ORBmatcher::Fuse(pKF, Scw, vpPoints, th, vpReplacePoint) (LoopClosing::SearchAndFuse,
// th 4): the search on the device (Scw decomposed there as the reference does), then the
// reference's loop in vpPoints order (ORBmatcher.cc:1239-1254): a KeyFrame MapPoint at the
// best feature, if not bad, goes to vpReplacePoint[i], else pMP is added.  The skip test
// (isBad, already in pKF->GetMapPoints() when the call starts) cannot change inside the loop
// (AddObservation / AddMapPoint make nothing bad and spAlreadyFound is a snapshot), so it is
// taken once.  Returns nFused.
template <class FrameT, class KeyFrameT, class MapPointT, class Mat>
int Fuse(orbg_ctx *ctx, KeyFrameT *pKF, const Mat &Scw, const std::vector<MapPointT *> &vpPoints,
         float th, std::vector<MapPointT *> &vpReplacePoint)
{
    const int n = (int)vpPoints.size();
    const KfArrays<KeyFrameT> a = kf_arrays(pKF, false);
    const orbg_keyframe kf = a.view(false);
    const auto spAlreadyFound = pKF->GetMapPoints();
    std::vector<orbg_map_point> mp(n > 0 ? n : 1);
    std::vector<uint8_t> md((size_t)(n > 0 ? n : 1) * 32, 0);
    for (int i = 0; i < n; i++) {
        MapPointT *p = vpPoints[i];
        orbg_map_point &m = mp[i];
        std::memset(&m, 0, sizeof(m));
        if (p->isBad() || spAlreadyFound.count(p)) continue;
        const auto X = p->GetWorldPos(), Pn = p->GetNormal();
        m.x = X.template at<float>(0);
        m.y = X.template at<float>(1);
        m.z = X.template at<float>(2);
        m.nx = Pn.template at<float>(0);
        m.ny = Pn.template at<float>(1);
        m.nz = Pn.template at<float>(2);
        m.min_dist = p->GetMinDistance();
        m.max_dist = p->GetMaxDistance();
        m.flags = ORBG_MP_VALID;
        mp_desc(p, &md[(size_t)i * 32]);
    }
    orbg_frustum_camera fc;
    std::memset(&fc, 0, sizeof(fc));
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 4; c++) fc.Tcw[4 * r + c] = Scw.template at<float>(r, c);
    fc.fx = pKF->fx;
    fc.fy = pKF->fy;
    fc.cx = pKF->cx;
    fc.cy = pKF->cy;
    fc.log_scale_factor = pKF->mfLogScaleFactor;
    fc.nlevels = pKF->mnScaleLevels;
    fc.bounds = orbg_bounds{FrameT::mnMinX, FrameT::mnMaxX, FrameT::mnMinY, FrameT::mnMaxY};
    std::vector<int32_t> best(n > 0 ? n : 1), dist(n > 0 ? n : 1);
    int ncand = 0;
    check(orbg_fuse_sim3(ctx, &kf, &fc, mp.data(), md.data(), n, th, best.data(), dist.data(),
                         &ncand),
          "orbg_fuse_sim3");
    int nFused = 0;
    for (int i = 0; i < n; i++) {
        if (best[i] < 0) continue;
        MapPointT *pMP = vpPoints[i];
        MapPointT *pMPinKF = pKF->GetMapPoint((size_t)best[i]);
        if (pMPinKF) {
            if (!pMPinKF->isBad()) vpReplacePoint[i] = pMPinKF;
        } else {
            pMP->AddObservation(pKF, (size_t)best[i]);
            pKF->AddMapPoint(pMP, (size_t)best[i]);
        }
        nFused++;
    }
    return nFused;
}

// ORBmatcher::SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th) (LoopClosing::
// ComputeSim3): writes vpMatches12 where both projection directions agree.  FrameT gives the
// Frame's float bounds.
template <class FrameT, class KeyFrameT, class MapPointT, class Mat>
int SearchBySim3(orbg_ctx *ctx, KeyFrameT *pKF1, KeyFrameT *pKF2,
                 std::vector<MapPointT *> &vpMatches12, const float &s12, const Mat &R12,
                 const Mat &t12, const float th)
{
    const std::vector<MapPointT *> vp1 = pKF1->GetMapPointMatches(), vp2 = pKF2->GetMapPointMatches();
    const int n1 = (int)vp1.size(), n2 = (int)vp2.size();
    auto side = [](const std::vector<MapPointT *> &vp, std::vector<orbg_map_point> &mp,
                   std::vector<uint8_t> &md) {
        const int n = (int)vp.size();
        mp.assign(n > 0 ? n : 1, orbg_map_point{});
        md.assign((size_t)(n > 0 ? n : 1) * 32, 0);
        for (int i = 0; i < n; i++) {
            MapPointT *p = vp[i];
            if (!p || p->isBad()) continue;
            const auto X = p->GetWorldPos();
            orbg_map_point &m = mp[i];
            m.x = X.template at<float>(0);
            m.y = X.template at<float>(1);
            m.z = X.template at<float>(2);
            m.min_dist = p->GetMinDistance();
            m.max_dist = p->GetMaxDistance();
            m.flags = ORBG_MP_VALID;
            mp_desc(p, &md[(size_t)i * 32]);
        }
    };
    std::vector<orbg_map_point> mp1, mp2;
    std::vector<uint8_t> md1, md2;
    side(vp1, mp1, md1);
    side(vp2, mp2, md2);
    std::vector<uint8_t> am1(n1 > 0 ? n1 : 1, 0), am2(n2 > 0 ? n2 : 1, 0);
    for (int i = 0; i < n1; i++) {  // vbAlreadyMatched1 / 2 (ORBmatcher.cc:1288-1297)
        MapPointT *pMP = vpMatches12[i];
        if (!pMP) continue;
        am1[i] = 1;
        const int idx2 = pMP->GetIndexInKeyFrame(pKF2);
        if (idx2 >= 0 && idx2 < n2) am2[idx2] = 1;
    }
    orbg_sim3_pair g;
    std::memset(&g, 0, sizeof(g));
    pose12(pKF1->GetPose(), g.T1w);
    pose12(pKF2->GetPose(), g.T2w);
    for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) g.R12[3 * r + c] = R12.template at<float>(r, c);
        g.t12[r] = t12.template at<float>(r);
    }
    g.s12 = s12;
    g.fx = pKF1->fx;
    g.fy = pKF1->fy;
    g.cx = pKF1->cx;
    g.cy = pKF1->cy;
    g.log_scale_factor = pKF1->mfLogScaleFactor;
    g.nlevels = pKF1->mnScaleLevels;
    g.bounds = orbg_bounds{FrameT::mnMinX, FrameT::mnMaxX, FrameT::mnMinY, FrameT::mnMaxY};
    const KfArrays<KeyFrameT> a1 = kf_arrays(pKF1, false), a2 = kf_arrays(pKF2, false);
    const orbg_keyframe k1 = a1.view(false), k2 = a2.view(false);
    std::vector<int32_t> m12(n1 > 0 ? n1 : 1);
    int nFound = 0;
    check(orbg_search_by_sim3(ctx, &k1, mp1.data(), md1.data(), am1.data(), &k2, mp2.data(),
                              md2.data(), am2.data(), &g, th, m12.data(), &nFound),
          "orbg_search_by_sim3");
    for (int i = 0; i < n1; i++)
        if (m12[i] >= 0) vpMatches12[i] = vp2[m12[i]];
    return nFound;
}

// Frame::ComputeStereoFromRGBD(imDepth) (Frame.cc:837-858) on the depth image as
// Tracking::GrabImageRGBD receives it (CV_16U raw or CV_32F): the convertTo(CV_32F,
// mDepthMapFactor) of Tracking.cc:233-234 happens in liborbg, at the keypoints' pixels.
template <class FrameT, class Mat>
void ComputeStereoFromRGBD(orbg_ctx *ctx, FrameT &F, const Mat &imDepthRaw, float mDepthMapFactor)
{
    const int n = (int)F.mvKeys.size();
    F.mvuRight.assign(n, -1.f);
    F.mvDepth.assign(n, -1.f);
    if (n == 0) return;
    const std::vector<orbg_keypoint> k = keys_of(F.mvKeys), ku = keys_of(F.mvKeysUn);
    check(orbg_rgbd_stereo(ctx, imDepthRaw.data,
                           imDepthRaw.type() == CV_32F ? ORBG_DEPTH_F32 : ORBG_DEPTH_U16,
                           mDepthMapFactor, imDepthRaw.cols, imDepthRaw.rows, imDepthRaw.step[0],
                           k.data(), ku.data(), n, F.mbf, F.mvuRight.data(), F.mvDepth.data()),
          "orbg_rgbd_stereo");
}

// MapPoint::ComputeDistinctiveDescriptors(): BestIdx over the observations' descriptor rows
// vDescriptors (1 x 32 CV_8U each, in the mObservations order with bad KeyFrames left out);
// the caller sets mDescriptor = vDescriptors[BestIdx].clone() (-1: none, the reference returns)
template <class Mat>
int DistinctiveDescriptorIndex(orbg_ctx *ctx, const std::vector<Mat> &vDescriptors)
{
    const int n = (int)vDescriptors.size();
    std::vector<uint8_t> d((size_t)(n > 0 ? n : 1) * 32);
    for (int i = 0; i < n; i++) std::memcpy(&d[(size_t)i * 32], vDescriptors[i].template ptr<uint8_t>(0), 32);
    int32_t best = -1;
    check(orbg_distinctive_descriptor(ctx, d.data(), n, &best), "orbg_distinctive_descriptor");
    return best;
}

}  // namespace ref
}  // namespace orbg_compat
