/*
 * oracle/orb_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C CPU restatement of the ORB-SLAM2 per-frame hot path, used as the
 * parity CHECKER by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg.  It is never linked into, loaded by, or called from the
 * product library (liborbg.so); the product fails loudly without its HIP code.
 *
 * What it restates (reference = /root/reference, read as text only):
 *   ORBextractor ctor tables ........ src/ORBextractor.cc:432-521
 *   ComputePyramid .................. src/ORBextractor.cc:1400-1443 (+ cv::resize pin)
 *   ComputeKeyPointsOctTree (FAST) .. src/ORBextractor.cc:966-1128  (+ cv::FAST pin)
 *   DistributeOctTree / DivideNode .. src/ORBextractor.cc:668-951, 537-614
 *   IC_Angle / computeOrientation ... src/ORBextractor.cc:83-111, 523-530 (+ fastAtan2 pin)
 *   GaussianBlur + computeOrbDesc ... src/ORBextractor.cc:1366-1396, 117-157, 1310-1317
 *   ORBmatcher::DescriptorDistance .. src/ORBmatcher.cc:1846-1862
 *   ORBmatcher::SearchForInit ....... src/ORBmatcher.cc:487-631, 1800-1841
 *   Frame grid / GetFeaturesInArea .. src/Frame.cc:292-307, 421-520
 *   Frame::ComputeStereoMatches ..... src/Frame.cc:619-834 (stereo_oracle.c)
 *   ORBmatcher::SearchByProjection .. src/ORBmatcher.cc:1503-1667, 59-154 (track_oracle.c)
 *   Optimizer::PoseOptimization ..... src/Optimizer.cc:356-631 + g2o LM / LDLT (pose_oracle.c)
 *   DBoW2 transform (Frame::ComputeBoW) Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h (bow_oracle.c)
 *   g2o edge arithmetic (double) .... Thirdparty/g2o/g2o/types/types_six_dof_expmap.{h,cpp},
 *                                     core/base_binary_edge.hpp:55-120, core/base_edge.h:58-102,
 *                                     core/robust_kernel_impl.cpp:65-91
 *
 * Parity pinning status (see DESIGN.md "Oracle"):
 *   - PINNED by the reference text: the rBRIEF pattern, umax, per-level feature
 *     counts / level sizes, matcher constants (tests/golden/ref_tables.json), and
 *     g2o's own central-difference Jacobian (base_binary_edge.hpp:131-205).
 *   - UNPINNED: whole keypoint/descriptor outputs.  The reference ships no tests,
 *     fixtures or golden vectors, and cannot be compiled here (it needs OpenCV,
 *     Eigen and Pangolin, none present).  The OpenCV primitives it calls are
 *     restated from OpenCV 3.4 semantics and are switchable (ORC_RESIZE_*, Gaussian
 *     weights) -- "parity unpinned" for those outputs.
 */
#ifndef ORB_ORACLE_H
#define ORB_ORACLE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_MAX_LEVELS 16

/* cv::KeyPoint field order (pt.x, pt.y, size, angle, response, octave, class_id): 28 bytes */
typedef struct {
    float x, y, size, angle, response;
    int32_t octave, class_id;
} orc_keypoint;

/* cv::resize INTER_LINEAR 8UC1 vertical-pass variants (see orb_oracle.c, orc_resize_linear_u8) */
enum {
    ORC_RESIZE_SCALAR = 0,     /* FixedPtCast<int,uchar,22> everywhere                   */
    ORC_RESIZE_SSE2_16_4 = 4,  /* OpenCV 2.4-3.3 SSE2 VResizeLinearVec_32s8u (16 then 4)  */
    ORC_RESIZE_SIMD_16_8 = 8   /* OpenCV 3.4 universal intrinsics (16 then 8)  [default] */
};

typedef struct {
    /* ctor arguments, ORBextractor.h:64-65 */
    int32_t nfeatures;
    float scale_factor;
    int32_t nlevels;
    int32_t ini_th_fast;
    int32_t min_th_fast;
    /* derived tables, ORBextractor.cc:437-476 */
    float scale[ORC_MAX_LEVELS];
    float inv_scale[ORC_MAX_LEVELS];
    float sigma2[ORC_MAX_LEVELS];
    float inv_sigma2[ORC_MAX_LEVELS];
    int32_t features_per_level[ORC_MAX_LEVELS];
    int32_t umax[16];
    /* OpenCV-primitive pins */
    int32_t resize_mode;       /* ORC_RESIZE_* */
    int32_t gauss_k[7];        /* 7-tap weights (sum 256 for the bit-exact 3.4.9+ table) */
    int32_t brief_fma;         /* 0: x*b + y*a rounded twice (default); 1: fused */
    int32_t sincos_mode;       /* ORC_SINCOS_*: the cosf/sinf of ORBextractor.cc:122 */
} orc_params;

/* cos/sin of the rBRIEF rotation (ORBextractor.cc:121-122: (float)cos(float), i.e. glibc's
 * cosf/sinf).  GLIBC restates glibc 2.35's flt-32 sinf/cosf (sysdeps/ieee754/flt-32/
 * s_sinf.c, s_cosf.c, sincosf.h, its __sincosf_table) and equals the host libm for every
 * float in [0, 7) (tools/sincosf_sweep.c); HOST calls the machine's libm (validation only);
 * PINNED is round 1's double Cody-Waite + Taylor evaluation. */
enum { ORC_SINCOS_GLIBC = 0, ORC_SINCOS_PINNED = 1, ORC_SINCOS_HOST = 2 };
float orc_glibc_sinf(float y);
float orc_glibc_cosf(float y);
/* mismatches of orc_glibc_sinf/cosf against the linked libm over every `stride`-th float bit
 * pattern in [lo, hi) */
long orc_sincosf_check(uint32_t lo, uint32_t hi, uint32_t stride);

/* ---- extractor ---- */
int orc_init_params(orc_params *p, int nfeatures, float scale_factor, int nlevels,
                    int ini_th_fast, int min_th_fast);
void orc_level_size(const orc_params *p, int w, int h, int level, int *lw, int *lh);

void orc_resize_linear_u8(const uint8_t *src, int sw, int sh, int sstep,
                          uint8_t *dst, int dw, int dh, int dstep, int mode);
void orc_gauss7_u8(const uint8_t *src, int w, int h, int sstep, uint8_t *dst, int dstep,
                   const int32_t k[7]);
int orc_fast_score(const uint8_t *p, int step);              /* cornerScore<16> + corner test */
int orc_fast_window(const uint8_t *img, int step, int w, int h, int th,
                    orc_keypoint *out, int cap);             /* cv::FAST(roi, kps, th, true) */
int orc_distribute_octree(const orc_keypoint *keys, int n, int minX, int maxX, int minY,
                          int maxY, int N, orc_keypoint *out, int cap);
float orc_fast_atan2(float y, float x);
float orc_ic_angle(const uint8_t *img, int step, float px, float py, const int32_t umax[16]);
void orc_pinned_sincos_deg(float angle_deg, float *c, float *s);
/* a = cos, b = sin of angle_deg * factorPI (ORBextractor.cc:120-122) by sincos_mode */
void orc_brief_sincos_deg(float angle_deg, int sincos_mode, float *a, float *b);
void orc_orb_descriptor(const orc_keypoint *kp, const uint8_t *img, int step, int brief_fma,
                        int sincos_mode, uint8_t desc[32]);

/* Full ORBextractor::operator() for one 8-bit image.
 * Returns the number of keypoints (>=0) or a negative error.  kps/desc may be NULL
 * to query the count.  If level_counts != NULL it receives per-level counts.
 * If pyr != NULL it must hold sum_l(lw*lh) bytes; receives the levels packed (pitch = lw).
 * If cand_counts != NULL it receives per-level FAST candidate counts. */
int orc_extract(const orc_params *p, const uint8_t *img, int w, int h, int step,
                orc_keypoint *kps, uint8_t *desc, int cap, int32_t *level_counts,
                uint8_t *pyr, int32_t *cand_counts);
/* Per-level candidate list (vToDistributeKeys, coordinates relative to minBorder) */
int orc_level_candidates(const orc_params *p, const uint8_t *lvl, int lw, int lh, int step,
                         int level, orc_keypoint *out, int cap);
/* Batch of frames on nthreads pthreads (cpu baseline); returns total keypoints */
long orc_extract_batch(const orc_params *p, const uint8_t *imgs, int nframes, int w, int h,
                       int nthreads, int32_t *counts_out);

/* frames = extract(t) + knn2(t, t-1) + SearchForInitialization(t-1 -> t); pthreads */
int orc_frames_batch(const orc_params *p, const uint8_t *imgs, int nframes, int w, int h,
                     int nthreads, int window, float nnratio, int32_t *nkp, int32_t *nmatch);
/* orc_frames_batch with every output kept: frame f's keypoints / descriptors at
 * f * cap_out (nkp[f] of them), its knn2 triples {best idx, best, second} over frame f-1
 * (cyclic) at (f * cap_out + i) * 3, and vnMatches12 of the pair (f-1, f) over frame f-1's
 * keypoints at f * cap_out (nkp[f-1] of them).  Any output pointer may be NULL. */
int orc_frames_full(const orc_params *p, const uint8_t *imgs, int nframes, int w, int h,
                    int nthreads, int window, float nnratio, int32_t *nkp, int32_t *nmatch,
                    int cap_out, orc_keypoint *kps_out, uint8_t *desc_out, int32_t *knn_out,
                    int32_t *m12_out);

/* ---- matcher ---- */
int orc_descriptor_distance(const uint8_t *a, const uint8_t *b);
void orc_knn2(const uint8_t *qdesc, int nq, const uint8_t *tdesc, int nt, int32_t *best_idx,
              int32_t *best_dist, int32_t *second_dist);

typedef struct {
    float min_x, max_x, min_y, max_y;   /* Frame::mnMinX.. (ComputeImageBounds) */
} orc_bounds;

/* ORBmatcher(nnratio, checkOri).SearchForInitialization(F1, F2, prev, matches12, window).
 * kps1/kps2 are mvKeysUn (x, y, angle, octave used).  prev_xy (2*n1 floats) is updated
 * in place.  Returns nmatches. */
int orc_search_for_initialization(const orc_keypoint *kps1, const uint8_t *desc1, int n1,
                                  const orc_keypoint *kps2, const uint8_t *desc2, int n2,
                                  const orc_bounds *b2, float *prev_xy, int32_t *matches12,
                                  int window, float nnratio, int check_ori);

/* ---- tracking matchers (track_oracle.c) ---- */
#define ORC_MP_VALID 1    /* lastframe: pMP && !mvbOutlier[i]; local: mbTrackInView && !isBad() */
#define ORC_MP_HAS_OBS 2  /* pMP->Observations() > 0 */

/* LastFrame.mvpMapPoints[i] as SearchByProjection(CurrentFrame, LastFrame) reads it */
typedef struct {
    float x, y, z;      /* pMP->GetWorldPos() */
    int32_t octave;     /* LastFrame.mvKeys[i].octave */
    float angle;        /* LastFrame.mvKeysUn[i].angle */
    int32_t flags;
} orc_lf_point;

/* a local map point after Frame::isInFrustum (MapPoint mTrack* members) */
typedef struct {
    float u, v, ur;     /* mTrackProjX, mTrackProjY, mTrackProjXR */
    int32_t level;      /* mnTrackScaleLevel */
    float view_cos;     /* mTrackViewCos */
    int32_t flags;
} orc_map_proj;

/* CurrentFrame / LastFrame camera state: 3x4 row-major mTcw, intrinsics, mbf, mb */
typedef struct {
    float Tcw[12], Tlw[12];
    float fx, fy, cx, cy, bf, b;
    int32_t mono, pad;
} orc_track_cam;

/* cv::gemm small-matrix pin: out = (float)(alpha * op(R) x + c), double work type.  R is
 * the 3x3 block of a 3x4 row-major matrix. */
void orc_gemm3(const float *R, int transR, const float *x, float alpha, const float *c,
               float *out);
/* bForward / bBackward of ORBmatcher.cc:1521-1522 */
void orc_track_direction(const orc_track_cam *cam, int *forward, int *backward);
/* match[n]: CurrentFrame.mvpMapPoints as a LastFrame point index (-1 = not written, -2 =
 * NULLed by the rotation filter); taken0 (may
 * be NULL): initial mvpMapPoints[i] && Observations() > 0.  Returns nmatches. */
int orc_search_by_projection_lastframe(const orc_keypoint *kps, const uint8_t *desc,
                                       const float *uright, int n, const uint8_t *taken0,
                                       const orc_bounds *b, const float *scale_factors,
                                       const orc_lf_point *pts, const uint8_t *pdesc, int np,
                                       const orc_track_cam *cam, float th, int check_ori,
                                       int32_t *match);
/* match[n]: map point index written by this call (-1 = untouched).  Returns nmatches. */
int orc_search_by_projection_local(const orc_keypoint *kps, const uint8_t *desc,
                                   const float *uright, int n, const uint8_t *taken0,
                                   const orc_bounds *b, const float *scale_factors,
                                   const orc_map_proj *mps, const uint8_t *mdesc, int nm,
                                   float th, float nnratio, int32_t *match);

/* ---- Frame / MapPoint geometry (frame_oracle.c) ---- */
/* Frame::mK (fx, fy, cx, cy) and mDistCoef (k1, k2, p1, p2[, k3]; k3 = 0 when absent) */
typedef struct {
    float fx, fy, cx, cy;
    float k1, k2, p1, p2, k3;
} orc_camera;
/* cv::undistortPoints(xy, out, K, D, noArray(), K) over n (x, y) pairs */
void orc_undistort_points(const orc_camera *cam, const float *xy, int n, float *out);
/* Frame::UndistortKeyPoints: mvKeysUn (k1 == 0: a copy) */
void orc_undistort_keypoints(const orc_camera *cam, const orc_keypoint *kps, int n,
                             orc_keypoint *out);
/* Frame::ComputeImageBounds */
void orc_image_bounds(const orc_camera *cam, int w, int h, orc_bounds *b);
/* Frame::mfLogScaleFactor = log(mfScaleFactor) */
float orc_log_scale_factor(float scale_factor);
/* what Frame::isInFrustum reads of a MapPoint; flags: ORC_MP_VALID = SearchLocalPoints
 * tests it (!isBad() && mnLastFrameSeen != frame), ORC_MP_HAS_OBS passed through */
typedef struct {
    float x, y, z;            /* GetWorldPos() */
    float nx, ny, nz;         /* GetNormal() */
    float min_dist, max_dist; /* mfMinDistance, mfMaxDistance */
    int32_t flags;
} orc_map_point;
/* the Frame state isInFrustum reads: mTcw (3x4 row-major), fx.., mbf, mfLogScaleFactor,
 * mnScaleLevels, mnMinX.. */
typedef struct {
    float Tcw[12];
    float fx, fy, cx, cy, bf;
    float log_scale_factor;
    int32_t nlevels;
    orc_bounds bounds;
} orc_frustum_cam;
/* Frame::isInFrustum(pMP, viewingCosLimit): out = the mTrack* members + flags (VALID =
 * mbTrackInView); returns mbTrackInView */
int orc_is_in_frustum(const orc_frustum_cam *cam, const orc_map_point *mp,
                      float viewing_cos_limit, orc_map_proj *out);
/* MapPoint::ComputeDistinctiveDescriptors over n observation descriptors: BestIdx (-1 if n
 * is 0) */
int orc_distinctive_descriptor(const uint8_t *desc, int n);
/* loops over n points / npoints map points (observations pool[rows[off[p]..off[p+1])]) */
int orc_is_in_frustum_n(const orc_frustum_cam *cam, const orc_map_point *mps, int n,
                        float viewing_cos_limit, orc_map_proj *out);
void orc_distinctive_descriptors_n(const uint8_t *pool, const int32_t *rows, const int32_t *off,
                                   int npoints, int32_t *best);

/* ---- LocalMapping matchers (mapping_oracle.c) ---- */
/* one KeyFrame as SearchForTriangulation reads it */
typedef struct {
    const orc_keypoint *kps;  /* mvKeysUn (x, y, angle, octave) */
    const uint8_t *desc;      /* mDescriptors */
    const float *uright;      /* mvuRight (< 0: monocular) */
    const uint8_t *has_mp;    /* GetMapPoint(i) != NULL */
    int32_t n;
    const int32_t *fv_nodes, *fv_off, *fv_feats;  /* mFeatVec */
    int32_t nfv;
} orc_tri_kf;
/* F12 (row-major 3x3, LocalMapping::ComputeF12), pKF1->GetCameraCenter(), pKF2's pose rows
 * and intrinsics */
typedef struct {
    float F12[9];
    float Cw1[3];
    float Tcw2[12];
    float fx2, fy2, cx2, cy2;
} orc_tri_geom;
/* ORBmatcher(nnratio, checkOri).SearchForTriangulation: matches12[kf1->n] = vMatches12 (the
 * KF2 index matched to each KF1 feature, -1), returns nmatches.  scale_factors / sigma2 =
 * pKF2->mvScaleFactors / mvLevelSigma2. */
int orc_search_for_triangulation(const orc_tri_kf *kf1, const orc_tri_kf *kf2,
                                 const orc_tri_geom *g, const float *scale_factors,
                                 const float *sigma2, int only_stereo, int check_ori,
                                 int32_t *matches12);
void orc_three_maxima(const int *hsize, int *ind1, int *ind2, int *ind3);
/* LocalMapping::CreateNewMapPoints (src/LocalMapping.cc:293-560) and ComputeF12 (:690-707).
 * A KeyFrame's pose (Tcw rows 0..2) and calibration as they read it. */
typedef struct {
    float Tcw[12];
    float fx, fy, cx, cy, invfx, invfy, mb, mbf;
} orc_kf_cam;
/* the keypoint side: mvKeysUn, mvKeys (UnprojectStereo; NULL: mvKeysUn), mvuRight (NULL: all
 * monocular), mvDepth */
typedef struct {
    const orc_keypoint *kps;
    const orc_keypoint *kps_raw;
    const float *uright;
    const float *depth;
    int32_t n;
} orc_kf_tri;
/* per-match outcome: the reference's `continue`s in order */
enum {
    ORC_TRI_NONE = 0, ORC_TRI_NEW = 1, ORC_TRI_PARALLAX = -1, ORC_TRI_W0 = -2, ORC_TRI_Z1 = -3,
    ORC_TRI_Z2 = -4, ORC_TRI_REPROJ1 = -5, ORC_TRI_REPROJ2 = -6, ORC_TRI_DIST0 = -7,
    ORC_TRI_SCALE = -8
};
/* glibc's atan2f restated (fdlibm e_atan2f.c / s_atanf.c) */
float orc_atan2f(float y, float x);
long orc_atan2f_check(uint32_t seed, long n);
/* g = F12 = ComputeF12(pKF1, pKF2), pKF1->GetCameraCenter(), pKF2's Tcw and intrinsics */
void orc_tri_geometry(const orc_kf_cam *c1, const orc_kf_cam *c2, orc_tri_geom *g);
/* the null vector of a 4x4 float matrix (double Jacobi on A^T A), the cv::SVD stand-in */
void orc_tri_nullvec(const float *A, double *v);
/* the triangulation loop over matches12 (SearchForTriangulation's vMatchedPairs as vMatches12):
 * status[i] (ORC_TRI_*) and x3d[3i..3i+2] (the new MapPoint's position when NEW, else 0) for
 * i < k1->n; scale_factors / sigma2 = mvScaleFactors / mvLevelSigma2, scale_factor =
 * pKF1->mfScaleFactor.  Returns the new points. */
int orc_triangulate(const orc_kf_tri *k1, const orc_kf_tri *k2, const orc_kf_cam *c1,
                    const orc_kf_cam *c2, const int32_t *matches12, const float *scale_factors,
                    const float *sigma2, float scale_factor, float *x3d, int8_t *status);
/* ORBmatcher::Fuse(pKF, vpMapPoints, th)'s per-MapPoint search: kf = the KeyFrame's mvKeysUn,
 * mDescriptors, mvuRight (n; the FeatureVector is not read), cam = its pose, intrinsics,
 * mbf, mfLogScaleFactor, mnScaleLevels and bounds; mps[i] (flags ORC_MP_VALID: pMP &&
 * !isBad() && !IsInKeyFrame(pKF)) with descriptor mdesc[i]; best_idx[i] = the KeyFrame
 * feature the reference fuses the point with (bestDist <= TH_LOW), else -1; best_dist[i] =
 * bestDist (256 when none).  Returns the number of points with a fusion target. */
int orc_fuse_search(const orc_tri_kf *kf, const orc_frustum_cam *cam, const orc_map_point *mps,
                    const uint8_t *mdesc, int nmp, float th, const float *scale_factors,
                    const float *inv_sigma2, int32_t *best_idx, int32_t *best_dist);
/* ORBmatcher::Fuse(pKF, Scw, vpPoints, th, vpReplacePoint)'s search (ORBmatcher.cc:1133-1238):
 * cam->Tcw = Scw's rows 0..2, decomposed by orc_sim3_decompose; no reprojection gate. */
void orc_sim3_decompose(const float *Scw, float *Tcw);
int orc_fuse_sim3_search(const orc_tri_kf *kf, const orc_frustum_cam *cam,
                         const orc_map_point *mps, const uint8_t *mdesc, int nmp, float th,
                         const float *scale_factors, int32_t *best_idx, int32_t *best_dist);

/* loop_oracle.c.  ORBmatcher::SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th,
 * ORBdist) (ORBmatcher.cc:1670-1798): pts[i] = pKF->GetMapPointMatches()[i] (flags
 * ORC_MP_VALID = pMP && !isBad() && !sAlreadyFound.count(pMP)), angle = pKF->mvKeysUn[i].angle;
 * cam = CurrentFrame (mTcw, fx.., mfLogScaleFactor, mnScaleLevels, float bounds); taken0[i2]
 * = CurrentFrame.mvpMapPoints[i2] != NULL on entry.  match[i2] = the pKF index written to
 * mvpMapPoints[i2], -1, or -2 (NULLed by the rotation filter); returns nmatches. */
typedef struct {
    float x, y, z;            /* GetWorldPos() */
    float min_dist, max_dist; /* mfMinDistance, mfMaxDistance */
    float angle;              /* pKF->mvKeysUn[i].angle */
    int32_t flags;
} orc_reloc_point;
int orc_search_by_projection_reloc(const orc_keypoint *kps, const uint8_t *desc, int n,
                                   const uint8_t *taken0, const orc_frustum_cam *cam,
                                   const float *scale_factors, const orc_reloc_point *pts,
                                   const uint8_t *pdesc, int np, float th, int orb_dist,
                                   int check_ori, int32_t *match);
/* ORBmatcher::SearchByProjection(pKF, Scw, vpPoints, vpMatched, th) (ORBmatcher.cc:353-470):
 * kps / desc = pKF's mvKeysUn / mDescriptors, cam->Tcw = Scw rows 0..2 (decomposed as in
 * orc_fuse_sim3_search), cam->bounds the Frame's float bounds (the KeyFrame's int ones are
 * their truncation); mps[i] flags ORC_MP_VALID = !isBad() && not in vpMatched on entry;
 * taken0[idx] = vpMatched[idx] != NULL.  match[idx] = the vpPoints index written. */
int orc_search_by_projection_sim3(const orc_keypoint *kps, const uint8_t *desc, int n,
                                  const uint8_t *taken0, const orc_frustum_cam *cam,
                                  const float *scale_factors, const orc_map_point *mps,
                                  const uint8_t *mdesc, int nm, int th, int32_t *match);
/* Frame::ComputeStereoFromRGBD (frame_oracle.c) */
void orc_rgbd_stereo(const void *depth, int u16, float factor, int w, int h, size_t pitch,
                     const orc_keypoint *kps, const orc_keypoint *kps_un, int n, float mbf,
                     float *uright, float *depth_out);
/* ORBmatcher::SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th) (ORBmatcher.cc:
 * 1262-1470): mp1[i] = pKF1->GetMapPointMatches()[i] (ORC_MP_VALID = pMP && !isBad()),
 * matched1[i] = vpMatches12[i] != NULL, matched2[idx2] = 1 at those points' index in pKF2 (NULL:
 * none); g = poses, Sim3, pKF1's intrinsics, mfLogScaleFactor, mnScaleLevels, float bounds.
 * matches12[i] = the pKF2 index agreed both ways, -1; returns nFound. */
typedef struct {
    float T1w[12], T2w[12];
    float R12[9], t12[3], s12;
    float fx, fy, cx, cy;
    float log_scale_factor;
    int32_t nlevels;
    orc_bounds bounds;
} orc_sim3_pair;
int orc_search_by_sim3(const orc_keypoint *k1, const uint8_t *d1, int n1, const orc_map_point *mp1,
                       const uint8_t *md1, const uint8_t *matched1, const orc_keypoint *k2,
                       const uint8_t *d2, int n2, const orc_map_point *mp2, const uint8_t *md2,
                       const uint8_t *matched2, const orc_sim3_pair *g, float th,
                       const float *scale_factors, int32_t *matches12);

/* ---- Optimizer::PoseOptimization (pose_oracle.c) ---- */
/* LM's pow(2 rho - 1, 3) as the once-rounded exact cube (optimization_algorithm_levenberg.cpp:135) */
double orc_lm_cube(double t);
/* one EdgeSE3ProjectXYZOnlyPose (stereo = 0) / EdgeStereoSE3ProjectXYZOnlyPose (1) */
typedef struct {
    float obs[3];       /* kpUn.pt.x, kpUn.pt.y, mvuRight[i] */
    float xw[3];        /* pMP->GetWorldPos() */
    float inv_sigma2;   /* mvInvLevelSigma2[kpUn.octave] */
    int32_t stereo;     /* mvuRight[i] >= 0 */
} orc_pose_edge;

typedef struct {
    float fx, fy, cx, cy, bf;  /* Frame::fx .. mbf */
    float pad;
} orc_pose_cam;

/* edges: the frame's keypoints with a MapPoint, in index order.  Tcw_in: pFrame->mTcw
 * (3x4 row-major float).  Outputs: the optimised SE3Quat (q x,y,z,w; t), its cv::Mat form
 * (Converter::toCvMat) and mvbOutlier per edge.  Returns nInitialCorrespondences - nBad. */
int orc_pose_optimization(const orc_pose_edge *edges, int n, const orc_pose_cam *cam,
                          const float Tcw_in[12], double q_out[4], double t_out[3],
                          float Tcw_out[12], uint8_t *outlier);
void orc_se3_from_tcw(const float Tcw[12], double q[4], double t[3]);
int orc_match_pose(const orc_keypoint *k1, int n1, const orc_keypoint *k2, int n2,
                   const int32_t *m12, const orc_pose_cam *cam, float depth,
                   const float *inv_sigma2, double q[4], double t[3]);
void orc_se3_to_tcw(const double q[4], const double t[3], float Tcw[12]);
void orc_se3_oplus(double q[4], double t[3], const double upd[6]);
int orc_ldlt_solve6(const double H[6][6], const double b[6], double x[6]);

/* ---- DBoW2 TemplatedVocabulary::transform (bow_oracle.c) ---- */
enum { ORC_TF_IDF = 0, ORC_TF = 1, ORC_IDF = 2, ORC_BINARY = 3 };           /* WeightingType */
enum { ORC_L1_NORM = 0, ORC_L2_NORM = 1, ORC_DOT_PRODUCT = 5 };            /* ScoringType */
typedef struct {
    int32_t k, L, scoring, weighting, nnodes, nwords;
    const uint8_t *desc;        /* [nnodes][32] node descriptors */
    const double *weight;       /* [nnodes] idf weight (words) */
    const int32_t *word_id;     /* [nnodes] word id (leaves, file order); 0 otherwise (Node()) */
    const int32_t *child_off;   /* [nnodes + 1] children CSR */
    const int32_t *child_idx;
} orc_vocab;

void orc_bow_word(const orc_vocab *v, const uint8_t *feat, int levelsup, int32_t *word,
                  double *weight, int32_t *nid);
/* BowVector (ascending word ids + L1-normalised weights) and FeatureVector (ascending node
 * ids, CSR of feature indices).  Returns the number of features not stopped. */
int orc_bow_transform(const orc_vocab *v, const uint8_t *desc, int n, int levelsup,
                      int32_t *bow_words, double *bow_weights, int *nbow, int32_t *fv_nodes,
                      int32_t *fv_off, int32_t *fv_feats, int *nfv);
/* ORBmatcher::SearchByBoW(KeyFrame*, Frame&, ...) (ORBmatcher.cc:195-348), bow_oracle.c */
int orc_search_by_bow(const uint8_t *kf_desc, const float *kf_angle, const uint8_t *kf_valid,
                      int n_kf, const int32_t *kf_nodes, const int32_t *kf_off,
                      const int32_t *kf_feats, int kf_nfv, const uint8_t *f_desc,
                      const float *f_angle, int n_f, const int32_t *f_nodes, const int32_t *f_off,
                      const int32_t *f_feats, int f_nfv, float nnratio, int check_ori,
                      int32_t *match);
/* ORBmatcher::SearchByBoW(KeyFrame*, KeyFrame*, vpMatches12): match12[n1] = KF2 index or -1 */
int orc_search_by_bow_kf(const uint8_t *desc1, const float *angle1, const uint8_t *valid1,
                         int n1, const int32_t *nodes1, const int32_t *off1,
                         const int32_t *feats1, int nfv1, const uint8_t *desc2,
                         const float *angle2, const uint8_t *valid2, int n2,
                         const int32_t *nodes2, const int32_t *off2, const int32_t *feats2,
                         int nfv2, float nnratio, int check_ori, int32_t *match12);
void orc_three_maxima(const int *hsize, int *ind1, int *ind2, int *ind3);

/* ---- Frame::ComputeStereoMatches (stereo_oracle.c) ----
 * kl/dl: left keypoints (mvKeys) + descriptors, kr/dr: right.  pyr_l / pyr_r: the two
 * pyramids packed as orc_extract writes them.  min_z: Frame::mb (see stereo_oracle.c).
 * uright/depth[nl] receive mvuRight / mvDepth (-1 where unmatched).  Returns the number of
 * keypoints with a depth. */
int orc_stereo_matches(const orc_params *p, const orc_keypoint *kl, const uint8_t *dl, int nl,
                       const orc_keypoint *kr, const uint8_t *dr, int nr, const uint8_t *pyr_l,
                       const uint8_t *pyr_r, int w, int h, float bf, float min_z,
                       float *uright, float *depth);

/* ---- local BA edge linearisation (double) ---- */
typedef struct {
    double q[4];   /* x, y, z, w (Eigen coeffs order) */
    double t[3];
    int32_t fixed;
    int32_t pad;
} orc_pose;

typedef struct {
    int32_t point;     /* vertex 0 (VertexSBAPointXYZ) */
    int32_t pose;      /* vertex 1 (VertexSE3Expmap)  */
    int32_t stereo;    /* 0: EdgeSE3ProjectXYZ, 1: EdgeStereoSE3ProjectXYZ */
    int32_t robust;    /* 1: Huber attached (first optimize), 0: removed */
    int32_t active;    /* level 0 edge (1) or setLevel(1) edge (0) */
    int32_t pad;
    double obs[3];
    double inv_sigma2;
    double fx, fy, cx, cy, bf;
    double huber_delta;   /* (double)(float)sqrt(5.991) / sqrt(7.815) */
} orc_edge;

typedef struct {
    double err[3];
    double chi2;
    double rho1;       /* Huber weight */
    double jp[3][3];   /* _jacobianOplusXi (point) */
    double jt[3][6];   /* _jacobianOplusXj (pose)  */
    double hpl[3][6];  /* per-edge off-diagonal block A^T W B */
} orc_edge_out;

/* computeError + linearizeOplus + constructQuadraticForm for every active edge.
 * hpose: npose*36 + bpose: npose*6, hpoint: npoint*9 + bpoint: npoint*3 (zeroed here). */
void orc_ba_linearize(const orc_pose *poses, int npose, const double *points, int npoint,
                      const orc_edge *edges, int nedge, orc_edge_out *eout, double *hpose,
                      double *bpose, double *hpoint, double *bpoint);
double orc_ba_errors(const orc_pose *poses, const double *points, const orc_edge *edges,
                     int nedge, double *err, double *chi2, double *rho0, uint8_t *depth_ok);
/* BlockSolver_6_3::solve with the Schur complement (block_solver.hpp:354-486) after
 * setLambda(lambda): inputs are orc_ba_linearize's outputs (hpl = A^T W B per edge).
 * dx_pose[npose*6] (0 for fixed poses), dx_point[npoint*3] (0 for points without an
 * active edge).  Returns the linear solver's success. */
int orc_ba_schur_solve(const orc_pose *poses, int npose, int npoint, const orc_edge *edges,
                       int nedge, const orc_edge_out *eout, const double *hpose,
                       const double *bpose, const double *hpoint, const double *bpoint,
                       double lambda, double *dx_pose, double *dx_point);
int orc_ldlt_dense_solve(double *A, int n, double *x);
/* SparseOptimizer::update for the two vertex types (in place; fixed poses untouched) */
void orc_ba_update(orc_pose *poses, int npose, double *points, int npoint, const double *dx_pose,
                   const double *dx_point);
/* optimizer.optimize(iterations) with OptimizationAlgorithmLevenberg (in place).  report[6] =
 * iterations run, trials, terminated (0, 1: rho 0 / 10 failed trials, 2: three weak
 * iterations), chi2 before, chi2 after, final lambda.  Returns the iterations run. */
int orc_ba_optimize(orc_pose *poses, int npose, double *points, int npoint, const orc_edge *edges,
                    int nedge, int iterations, double report[6]);
int orc_ba_optimize_ctl(orc_pose *poses, int npose, double *points, int npoint,
                        const orc_edge *edges, int nedge, int iterations, int stop_it,
                        int stop_trial, double *last_chi2, double report[6]);
/* central-difference Jacobian of computeError (base_binary_edge.hpp:131-205, delta 1e-9) */
void orc_ba_numeric_jacobian(const orc_pose *pose, const double *xyz, const orc_edge *e,
                             double jp[3][3], double jt[3][6]);

#ifdef __cplusplus
}
#endif
#endif
