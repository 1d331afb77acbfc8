/*
 * orbg.h -- C ABI of the MI355X-native ORB-SLAM2 hot path (liborbg.so).
 *
 * Plain pointers and sizes only; no C++ or torch types cross this boundary.
 * Each entry point replaces one reference interface (/root/reference):
 *
 *   orbg_create / orbg_params ....... ORBextractor::ORBextractor(nfeatures, scaleFactor,
 *                                     nlevels, iniThFAST, minThFAST)   include/ORBextractor.h:64-65
 *                                                                      src/ORBextractor.cc:432-521
 *   orbg_get_scale_tables ........... GetLevels/GetScaleFactor(s)/GetInverseScaleFactors/
 *                                     GetScaleSigmaSquares/GetInverseScaleSigmaSquares
 *                                                                      include/ORBextractor.h:78-98
 *   orbg_extract .................... ORBextractor::operator()(image, mask, keypoints, descriptors)
 *                                                                      include/ORBextractor.h:74-76
 *                                                                      src/ORBextractor.cc:1330-1397
 *   orbg_get_level .................. public std::vector<cv::Mat> mvImagePyramid
 *                                                                      include/ORBextractor.h:101
 *   orbg_descriptor_distance ........ static ORBmatcher::DescriptorDistance
 *                                                                      src/ORBmatcher.cc:1846-1862
 *   orbg_hamming_knn2 ............... brute-force 2-NN over DescriptorDistance (the matcher
 *                                     loops' strict-< best/second rule, ORBmatcher.cc:541-556)
 *   orbg_search_for_initialization .. ORBmatcher(nnratio,checkOri).SearchForInitialization(
 *                                     F1, F2, vbPrevMatched, vnMatches12, windowSize)
 *                                                                      src/ORBmatcher.cc:487-631
 *   orbg_stereo_batch_device ........ Frame::ComputeStereoMatches  src/Frame.cc:619-834
 *   orbg_search_by_projection_lastframe
 *                                     ORBmatcher(0.9,true).SearchByProjection(CurrentFrame,
 *                                     LastFrame, th, bMono)         src/ORBmatcher.cc:1503-1667
 *   orbg_search_by_projection_local . ORBmatcher(nnratio).SearchByProjection(F, vpMapPoints, th)
 *                                                                      src/ORBmatcher.cc:59-154
 *   orbg_pose_optimization .......... Optimizer::PoseOptimization(Frame*)  src/Optimizer.cc:356-631
 *   orbg_ba_schur_solve ............. g2o BlockSolver<6,3>::solve (Schur complement + pose solve)
 *                                     Thirdparty/g2o/g2o/core/block_solver.hpp:354-486
 *   orbg_vocab_load_text ............ TemplatedVocabulary::loadFromTextFile
 *                                     Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1337-1420
 *   orbg_bow_transform .............. TemplatedVocabulary::transform(features, BowVector,
 *                                     FeatureVector, levelsup) as Frame::ComputeBoW calls it
 *                                     TemplatedVocabulary.h:1126-1189, 1220-1259; Frame.cc:532-539
 *   orbg_search_by_bow .............. ORBmatcher::SearchByBoW(KeyFrame*, Frame&, ...)
 *                                     src/ORBmatcher.cc:195-348 (Tracking.cc:1069, 2009)
 *   orbg_search_by_bow_kf ........... ORBmatcher::SearchByBoW(KeyFrame*, KeyFrame*, vpMatches12)
 *                                     src/ORBmatcher.cc:634-769 (LoopClosing.cc:485)
 *   orbg_undistort_keypoints ........ Frame::UndistortKeyPoints  src/Frame.cc:542-572
 *   orbg_compute_image_bounds ....... Frame::ComputeImageBounds  src/Frame.cc:575-611
 *   orbg_is_in_frustum .............. Frame::isInFrustum(pMP, viewingCosLimit)  src/Frame.cc:342-409
 *                                     (Tracking::SearchLocalPoints, Tracking.cc:1676-1691)
 *   orbg_distinctive_descriptor ..... MapPoint::ComputeDistinctiveDescriptors  src/MapPoint.cc:342-420
 *   orbg_search_for_triangulation ... ORBmatcher::SearchForTriangulation(pKF1, pKF2, F12,
 *                                     vMatchedPairs, bOnlyStereo)  src/ORBmatcher.cc:779-957
 *                                     (LocalMapping::CreateNewMapPoints, LocalMapping.cc:378)
 *   orbg_fuse ....................... ORBmatcher::Fuse(pKF, vpMapPoints, th)'s per-MapPoint search
 *   orbg_fuse_sim3 .................. ORBmatcher::Fuse(pKF, Scw, vpPoints, th, vpReplacePoint)'s search
 *   orbg_search_by_projection_reloc . ORBmatcher::SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist)
 *   orbg_search_by_projection_sim3 .. ORBmatcher::SearchByProjection(pKF, Scw, vpPoints, vpMatched, th)
 *   orbg_rgbd_stereo ................ Frame::ComputeStereoFromRGBD (+ GrabImageRGBD's depth scaling)
 *   orbg_search_by_sim3 ............. ORBmatcher::SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th)
 *                                     src/ORBmatcher.cc:968-1069 (LocalMapping::SearchInNeighbors,
 *                                     LocalMapping.cc:622-690)
 *   orbg_ba_linearize ............... g2o computeActiveErrors + BlockSolver::buildSystem arithmetic
 *                                     for EdgeSE3ProjectXYZ / EdgeStereoSE3ProjectXYZ inside
 *                                     Optimizer::LocalBundleAdjustment  src/Optimizer.cc:633-979
 *
 * Batched, device-resident entry points (orbg_*_device) run the same kernels over many
 * frames at once; they exist for the batched-sequence mode and the bench.
 *
 * Conventions: every int-returning function returns ORBG_OK (0) or a negative errno-style
 * code; orbg_last_error() gives a message for the calling thread.  No C++ exception crosses
 * the ABI.  The caller owns all output buffers.  A context owns its device buffers and one
 * HIP stream; a context is not thread-safe, distinct contexts may run concurrently (the two
 * stereo extractors of Frame.cc:110-113).
 */
#ifndef ORBG_H
#define ORBG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORBG_ABI_VERSION 1
#define ORBG_MAX_LEVELS 16

#define ORBG_OK 0
#define ORBG_EIO -5       /* HIP runtime / device error */
#define ORBG_ENOMEM -12
#define ORBG_EINVAL -22
#define ORBG_ERANGE -34   /* caller capacity too small; *n_out holds the needed count */
#define ORBG_ENOTSUP -95  /* configuration outside what the reference defines */

/* cv::resize INTER_LINEAR 8UC1 vertical-pass variant (OpenCV build pin) */
#define ORBG_RESIZE_SCALAR 0
#define ORBG_RESIZE_SSE2_16_4 4
#define ORBG_RESIZE_SIMD_16_8 8

typedef struct orbg_ctx orbg_ctx;

typedef struct {
    /* ORBextractor ctor arguments */
    int32_t nfeatures;
    float scale_factor;
    int32_t nlevels;
    int32_t ini_th_fast;
    int32_t min_th_fast;
    /* OpenCV primitive pins (orbg_params_default sets the OpenCV 3.4 values) */
    int32_t resize_mode;   /* ORBG_RESIZE_* */
    int32_t gauss_k[7];    /* GaussianBlur 7x7 sigma=2 fixed-point weights */
    int32_t brief_fma;     /* 1: fuse x*b + y*a in rBRIEF sampling (reference built -ffp-contract=fast) */
    /* batch capacity (frames per orbg_extract_batch_device call); 0 -> 1 */
    int32_t max_batch;
    /* cos/sin of the rBRIEF rotation (ORBextractor.cc:122, (float)cos(float) = glibc cosf):
     * ORBG_SINCOS_GLIBC restates glibc 2.35's sinf/cosf (bit-equal to the host libm on every
     * float in [0, 7)); ORBG_SINCOS_PINNED is round 1's correctly rounded evaluation */
    int32_t sincos_mode;
} orbg_params;

#define ORBG_SINCOS_GLIBC 0
#define ORBG_SINCOS_PINNED 1

/* cv::KeyPoint layout: pt.x, pt.y, size, angle, response, octave, class_id (28 bytes) */
typedef struct {
    float x, y, size, angle, response;
    int32_t octave, class_id;
} orbg_keypoint;

/* ---------------- context / extractor ---------------- */
void orbg_params_default(orbg_params *p);
int orbg_create(int device, const orbg_params *p, orbg_ctx **out);
void orbg_destroy(orbg_ctx *ctx);
const char *orbg_last_error(void);
int orbg_abi_version(void);

/* GetLevels / GetScaleFactor(s) / inverse / sigma^2 tables; any pointer may be NULL.
 * Arrays must hold nlevels entries.  features_per_level = mnFeaturesPerLevel, umax[16]. */
int orbg_get_scale_tables(const orbg_ctx *ctx, int32_t *nlevels, float *scale_factor,
                          float *scale, float *inv_scale, float *sigma2, float *inv_sigma2,
                          int32_t *features_per_level, int32_t *umax);
/* the 256 rBRIEF test pairs (x0,y0,x1,y1) the kernels use (bit_pattern_31_) */
int orbg_get_pattern(int32_t out[1024]);

/* ORBextractor::operator() on one host image (CV_8UC1, row pitch `step`).
 * w == 0 or h == 0: returns ORBG_OK with *n_out = -1 and outputs untouched (:1333-1334).
 * Otherwise kps[0..n) in level order, desc n x 32 bytes row-major.  If cap < n, returns
 * ORBG_ERANGE with *n_out = n and nothing written. */
int orbg_extract(orbg_ctx *ctx, const uint8_t *img, int w, int h, size_t step,
                 orbg_keypoint *kps, uint8_t *desc, int cap, int *n_out);

/* mvImagePyramid[level] of frame `frame` of the last extraction (host copy). */
int orbg_get_level(orbg_ctx *ctx, int frame, int level, uint8_t *dst, size_t dst_step, int *lw,
                   int *lh);
/* The GaussianBlur(7x7, sigma 2, REFLECT_101) of pyramid level `level` of frame `frame` of the
 * last extraction: the image computeOrbDescriptor samples (ORBextractor.cc:1375-1377, a local
 * cv::Mat there, no public member).  Parity / debugging accessor; same contract as
 * orbg_get_level. */
int orbg_get_blurred_level(orbg_ctx *ctx, int frame, int level, uint8_t *dst, size_t dst_step,
                           int *lw, int *lh);

/* ---------------- batched, device-resident ---------------- */
/* d_imgs: device pointer, nframes images of w x h, row pitch `step`, frame pitch
 * `frame_stride` bytes.  Enqueued on the context stream; the caller keeps d_imgs alive
 * until the next call (level 0 of the pyramid IS the input). */
int orbg_extract_batch_device(orbg_ctx *ctx, const uint8_t *d_imgs, int nframes, int w, int h,
                              size_t step, size_t frame_stride);
/* device pointers to the last batch's outputs: frame f keypoints at d_kps + f*frame_cap,
 * descriptors at d_desc + f*frame_cap*32, count d_counts[f]. */
int orbg_batch_outputs(orbg_ctx *ctx, orbg_keypoint **d_kps, uint8_t **d_desc,
                       int32_t **d_counts, int32_t *frame_cap);
/* copy frame `frame` of the last batch to the host (synchronises) */
int orbg_download_frame(orbg_ctx *ctx, int frame, orbg_keypoint *kps, uint8_t *desc, int cap,
                        int *n_out);

/* Match pairs of frames of the last batch on the device: for pair i, F1 = frame f1[i]
 * (reference / previous), F2 = frame f2[i] (current).
 *  - knn2: for every F2 keypoint, best/second distance and best index over all F1
 *    descriptors (all-pairs Hamming).
 *  - SearchForInitialization(F1, F2, vbPrevMatched = F1 keypoint positions, window)
 *    with image bounds (0, w, 0, h) (undistorted KITTI-style frames, Frame.cc:603-609).
 * Results stay on the device (orbg_match_outputs). */
int orbg_match_batch_device(orbg_ctx *ctx, const int32_t *f1, const int32_t *f2, int npairs,
                            int window, float nnratio, int check_ori);
int orbg_match_outputs(orbg_ctx *ctx, int32_t **d_knn /* [npairs][frame_cap][3] */,
                       int32_t **d_matches12 /* [npairs][frame_cap] */,
                       int32_t **d_nmatches /* [npairs] */, int32_t *frame_cap);
int orbg_download_matches(orbg_ctx *ctx, int pair, int32_t *knn, int32_t *matches12,
                          int cap, int32_t *nmatches);

/* Extraction runs on the context stream; batch matching and the summary run on a second
 * (match) stream so the matching of batch k overlaps the extraction of batch k+1.  The
 * per-frame outputs alternate between two buffers (orbg_batch_outputs returns the ones of
 * the last extraction); every host-side read (download, get_level, stats, sync) drains
 * both streams. */
/* Frame::ComputeStereoMatches (src/Frame.cc:619-834) for npairs (left, right) frames of the
 * last batch: row-band descriptor match, 11x11 SAD refinement at the keypoint's level,
 * parabola, median cut.  bf = Frame::mbf; min_z = Frame::mb, which the reference reads before
 * assigning it (Frame.cc:661 vs :148) -- pass bf / fx, the value assigned right after
 * (min_z <= 0: no maximum disparity).  Runs where the batch's keypoint half ran (it reads
 * this batch's pyramid): the context stream, or with pipelined batches the internal back
 * stream.  Results per pair over the left frame's keypoints: mvuRight, mvDepth (-1 where
 * unmatched) and the number of depths; device readers order themselves after the match
 * stream via orbg_stereo_summary, or call orbg_sync. */
int orbg_stereo_batch_device(orbg_ctx *ctx, const int32_t *left, const int32_t *right,
                             int npairs, float bf, float min_z);
int orbg_stereo_outputs(orbg_ctx *ctx, float **d_uright /* [npairs][frame_cap] */,
                        float **d_depth /* [npairs][frame_cap] */,
                        int32_t **d_nvalid /* [npairs] */, int32_t *frame_cap);
/* The stereo Frame constructor on host images (Frame.cc:86-161): ORBextractor on the left
 * and right image (both CV_8UC1, same size and row pitch) + ComputeStereoMatches.  Outputs
 * as orbg_extract for each image (ORBG_ERANGE with *n_l / *n_r set if a capacity is short);
 * uright / depth receive *n_l entries (mvuRight, mvDepth). */
int orbg_stereo_frame(orbg_ctx *ctx, const uint8_t *left, const uint8_t *right, int w, int h,
                      size_t step, float bf, float min_z, orbg_keypoint *kps_l, uint8_t *desc_l,
                      int cap_l, int *n_l, orbg_keypoint *kps_r, uint8_t *desc_r, int cap_r,
                      int *n_r, float *uright, float *depth);
/* per-pair summary of the last stereo batch, written on the match stream (orbg_match_stream,
 * ordered after the stereo pass, as orbg_batch_summary) into a device buffer: order readers
 * after the match stream, or orbg_sync.  d_out[p] = keypoints of the left frame of pair p,
 * d_out[npairs + p] = keypoints with a depth */
int orbg_stereo_summary(orbg_ctx *ctx, int32_t *d_out);
/* copies cap entries of pair `pair` (synchronises) */
int orbg_download_stereo(orbg_ctx *ctx, int pair, float *uright, float *depth, int cap,
                         int32_t *nvalid);

/* Device error flags are sticky: a frame whose quadtree level overflowed a capacity (its
 * keypoints would be incomplete) sets a flag that stays set until read.  orbg_sync,
 * orbg_check_errors, orbg_batch_stats and orbg_download_frame drain the streams, read and
 * clear it, and return ORBG_ENOTSUP (orbg_last_error names the flags and the first frame)
 * if any batch since the last read raised one.  The device matchers that read per-pair
 * counts from device memory (orbg_fuse[_sim3]_batch_device, orbg_search_by_sim3_batch_device)
 * clamp a count past its capacity (KeyFrame counts to `cap`, MapPoint counts to `mcap`) and
 * raise flag 0x10000; the next read returns ORBG_EINVAL naming the first pair. */
int orbg_sync(orbg_ctx *ctx);
int orbg_check_errors(orbg_ctx *ctx);
void *orbg_stream(orbg_ctx *ctx);       /* hipStream_t of extraction (and host-data calls) */
void *orbg_match_stream(orbg_ctx *ctx); /* hipStream_t of batch matching and the summary */
/* launch on a caller-owned hipStream_t (e.g. torch's current stream) instead of the
 * context's own; NULL restores the context stream */
int orbg_set_stream(orbg_ctx *ctx, void *stream);
/* Pipelined batches (batched-sequence mode; no reference counterpart -- the reference
 * extracts one frame per Tracking call): with enable != 0 the image half of a batch
 * (pyramid, FAST cells, GaussianBlur) runs on the context stream and its keypoint half
 * (quadtree, orientation + rBRIEF, stereo) on an internal high-priority stream, so the image
 * half of batch k+1 overlaps the keypoint half of batch k.  Outputs, the batch's errors and
 * the summary are unchanged; the per-frame outputs of a batch are complete when the match
 * stream's work on them is (orbg_match_batch_device / orbg_batch_summary order themselves
 * after it) or after orbg_sync.  The batch's input images must stay unchanged until then.
 * Also selected with the environment variable ORBG_PIPELINE=1 at orbg_create.
 * Synchronises.  ORBG_ENOTSUP without the internal stream. */
int orbg_set_pipeline(orbg_ctx *ctx, int enable);
int orbg_get_pipeline(const orbg_ctx *ctx);
/* Serial execution (measurement; no reference counterpart): with enable != 0 every
 * extraction kernel runs on the context stream, one after the other (no pipelining, no
 * internal streams), so per-kernel event times are the kernels' own.  Outputs unchanged.
 * Synchronises. */
int orbg_set_serial(orbg_ctx *ctx, int enable);
/* Caller buffers written on the match stream (orbg_batch_summary, orbg_batch_matches,
 * orbg_match_pose_batch_device, orbg_stereo_summary) are stream-ordered on the writer side:
 * at entry each records an event on the context stream (orbg_set_stream) and the match
 * stream waits for it, so work the caller queued on the context stream before the call (a
 * fill of d_out, an upload) completes before liborbg writes.  Work on any OTHER stream must
 * be ordered by the caller.  Readers order themselves after orbg_match_stream, or orbg_sync.
 *
 * per-frame trajectory summary of the last batch, written on the match stream into a
 * device buffer: d_out[f] = keypoints of frame f (f < nframes), then
 * d_out[nframes + p] = SearchForInitialization matches of pair p (p < npairs of the last
 * orbg_match_batch_device, 0 if none) */
int orbg_batch_summary(orbg_ctx *ctx, int32_t *d_out);
/* Caller reads of the last batch's device outputs (orbg_batch_outputs, and
 * orbg_stereo_outputs after a stereo pass) on a caller stream (NULL: the match stream), for
 * pipelined batches where they are written on internal streams:
 *   orbg_batch_acquire: `stream` waits until those outputs are written;
 *   orbg_batch_release: every read enqueued on `stream` so far finishes before liborbg
 *   overwrites those outputs (the extraction that reuses the output slot, the next stereo
 *   pass wait for it).  Releases on several reader streams of one batch chain: each waits
 *   for the previous release, so the slot waits for every reader.
 * Enqueue only; no host synchronisation. */
int orbg_batch_acquire(orbg_ctx *ctx, void *stream);
int orbg_batch_release(orbg_ctx *ctx, void *stream);
/* vnMatches12 of every pair of the last orbg_match_batch_device (ORBmatcher.cc:487-631's
 * output; the batched-sequence gather of SURVEY 8e), written on the match stream into a
 * device buffer: d_out[p * frame_cap + i] = index in frame f2[p] matched to keypoint i of
 * frame f1[p], -1 if none or i >= keypoints of f1[p].  *frame_cap (if non-NULL) receives the
 * row length; d_out == NULL only queries it.  ORBG_EINVAL without a match batch. */
int orbg_batch_matches(orbg_ctx *ctx, int32_t *d_out, int32_t *frame_cap);
/* host-side statistics of the last batch (synchronises): FAST candidates over all
 * cells/levels/frames and output keypoints over all frames (for bandwidth accounting) */
int orbg_batch_stats(orbg_ctx *ctx, int64_t *ncandidates, int64_t *nkeypoints);
/* the quadtree launch plan of the last planned image size (DistributeOctTree,
 * ORBextractor.cc:668-951): the FAST-candidate caps of level 0's split pair of k_octree_lds
 * launches in a batch (first_cap; 0 = no split) and of its single launch (level0_cap), and of
 * the levels-1.. launch (upper_cap); a level with more candidates goes to the k_octree
 * fallback.  ORBG_EINVAL before any extraction. */
int orbg_get_quadtree_caps(const orbg_ctx *ctx, int32_t *first_cap, int32_t *level0_cap,
                           int32_t *upper_cap);
/* the GaussianBlur plan of the last planned image size (ORBextractor.cc:1375-1377): *fused =
 * 1 when the FAST cells blur their detection regions from the window tiles they stage (the
 * pixels of every level's rectangle of regions, *interior_px per frame) and a border pass
 * blurs the rest (*border_px per frame); 0 when one blur pass covers every level.  Any
 * pointer may be NULL.  ORBG_EINVAL before any extraction. */
int orbg_get_blur_plan(const orbg_ctx *ctx, int32_t *fused, int64_t *interior_px,
                       int64_t *border_px);
/* the blurred levels' device layout of the last planned image size: *tiled = 1 for 16 x 8-pixel
 * tiles of 128 bytes (k_blur2's default store form, read by the rBRIEF phase), 0 for rows
 * (ORBG_BLUR_TILED=0 at orbg_create, or a blur written by another pass).  Internal; the
 * accessor orbg_get_blurred_level always returns rows.  ORBG_EINVAL before any extraction. */
int orbg_get_blur_layout(const orbg_ctx *ctx, int32_t *tiled);

/* per-kernel timing with HIP events on the context stream (for bench roofline) */
int orbg_profile_enable(orbg_ctx *ctx, int enable);
/* returns number of kernel kinds; fills name/total_ms/launches for index i */
int orbg_profile_read(orbg_ctx *ctx, int i, const char **name, double *total_ms,
                      int64_t *launches);
int orbg_profile_reset(orbg_ctx *ctx);

/* ---------------- matcher (host data) ---------------- */
int orbg_descriptor_distance(const uint8_t *a, const uint8_t *b);

/* best/second over all train descriptors for every query (strict <, lowest index on ties) */
int orbg_hamming_knn2(orbg_ctx *ctx, const uint8_t *qdesc, int nq, const uint8_t *tdesc, int nt,
                      int32_t *best_idx, int32_t *best_dist, int32_t *second_dist);

typedef struct {
    float min_x, max_x, min_y, max_y; /* Frame::mnMinX, mnMaxX, mnMinY, mnMaxY */
} orbg_bounds;

/* kps1/kps2 are mvKeysUn (x, y, angle, octave used); prev_xy (2*n1 floats) is
 * vbPrevMatched, updated in place; matches12[n1] = vnMatches12. */
int orbg_search_for_initialization(orbg_ctx *ctx, const orbg_keypoint *kps1,
                                   const uint8_t *desc1, int n1, const orbg_keypoint *kps2,
                                   const uint8_t *desc2, int n2, const orbg_bounds *bounds2,
                                   float *prev_xy, int32_t *matches12, int window,
                                   float nnratio, int check_ori, int *nmatches);

/* ---------------- tracking matchers ----------------
 * The MapPoint / Frame state the two SearchByProjection loops read enters as flat records;
 * their writes come back as match[N] (CurrentFrame.mvpMapPoints as a query index; -1 = not
 * written; -2 = set to NULL by the rotation-consistency filter) and nmatches.  The frame side is CurrentFrame (F): kps = mvKeysUn,
 * desc = mDescriptors, uright = mvuRight (NULL for monocular), taken0 (NULL = none) =
 * "mvpMapPoints[i] && mvpMapPoints[i]->Observations() > 0" on entry, bounds = mnMinX...
 * Scale factors are the context's (ORBextractor GetScaleFactors). */
#define ORBG_MP_VALID 1    /* lastframe: pMP && !LastFrame.mvbOutlier[i]; local: mbTrackInView && !isBad() */
#define ORBG_MP_HAS_OBS 2  /* pMP->Observations() > 0 */

typedef struct {
    float x, y, z;     /* pMP->GetWorldPos() */
    int32_t octave;    /* LastFrame.mvKeys[i].octave */
    float angle;       /* LastFrame.mvKeysUn[i].angle */
    int32_t flags;     /* ORBG_MP_* */
} orbg_lastframe_point;

typedef struct {
    float u, v, ur;    /* mTrackProjX, mTrackProjY, mTrackProjXR (Frame::isInFrustum) */
    int32_t level;     /* mnTrackScaleLevel */
    float view_cos;    /* mTrackViewCos */
    int32_t flags;     /* ORBG_MP_* */
} orbg_map_projection;

typedef struct {
    float Tcw[12];     /* CurrentFrame.mTcw rows 0..2 (row-major 3x4) */
    float Tlw[12];     /* LastFrame.mTcw rows 0..2 */
    float fx, fy, cx, cy, bf, b;  /* Frame::fx.., mbf, mb */
    int32_t mono;      /* bMono */
    int32_t pad;
} orbg_track_camera;

/* ORBmatcher(nnratio, checkOri).SearchByProjection(CurrentFrame, LastFrame, th, bMono):
 * pts[np] / pdesc = LastFrame.mvpMapPoints[i] (one record per LastFrame keypoint). */
int orbg_search_by_projection_lastframe(orbg_ctx *ctx, const orbg_keypoint *kps,
                                        const uint8_t *desc, const float *uright, int n,
                                        const uint8_t *taken0, const orbg_bounds *bounds,
                                        const orbg_lastframe_point *pts, const uint8_t *pdesc,
                                        int np, const orbg_track_camera *cam, float th,
                                        int check_ori, int32_t *match, int *nmatches);

/* ORBmatcher(nnratio).SearchByProjection(F, vpMapPoints, th): mps[nm] / mdesc. */
int orbg_search_by_projection_local(orbg_ctx *ctx, const orbg_keypoint *kps,
                                    const uint8_t *desc, const float *uright, int n,
                                    const uint8_t *taken0, const orbg_bounds *bounds,
                                    const orbg_map_projection *mps, const uint8_t *mdesc, int nm,
                                    float th, float nnratio, int32_t *match, int *nmatches);

/* Batched, device-resident form of both (mode ORBG_TRACK_LASTFRAME / ORBG_TRACK_LOCAL) and
 * of the relocalization / loop searches below (ORBG_TRACK_RELOC / ORBG_TRACK_LOOP): every
 * pointer is device memory, frame f's arrays at f * frame_cap (keypoint side) and
 * f * query_cap (query side); enqueued on the context stream. */
#define ORBG_TRACK_LASTFRAME 0
#define ORBG_TRACK_LOCAL 1
#define ORBG_TRACK_RELOC 2
#define ORBG_TRACK_LOOP 3
struct orbg_frustum_camera;
typedef struct {
    const orbg_keypoint *kps;    /* [B][frame_cap] */
    const uint8_t *desc;         /* [B][frame_cap][32] */
    const float *uright;         /* [B][frame_cap] or NULL */
    const uint8_t *taken0;       /* [B][frame_cap] or NULL */
    const int32_t *counts;       /* [B] */
    const orbg_bounds *bounds;   /* [B] */
    int32_t frame_cap;
    const void *queries;         /* [B][query_cap] orbg_lastframe_point / orbg_map_projection /
                                    orbg_reloc_point / orbg_map_point, by mode */
    const uint8_t *qdesc;        /* [B][query_cap][32] */
    const int32_t *qcounts;      /* [B] */
    int32_t query_cap;
    const orbg_track_camera *cams;  /* [B], last-frame mode */
    float th, nnratio;
    int32_t check_ori;
    int32_t *match;              /* [B][frame_cap] out */
    int32_t *nmatches;           /* [B] out */
    /* appended in round 4 (ABI note): read only in the relocalization / loop
     * modes, so a caller built against the older, shorter struct stays valid in the
     * last-frame / local-map modes */
    const struct orbg_frustum_camera *fcams;  /* [B], relocalization / loop modes */
    int32_t orb_dist;            /* relocalization: ORBdist */
} orbg_track_batch;
int orbg_search_by_projection_batch_device(orbg_ctx *ctx, int mode, const orbg_track_batch *tb,
                                           int nframes);

/* ---------------- Frame / MapPoint geometry ---------------- */
/* Frame::mK (fx, fy, cx, cy) and Frame::mDistCoef (k1, k2, p1, p2[, k3]: k3 = 0 when the
 * settings file has none, Tracking.cc's DistCoef of 4 entries) */
typedef struct {
    float fx, fy, cx, cy;
    float k1, k2, p1, p2, k3;
} orbg_camera;

/* Frame::UndistortKeyPoints (src/Frame.cc:542-572): kps_un[i] = kps[i] with pt replaced by
 * cv::undistortPoints(pt, K, D, noArray(), K) (OpenCV 3.4: 5 fixed-point iterations in
 * double); k1 == 0: a copy (mvKeysUn = mvKeys).  Host arrays; kps_un may alias
 * kps. */
int orbg_undistort_keypoints(orbg_ctx *ctx, const orbg_camera *cam, const orbg_keypoint *kps,
                             int n, orbg_keypoint *kps_un);
/* The same on the device for a batch: frame f's counts[f] keypoints at d_kps + f * frame_cap
 * -> d_kps_un + f * frame_cap (entries past counts[f] untouched).  Context stream. */
int orbg_undistort_batch_device(orbg_ctx *ctx, const orbg_camera *cam, const orbg_keypoint *d_kps,
                                const int32_t *d_counts, int frame_cap, int nframes,
                                orbg_keypoint *d_kps_un);
/* Frame::ComputeStereoFromRGBD (src/Frame.cc:837-858; the RGB-D Frame constructor) after
 * Tracking::GrabImageRGBD's depth conversion (Tracking.cc:233-234: imDepth.convertTo(CV_32F,
 * mDepthMapFactor) when |mDepthMapFactor - 1| > 1e-5 or the image is not CV_32F).  depth:
 * a w x h image, row pitch `pitch` bytes, ORBG_DEPTH_U16 (raw) or ORBG_DEPTH_F32; factor =
 * mDepthMapFactor (1 / DepthMapFactor of the settings); a pixel's depth is raw * factor
 * rounded once to float (convertTo's float alpha), or the float itself when it is F32 and
 * factor is within 1e-5 of 1.  kps = mvKeys (their truncated (x, y) index the depth image;
 * outside it: no depth), kps_un = mvKeysUn.  Per keypoint: d > 0 -> depth[i] = d,
 * uright[i] = kps_un[i].x - mbf / d; else both -1. */
#define ORBG_DEPTH_F32 0
#define ORBG_DEPTH_U16 1
int orbg_rgbd_stereo(orbg_ctx *ctx, const void *depth, int depth_type, float factor, int w, int h,
                     size_t pitch, const orbg_keypoint *kps, const orbg_keypoint *kps_un, int n,
                     float mbf, float *uright, float *depth_out);
/* The same on the device for a batch: frame f's depth image at d_depth + f * image_stride
 * bytes, its counts[f] keypoints at d_kps / d_kps_un + f * frame_cap, outputs at + f * frame_cap
 * (entries past counts[f] untouched).  Context stream. */
int orbg_rgbd_stereo_batch_device(orbg_ctx *ctx, const void *d_depth, int depth_type, float factor,
                                  int w, int h, size_t pitch, size_t image_stride,
                                  const orbg_keypoint *d_kps, const orbg_keypoint *d_kps_un,
                                  const int32_t *d_counts, int frame_cap, int nframes, float mbf,
                                  float *d_uright, float *d_depth_out);
/* Frame::ComputeImageBounds (src/Frame.cc:575-611) for a w x h image: mnMinX .. mnMaxY (the
 * undistorted image corners when k1 != 0, else 0, w, 0, h).  Host only (four points, the
 * expression k_undistort evaluates). */
int orbg_compute_image_bounds(const orbg_camera *cam, int w, int h, orbg_bounds *out);
/* Batched-sequence mode with a distorted camera (TUM / EuRoC settings): after
 * orbg_set_camera(ctx, cam) with cam->k1 != 0, orbg_match_batch_device first undistorts the
 * batch's keypoints on the match stream (Frame::UndistortKeyPoints, as the Frame constructor
 * does after ExtractORB, Frame.cc:259) and SearchForInitialization (and the pose stub)
 * read mvKeysUn with ComputeImageBounds' bounds; orbg_batch_keys_un returns the device array
 * ([frames][frame_cap], valid after that match stream work).  cam == NULL or k1 == 0: the
 * default (mvKeysUn = mvKeys, bounds 0, w, 0, h). */
int orbg_set_camera(orbg_ctx *ctx, const orbg_camera *cam);
int orbg_batch_keys_un(orbg_ctx *ctx, orbg_keypoint **d_kps_un, int32_t *frame_cap);

/* What Frame::isInFrustum reads of a MapPoint: GetWorldPos(), GetNormal(), mfMinDistance,
 * mfMaxDistance; flags: ORBG_MP_VALID = Tracking::SearchLocalPoints tests the point
 * (!isBad() && mnLastFrameSeen != CurrentFrame.mnId, Tracking.cc:1680-1683), ORBG_MP_HAS_OBS
 * passed through to the projection. */
typedef struct {
    float x, y, z;
    float nx, ny, nz;
    float min_dist, max_dist;
    int32_t flags;
} orbg_map_point;
/* The Frame state isInFrustum reads: mTcw rows 0..2 (row-major 3x4), fx, fy, cx, cy, mbf,
 * mfLogScaleFactor (= log(mfScaleFactor), in double then float), mnScaleLevels, mnMinX.. */
typedef struct orbg_frustum_camera {
    float Tcw[12];
    float fx, fy, cx, cy, bf;
    float log_scale_factor;
    int32_t nlevels;
    orbg_bounds bounds;
} orbg_frustum_camera;
/* Frame::isInFrustum(pMP, viewing_cos_limit) for n map points (host arrays): proj[i] = the
 * mTrack* members SearchByProjection(F, vpMapPoints) reads (orbg_map_projection:
 * mTrackProjX/Y/XR, mnTrackScaleLevel, mTrackViewCos; flags ORBG_MP_VALID = mbTrackInView,
 * ORBG_MP_HAS_OBS passed through).  A point not in view gets only its flags written (the
 * reference leaves the other members as they were).  *nvisible = points in view. */
int orbg_is_in_frustum(orbg_ctx *ctx, const orbg_frustum_camera *cam, const orbg_map_point *mps,
                       int n, float viewing_cos_limit, orbg_map_projection *proj, int *nvisible);
/* Batched, device memory: frame f's counts[f] points at d_mps + f * cap, camera d_cams[f],
 * projections at d_proj + f * cap, d_nvisible[f].  Context stream. */
int orbg_is_in_frustum_batch_device(orbg_ctx *ctx, const orbg_frustum_camera *d_cams,
                                    const orbg_map_point *d_mps, const int32_t *d_counts, int cap,
                                    int nframes, float viewing_cos_limit,
                                    orbg_map_projection *d_proj, int32_t *d_nvisible);
/* MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:342-420) for one map point: the n
 * observation descriptors (n x 32 bytes, in the mObservations order, bad KeyFrames left out)
 * -> *best = BestIdx, the row with the least median distance to the others (the first on
 * ties), -1 if n == 0. */
int orbg_distinctive_descriptor(orbg_ctx *ctx, const uint8_t *desc, int n, int32_t *best);
/* Batched, device memory: map point p's observations are descriptor rows
 * d_pool[d_rows[d_off[p]] .. d_rows[d_off[p+1]-1]] (32 bytes each, e.g. the KeyFrames'
 * mDescriptors resident in HBM); d_best[p] = BestIdx (-1: no observation) and, if d_desc is
 * not NULL, d_desc[p * 32 ..] = that descriptor (mDescriptor).  Context stream. */
int orbg_distinctive_descriptors_batch_device(orbg_ctx *ctx, const uint8_t *d_pool,
                                              const int32_t *d_rows, const int32_t *d_off,
                                              int npoints, int32_t *d_best, uint8_t *d_desc);

/* ---------------- LocalMapping matchers ---------------- */
/* A set of KeyFrames in device memory, frame k's rows at + k * cap (fv_off at + k * (cap + 1)):
 * mDescriptors [cap][32], mvKeysUn [cap] (x, y, angle, octave read), mvuRight [cap] (NULL: all
 * monocular), has_mp [cap] = GetMapPoint(i) != NULL (NULL: none), counts[k] = N, and mFeatVec
 * in orbg_bow_transform_batch_device's layout. */
typedef struct {
    const uint8_t *desc;
    const orbg_keypoint *kps;
    const float *uright;
    const uint8_t *has_mp;
    const int32_t *counts;
    const int32_t *fv_nodes, *fv_off, *fv_feats, *nfv;
} orbg_keyframes;
/* The geometry of one SearchForTriangulation pair: F12 (row-major 3x3, LocalMapping::
 * ComputeF12), pKF1->GetCameraCenter(), pKF2->mTcw rows 0..2 (row-major 3x4) and pKF2's
 * fx, fy, cx, cy (the epipole, ORBmatcher.cc:800-806). */
typedef struct {
    float F12[9];
    float Cw1[3];
    float Tcw2[12];
    float fx2, fy2, cx2, cy2;
} orbg_triangulation_pair;
/* ORBmatcher(nnratio, checkOri).SearchForTriangulation(pKF1, pKF2, F12, vMatchedPairs,
 * bOnlyStereo) for pairs p: KeyFrames d_kf1[p], d_kf2[p] of `kfs`, geometry d_geo[p].
 * d_matches12[p * cap + i] = vMatches12[i] (the pKF2 index matched to pKF1's feature i, -1;
 * vMatchedPairs = the (i, d_matches12[i]) with d_matches12[i] >= 0 in i order) for i < N of
 * pKF1; d_nmatches[p] = the return value.  Scale factors and sigma^2 are the context's
 * (pKF2->mvScaleFactors / mvLevelSigma2).  Context stream.  ORBG_ENOTSUP past 65535
 * features per frame. */
int orbg_search_for_triangulation_batch_device(orbg_ctx *ctx, const orbg_keyframes *kfs, int cap,
                                               const int32_t *d_kf1, const int32_t *d_kf2,
                                               const orbg_triangulation_pair *d_geo, int npairs,
                                               int only_stereo, int check_ori,
                                               int32_t *d_matches12, int32_t *d_nmatches);
/* One KeyFrame from host arrays (as orbg_keyframes, one frame; uright / has_mp may be NULL) */
typedef struct {
    const orbg_keypoint *kps;
    const uint8_t *desc;
    const float *uright;
    const uint8_t *has_mp;
    int32_t n;
    const int32_t *fv_nodes, *fv_off, *fv_feats;
    int32_t nfv;
} orbg_keyframe;
/* The same for one pair from host arrays: matches12[kf1->n], *nmatches. */
int orbg_search_for_triangulation(orbg_ctx *ctx, const orbg_keyframe *kf1, const orbg_keyframe *kf2,
                                  const orbg_triangulation_pair *geo, int only_stereo,
                                  int check_ori, int32_t *matches12, int *nmatches);

/* LocalMapping::CreateNewMapPoints (src/LocalMapping.cc:293-560) around that search: the
 * pair's geometry before it (ComputeF12, :690-707) and the triangulation of its matches after
 * it (:395-560).  A KeyFrame's pose and calibration as they read them: mTcw rows 0..2
 * (row-major 3x4), fx, fy, cx, cy, invfx, invfy, mb, mbf. */
typedef struct {
    float Tcw[12];
    float fx, fy, cx, cy, invfx, invfy, mb, mbf;
} orbg_kf_camera;
/* d_geo[p] = the orbg_triangulation_pair of KeyFrames d_kf1[p] (current) and d_kf2[p]
 * (neighbour), cameras d_cams[kf]: F12 = K1^-T [t12]x R12 K2^-1 in the reference's float
 * evaluation (A.inv()*B as solve(), K2.inv() closed form, gemms in double), pKF1's camera
 * centre, pKF2's pose and intrinsics.  Context stream. */
int orbg_triangulation_geometry_batch_device(orbg_ctx *ctx, const orbg_kf_camera *d_cams,
                                             const int32_t *d_kf1, const int32_t *d_kf2,
                                             int npairs, orbg_triangulation_pair *d_geo);
/* The same for one pair from host structs. */
int orbg_triangulation_geometry(orbg_ctx *ctx, const orbg_kf_camera *cam1,
                                const orbg_kf_camera *cam2, orbg_triangulation_pair *geo);
/* Per-match outcome of the triangulation, the reference's `continue`s in order: */
enum {
    ORBG_TRI_NONE = 0,      /* no match (matches12[i] < 0) */
    ORBG_TRI_NEW = 1,       /* a new MapPoint at x3d */
    ORBG_TRI_PARALLAX = -1, /* no stereo and too little parallax */
    ORBG_TRI_W0 = -2,       /* the homogeneous solution's w == 0 */
    ORBG_TRI_Z1 = -3,       /* behind pKF1 */
    ORBG_TRI_Z2 = -4,       /* behind pKF2 */
    ORBG_TRI_REPROJ1 = -5,  /* chi-square gate in pKF1 (5.991 mono / 7.8 stereo) */
    ORBG_TRI_REPROJ2 = -6,  /* ... in pKF2 */
    ORBG_TRI_DIST0 = -7,    /* at a camera centre */
    ORBG_TRI_SCALE = -8     /* scale inconsistency (ratioFactor = 1.5 mfScaleFactor) */
};
/* For pairs p (KeyFrames d_kf1[p], d_kf2[p] of `kfs`: mvKeysUn, mvuRight, counts read; mvKeys
 * d_kps_raw + kf * cap for UnprojectStereo (NULL: mvKeysUn), mvDepth d_depth + kf * cap
 * (read where mvuRight >= 0; required with uright), cameras d_cams[kf]) and their
 * SearchForTriangulation output d_matches12 + p * cap: d_status[p * cap + i] (ORBG_TRI_*)
 * and d_x3d[3 (p * cap + i) ..] (the new point when NEW, else 0) for i < N of pKF1,
 * d_nnew[p] = new points.  The MapPoint creation itself (new MapPoint, AddObservation,
 * ComputeDistinctiveDescriptors, UpdateNormalAndDepth, mlpRecentAddedMapPoints) is the
 * caller's, in i order.  Scale factors / sigma^2 / mfScaleFactor are the
 * context's.  A match past pKF2's N counts as no match.  Context stream. */
int orbg_triangulate_batch_device(orbg_ctx *ctx, const orbg_keyframes *kfs,
                                  const orbg_keypoint *d_kps_raw, const float *d_depth, int cap,
                                  const orbg_kf_camera *d_cams, const int32_t *d_kf1,
                                  const int32_t *d_kf2, const int32_t *d_matches12, int npairs,
                                  float *d_x3d, int8_t *d_status, int32_t *d_nnew);
/* One KeyFrame's triangulation inputs from host arrays (kps_raw / uright may be NULL; depth
 * required with uright) */
typedef struct {
    const orbg_keypoint *kps;
    const orbg_keypoint *kps_raw;
    const float *uright;
    const float *depth;
    int32_t n;
} orbg_keyframe_geo;
/* One pair from host arrays: status[kf1->n], x3d[3 kf1->n], *nnew. */
int orbg_triangulate(orbg_ctx *ctx, const orbg_keyframe_geo *kf1, const orbg_keyframe_geo *kf2,
                     const orbg_kf_camera *cam1, const orbg_kf_camera *cam2,
                     const int32_t *matches12, float *x3d, int8_t *status, int *nnew);

/* ORBmatcher::Fuse(pKF, vpMapPoints, th) (src/ORBmatcher.cc:968-1107) splits into a search,
 * per MapPoint independent of the others (projection with pKF's pose, IsInImage, the
 * [0.8 dmin, 1.2 dmax] and 60-degree gates, PredictScale, GetFeaturesInArea(u, v, th *
 * mvScaleFactors[level]), the level window [level - 1, level], the chi-square reprojection
 * gates 5.99 / 7.8, the least descriptor distance -- the first in GetFeaturesInArea's order),
 * and the sequential map update of every point whose best distance is <= TH_LOW (Replace or
 * AddObservation, :1071-1104), which the caller applies in vpMapPoints order.
 * This is the search: best_idx[i] = the pKF feature the reference fuses point i with, -1 if
 * none; best_dist[i] = bestDist (256: no candidate).  mps[i].flags ORBG_MP_VALID = pMP &&
 * !isBad() && !IsInKeyFrame(pKF) when the call starts; cam = pKF's pose, fx.., mbf,
 * mfLogScaleFactor, mnScaleLevels and the Frame's (float) image bounds the KeyFrame's grid was
 * built with: the grid and its cell sizes use them, IsInImage and GetFeaturesInArea's cell
 * range the KeyFrame's int mnMinX .. mnMaxY, their truncation (KeyFrame.h:288-291,
 * KeyFrame.cc:51).  Scale factors / inverse sigma^2 are the context's.  One KeyFrame from host
 * arrays (kf->fv_* unused): */
int orbg_fuse(orbg_ctx *ctx, const orbg_keyframe *kf, const orbg_frustum_camera *cam,
              const orbg_map_point *mps, const uint8_t *mdesc, int nmp, float th,
              int32_t *best_idx, int32_t *best_dist, int *nfused);
/* Batched, device memory: pair p = KeyFrame d_kf[p] of `kfs` (desc, kps, uright, counts
 * read) with camera d_cams[p] and the d_mcounts[p] MapPoints at d_mps + p * mcap (descriptors
 * d_mdesc + p * mcap * 32); outputs at + p * mcap, d_nfused[p] = points with a target
 * (written even when mcap == 0: zero).  Context stream.  ORBG_ENOTSUP past 8192 keypoints per
 * KeyFrame (the grid lives in LDS). */
int orbg_fuse_batch_device(orbg_ctx *ctx, const orbg_keyframes *kfs, int cap, const int32_t *d_kf,
                           const orbg_frustum_camera *d_cams, const orbg_map_point *d_mps,
                           const uint8_t *d_mdesc, const int32_t *d_mcounts, int mcap, int npairs,
                           float th, int32_t *d_best_idx, int32_t *d_best_dist,
                           int32_t *d_nfused);
/* ORBmatcher::Fuse(pKF, Scw, vpPoints, th, vpReplacePoint) (src/ORBmatcher.cc:1133-1258;
 * caller LoopClosing::SearchAndFuse, LoopClosing.cc:944-980, th 4): the same split.  cam->Tcw
 * holds Scw's rows 0..2 (s*Rcw | s*tcw, Converter::toCvMat of the corrected g2o::Sim3); the
 * kernel decomposes it as the reference does (scw = sqrt of row 0's double dot product, Rcw |
 * tcw = Scw / scw with the float alpha 1 / scw, :1143-1148; Ow = -Rcw^T tcw), then projects
 * and gates exactly as orbg_fuse but ranks the candidates by descriptor distance alone (no
 * reprojection gate; kf->uright and cam->bf unused).  mps[i].flags ORBG_MP_VALID = !isBad() &&
 * not in pKF->GetMapPoints() at the call's start.  Outputs as orbg_fuse; the caller then
 * walks vpPoints in order: best_idx[i] >= 0 -> pKF's MapPoint at best_idx[i], if any and not
 * bad, becomes vpReplacePoint[i], else AddObservation / AddMapPoint (:1239-1254). */
int orbg_fuse_sim3(orbg_ctx *ctx, const orbg_keyframe *kf, const orbg_frustum_camera *cam,
                   const orbg_map_point *mps, const uint8_t *mdesc, int nmp, float th,
                   int32_t *best_idx, int32_t *best_dist, int *nfused);
/* Batched, device memory, as orbg_fuse_batch_device (kfs->uright may be NULL). */
int orbg_fuse_sim3_batch_device(orbg_ctx *ctx, const orbg_keyframes *kfs, int cap,
                                const int32_t *d_kf, const orbg_frustum_camera *d_cams,
                                const orbg_map_point *d_mps, const uint8_t *d_mdesc,
                                const int32_t *d_mcounts, int mcap, int npairs, float th,
                                int32_t *d_best_idx, int32_t *d_best_dist, int32_t *d_nfused);

/* ORBmatcher(0.75, checkOri).SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th,
 * ORBdist) (src/ORBmatcher.cc:1670-1798; Tracking::Relocalization, Tracking.cc:2120 th 10 /
 * ORBdist 100, :2141 th 3 / 64): the CurrentFrame side is kps / desc (mvKeysUn,
 * mDescriptors), taken0[i2] = mvpMapPoints[i2] != NULL on entry (NULL: none), cam =
 * CurrentFrame's pose, fx.., mfLogScaleFactor, mnScaleLevels and mnMinX..; pts[i] =
 * pKF->GetMapPointMatches()[i] with pKF->mvKeysUn[i].angle (flags ORBG_MP_VALID = pMP &&
 * !isBad() && !sAlreadyFound.count(pMP)).  match[i2] = the pKF index written to
 * mvpMapPoints[i2], -1 untouched, -2 set to NULL by the rotation filter. */
typedef struct {
    float x, y, z;            /* GetWorldPos() */
    float min_dist, max_dist; /* mfMinDistance, mfMaxDistance */
    float angle;              /* pKF->mvKeysUn[i].angle */
    int32_t flags;
} orbg_reloc_point;
int orbg_search_by_projection_reloc(orbg_ctx *ctx, const orbg_keypoint *kps, const uint8_t *desc,
                                    int n, const uint8_t *taken0, const orbg_frustum_camera *cam,
                                    const orbg_reloc_point *pts, const uint8_t *pdesc, int np,
                                    float th, int orb_dist, int check_ori, int32_t *match,
                                    int *nmatches);
/* ORBmatcher::SearchByProjection(pKF, Scw, vpPoints, vpMatched, th) (src/ORBmatcher.cc:
 * 353-470; LoopClosing::ComputeSim3, LoopClosing.cc:669, th 10): kps / desc = pKF's,
 * taken0[idx] = vpMatched[idx] != NULL on entry, cam->Tcw = Scw rows 0..2 (decomposed on the
 * device as orbg_fuse_sim3 does), cam->bounds the Frame's float bounds (the KeyFrame's int
 * bounds are their truncation); mps[i] = vpPoints[i] (flags ORBG_MP_VALID = !isBad() && not
 * in vpMatched on entry).  match[idx] = the vpPoints index written to vpMatched[idx], -1. */
int orbg_search_by_projection_sim3(orbg_ctx *ctx, const orbg_keypoint *kps, const uint8_t *desc,
                                   int n, const uint8_t *taken0, const orbg_frustum_camera *cam,
                                   const orbg_map_point *mps, const uint8_t *mdesc, int nm,
                                   int th, int32_t *match, int *nmatches);

/* ORBmatcher::SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th) (src/ORBmatcher.cc:
 * 1262-1470; LoopClosing::ComputeSim3, LoopClosing.cc:594, th 7.5): pKF1's map points
 * projected into pKF2 through the Sim3 and pKF2's into pKF1, each to its least-distance
 * feature (TH_HIGH), kept where the two directions agree.  kf1 / kf2: mvKeysUn, mDescriptors,
 * n (the rest unused); mp1[i] / md1 = pKF1->GetMapPointMatches()[i] (flags ORBG_MP_VALID = pMP
 * && !isBad()), likewise mp2 / md2; matched1[i] = vpMatches12[i] != NULL, matched2[idx2] = 1
 * for each such point's GetIndexInKeyFrame(pKF2) (NULL: none); g = the two poses, the Sim3,
 * pKF1's intrinsics (used both ways, as the reference does), mfLogScaleFactor,
 * mnScaleLevels and the Frame's float bounds.  matches12[i] = the pKF2 index whose MapPoint
 * becomes vpMatches12[i], -1 (slots already set keep theirs); *nfound = nFound. */
typedef struct {
    float T1w[12], T2w[12];      /* pKF1 / pKF2 GetPose() rows 0..2 */
    float R12[9], t12[3], s12;   /* the Sim3 (R12 row-major) */
    float fx, fy, cx, cy;        /* pKF1->fx .. */
    float log_scale_factor;
    int32_t nlevels;
    orbg_bounds bounds;
} orbg_sim3_pair;
int orbg_search_by_sim3(orbg_ctx *ctx, const orbg_keyframe *kf1, const orbg_map_point *mp1,
                        const uint8_t *md1, const uint8_t *matched1, const orbg_keyframe *kf2,
                        const orbg_map_point *mp2, const uint8_t *md2, const uint8_t *matched2,
                        const orbg_sim3_pair *g, float th, int32_t *matches12, int *nfound);
/* Batched, device memory: pair p = KeyFrames d_kf1[p], d_kf2[p] of `kfs` (desc, kps, counts
 * read) with d_pairs[p]; map points per KeyFrame slot at d_mps + kf * cap (descriptors
 * d_mdesc + (kf * cap) * 32); d_matched1 / d_matched2 [npairs][cap] or NULL; outputs
 * d_matches12 + p * cap, d_nfound[p].  Context stream; ORBG_ENOTSUP past 8192 keypoints. */
int orbg_search_by_sim3_batch_device(orbg_ctx *ctx, const orbg_keyframes *kfs, int cap,
                                     const int32_t *d_kf1, const int32_t *d_kf2,
                                     const orbg_sim3_pair *d_pairs, const orbg_map_point *d_mps,
                                     const uint8_t *d_mdesc, const uint8_t *d_matched1,
                                     const uint8_t *d_matched2, int npairs, float th,
                                     int32_t *d_matches12, int32_t *d_nfound);

/* ---------------- Optimizer::PoseOptimization ----------------
 * One edge per Frame keypoint with a MapPoint (index order): EdgeSE3ProjectXYZOnlyPose when
 * mvuRight[i] < 0, else EdgeStereoSE3ProjectXYZOnlyPose (Optimizer.cc:381-460). */
typedef struct {
    float obs[3];      /* kpUn.pt.x, kpUn.pt.y, mvuRight[i] */
    float xw[3];       /* pMP->GetWorldPos() */
    float inv_sigma2;  /* mvInvLevelSigma2[kpUn.octave] */
    int32_t stereo;    /* mvuRight[i] >= 0 */
} orbg_pose_edge;

typedef struct {
    float fx, fy, cx, cy, bf; /* Frame::fx, fy, cx, cy, mbf */
    float pad;
} orbg_pose_camera;

/* Optimizer::PoseOptimization(pFrame): tcw_in = pFrame->mTcw rows 0..2 (row-major 3x4).
 * Outputs the optimised SE3Quat (q x,y,z,w; t), its cv::Mat form tcw_out (SetPose), the
 * mvbOutlier flag per edge and the return value (nInitialCorrespondences - nBad) in
 * *ninliers.  Fewer than 3 edges: pose unchanged, 0. */
int orbg_pose_optimization(orbg_ctx *ctx, const orbg_pose_edge *edges, int n,
                           const orbg_pose_camera *cam, const float tcw_in[12], double q_out[4],
                           double t_out[3], float tcw_out[12], uint8_t *outlier, int *ninliers);

/* Batched, device-resident: frame f's edges at edges + f * edge_cap, counts[f] of them;
 * cams[f], tcw_in[f * 12]; outputs q_out[f * 4], t_out[f * 3], tcw_out[f * 12],
 * outlier[f * edge_cap], ninliers[f].  One workgroup per frame, on the context stream. */
int orbg_pose_optimization_batch_device(orbg_ctx *ctx, const orbg_pose_edge *edges,
                                        const int32_t *counts, int edge_cap,
                                        const orbg_pose_camera *cams, const float *tcw_in,
                                        double *q_out, double *t_out, float *tcw_out,
                                        uint8_t *outlier, int32_t *ninliers, int nframes);

/* The per-frame pose of the batched-sequence mode (SURVEY.md 8e "pose/trajectory stub"):
 * Optimizer::PoseOptimization (src/Optimizer.cc:356-631) of frame f2[p] of every pair of the
 * last orbg_match_batch_device, with that call's SearchForInitialization matches as the map
 * points: F1 keypoint i matched to F2 keypoint j gives one mono edge, obs = F2 keypoint j,
 * Xw = F1 keypoint i back-projected at `depth` in F1's camera ((x - cx) z / fx,
 * (y - cy) z / fy, z), Omega = mvInvLevelSigma2[octave of j]; edges in F2 index order (the
 * reference's loop over pFrame's keypoints); initial pose identity (F1's camera = world).
 * Outputs per pair on the match stream (device memory): d_q[4p..4p+3] the SE3Quat rotation
 * (x, y, z, w), d_t[3p..3p+2] its translation (F2's pose relative to F1) and d_ninliers[p]
 * (PoseOptimization's return value). */
int orbg_match_pose_batch_device(orbg_ctx *ctx, const orbg_pose_camera *cam, float depth,
                                 double *d_q, double *d_t, int32_t *d_ninliers);

/* ---------------- local BA linearisation ---------------- */
typedef struct {
    double q[4]; /* SE3Quat rotation, Eigen coeffs order (x, y, z, w), normalised */
    double t[3];
    int32_t fixed;
    int32_t pad;
} orbg_pose;

typedef struct {
    int32_t point;   /* vertex 0: VertexSBAPointXYZ */
    int32_t pose;    /* vertex 1: VertexSE3Expmap */
    int32_t stereo;  /* 0 EdgeSE3ProjectXYZ, 1 EdgeStereoSE3ProjectXYZ */
    int32_t robust;  /* Huber kernel attached */
    int32_t active;  /* level-0 edge */
    int32_t pad;
    double obs[3];
    double inv_sigma2;
    double fx, fy, cx, cy, bf;
    double huber_delta;
} orbg_edge;

typedef struct {
    double err[3];
    double chi2;
    double rho1;
    double jp[3][3];
    double jt[3][6];
    double hpl[3][6];
} orbg_edge_out;

/* Host arrays in, host arrays out (uploads, runs the device kernels, downloads).
 * eout may be NULL.  hpose npose*36, bpose npose*6, hpoint npoint*9, bpoint npoint*3. */
int orbg_ba_linearize(orbg_ctx *ctx, const orbg_pose *poses, int npose, const double *points,
                      int npoint, const orbg_edge *edges, int nedge, orbg_edge_out *eout,
                      double *hpose, double *bpose, double *hpoint, double *bpoint);

/* Device-resident variant (batched LBA windows): every pointer is device memory, enqueued
 * on the context stream.  pose_off[npose+1] / pose_edges[nedge] and point_off[npoint+1] /
 * point_edges[nedge] list each vertex's edges (CSR, built once per window: the graph does
 * not change across LM iterations; a point's edges in ascending edge order).  d_eout is
 * required; its hpl (and, per orbg_ba_set_edge_errors / _jacobians, the error terms and
 * Jacobians) are overwritten.  Point blocks are summed per point by one thread per point
 * over its edges; pose blocks H_pp | b_p are accumulated with MFMA f64. */
int orbg_ba_linearize_device(orbg_ctx *ctx, const orbg_pose *d_poses, int npose,
                             const double *d_points, int npoint, const orbg_edge *d_edges,
                             int nedge, const int32_t *d_pose_off, const int32_t *d_pose_edges,
                             const int32_t *d_point_off, const int32_t *d_point_edges,
                             orbg_edge_out *d_eout, double *d_hpose, double *d_bpose,
                             double *d_hpoint, double *d_bpoint);

/* buildSystem alone, for an LM iteration kept in HBM: as orbg_ba_linearize_device, but
 * H_pl goes to d_hpl[18e .. 18e+17] (edge e's 3x6 block, row-major, the _Hpl block
 * constructQuadraticForm adds, base_binary_edge.hpp:105-117) instead of the 400-byte
 * orbg_edge_out records, and no per-edge Jacobian or error term is stored (the LM's error
 * pass, orbg_ba_errors_device, provides them): per edge 144 bytes out instead of a strided
 * record.  Same blocks and the same H_pl bits as orbg_ba_linearize_device. */
int orbg_ba_build_system_device(orbg_ctx *ctx, const orbg_pose *d_poses, int npose,
                                const double *d_points, int npoint, const orbg_edge *d_edges,
                                int nedge, const int32_t *d_pose_off, const int32_t *d_pose_edges,
                                const int32_t *d_point_off, const int32_t *d_point_edges,
                                double *d_hpl, double *d_hpose, double *d_bpose,
                                double *d_hpoint, double *d_bpoint);

/* A device-resident LBA graph: the edge set of g2o's SparseOptimizer for one or many windows
 * (Optimizer.cc:662-851 builds it; optimize(5), the outlier pass and optimize(10) at
 * :857-905 rebuild the system over it every LM iteration).  Created once from host edges,
 * kept in HBM packed: 24 bytes per edge (vertices, type / robust / active flags, f32
 * observations) plus deduplicated camera and (inv_sigma2, huber_delta) tables and the
 * per-vertex edge lists, so an iteration reads a quarter of orbg_edge's bytes.  ORB-SLAM2's
 * observations are cv::KeyPoint floats: a graph needs every observation f32-exact (the mono
 * third entry is ignored), at most 256 distinct (fx, fy, cx, cy, bf) and 65536 distinct
 * (inv_sigma2, huber_delta); otherwise ORBG_ENOTSUP, and the record entry points apply.
 * Per-edge outputs (H_pl, errors) are bit-identical to orbg_ba_build_system_device /
 * orbg_ba_errors_device on the same edges.  Block sums are deterministic here: every point
 * block is summed over its edges in edge order (a point whose edges straddle two 256-edge
 * workgroups is summed by a follow-up pass, no atomics), the oracle's order; a pose block is
 * the sum over its 64-edge slices in slice order (each slice an MFMA f64 accumulation).  The
 * record entry points sum a straddling point as two partials and pose slices by fp64
 * atomics, so those blocks agree with the graph's to rounding, not bit for bit.  The graph
 * keeps its slice tables, special-point list and pose partials (built once), so a build is
 * four launches (edges, special points, pose slices, pose reduction) with no zero fills.  A graph belongs to the device of the context that
 * created it. */
typedef struct orbg_ba_graph orbg_ba_graph;
int orbg_ba_graph_create(orbg_ctx *ctx, const orbg_edge *edges, int nedge, int npose,
                         int npoint, orbg_ba_graph **out);
int orbg_ba_graph_destroy(orbg_ba_graph *graph);
/* setLevel(1) / setLevel(0) of the outlier pass (Optimizer.cc:871-901): active[e] (host,
 * 0 or 1) for every edge, in the order given at creation; ordered on the context stream
 * (uploaded from pinned staging: no host synchronisation beyond waiting for the previous
 * call's upload). */
int orbg_ba_graph_set_active(orbg_ctx *ctx, orbg_ba_graph *graph, const uint8_t *active);
/* e->setRobustKernel(0) / the Huber kernel per edge (Optimizer.cc:884, :900 remove it from
 * every edge after the outlier pass): robust[e] (host, 0 or 1), ordered like set_active. */
int orbg_ba_graph_set_robust(orbg_ctx *ctx, orbg_ba_graph *graph, const uint8_t *robust);
/* buildSystem over the graph: outputs as orbg_ba_build_system_device (d_hpl [nedge][3][6]). */
int orbg_ba_graph_build_system(orbg_ctx *ctx, orbg_ba_graph *graph, const orbg_pose *d_poses,
                               const double *d_points, double *d_hpl, double *d_hpose,
                               double *d_bpose, double *d_hpoint, double *d_bpoint);
/* computeActiveErrors over the graph: outputs as orbg_ba_errors_device. */
int orbg_ba_graph_errors(orbg_ctx *ctx, orbg_ba_graph *graph, const orbg_pose *d_poses,
                         const double *d_points, double *d_err, double *d_chi2, double *d_rho0,
                         uint8_t *d_depth_ok);
/* g2o's BlockSolver<6,3>::solve over an orbg_ba_graph, device-resident (Thirdparty/g2o/g2o/
 * core/block_solver.hpp:354-486 after setLambda, optimization_algorithm_levenberg.cpp:61-164):
 * orbg_ba_graph_schur_plan builds the Schur structure once -- free poses (`fixed`: host
 * [npose], g2o's vertex->fixed(), Optimizer.cc:714,729), the pose-pair lists of every shared
 * landmark in landmark order, the independent dense systems (one per LBA window of the
 * graph) -- and uploads it; orbg_ba_graph_set_active rebuilds it for the new active set.
 * orbg_ba_graph_schur_solve then reads the graph build's device blocks (d_hpl [nedge][3][6],
 * H_pp / b_p, H_ll / b_l) and writes the increments d_dx_pose [npose][6] (0 for fixed poses),
 * d_dx_point [npoint][3] and *d_ok (0: a zero / non-finite LDLT pivot, increments 0), in
 * stream order on the context stream with no host copy: build -> errors -> solve -> update
 * is one stream.  The Schur products run on v_mfma_f64_4x4x4f64; every sum in the order
 * oracle/ba_oracle.c orc_ba_schur_solve pins (bit-identical). */
int orbg_ba_graph_schur_plan(orbg_ctx *ctx, orbg_ba_graph *graph, const uint8_t *fixed);
int orbg_ba_graph_schur_solve(orbg_ctx *ctx, orbg_ba_graph *graph, double lambda,
                              const double *d_hpl, const double *d_hpose, const double *d_bpose,
                              const double *d_hpoint, const double *d_bpoint, double *d_dx_pose,
                              double *d_dx_point, int32_t *d_ok);
/* SparseOptimizer::update for LocalBundleAdjustment's vertex types (device memory, context
 * stream): VertexSE3Expmap::oplusImpl (types_six_dof_expmap.h:73-76: estimate =
 * SE3Quat::exp(dx) * estimate, se3quat.h:223-257; poses with `fixed` set are copied
 * unchanged) and VertexSBAPointXYZ::oplusImpl (estimate += dx).  In place when the outputs
 * are the inputs. */
int orbg_ba_update_device(orbg_ctx *ctx, const orbg_pose *d_poses, int npose,
                          const double *d_points, int npoint, const double *d_dx_pose,
                          const double *d_dx_point, orbg_pose *d_poses_out, double *d_points_out);
/* optimizer.optimize(iterations) of LocalBundleAdjustment (Optimizer.cc:857, :905) on an
 * orbg_ba_graph, OptimizationAlgorithmLevenberg::solve per iteration
 * (optimization_algorithm_levenberg.cpp:61-164: tau 1e-5, goodStep scales 1/3 and 2/3, 10
 * trials after failure, the (iniChi - chi) * 1e3 < iniChi three-strikes stop): build ->
 * Schur solve -> update -> error pass -> accept or pop, all on the context stream over the
 * estimates in HBM (d_poses / d_points, updated in place); the host reads the trial's three
 * scalars (activeRobustChi2, computeScale, the solver's ok) once per trial.  The scalars
 * are deterministic device reductions (a fixed grid-stride + tree order; g2o sums
 * sequentially).  orbg_ba_graph_schur_plan must have been called (it holds the fixed poses;
 * `fixed` of d_poses must agree); the active edges are the graph's (orbg_ba_graph_set_active).
 * report (may be NULL): iterations run, trials, chi2 before / after, the final lambda, and
 * terminated = 1 (rho == 0 or 10 failed trials) or 2 (three iterations without a 1e-3
 * relative decrease), 0 if every iteration ran. */
typedef struct {
    int32_t iterations, trials, terminated, pad;
    double initial_chi2, final_chi2, lambda;
} orbg_lm_report;
int orbg_ba_graph_optimize(orbg_ctx *ctx, orbg_ba_graph *graph, orbg_pose *d_poses,
                           double *d_points, int iterations, orbg_lm_report *report);

/* orbg_ba_graph_optimize with g2o's force-stop flag and iteration actions
 * (SparseOptimizer::setForceStopFlag(bool*), sparse_optimizer.h:184-188, installed by
 * LocalBundleAdjustment at Optimizer.cc:700-701 and raised by LocalMapping when Tracking
 * inserts a key frame; SparseOptimizer::addPostIterationAction).  Every member may be NULL:
 *   force_stop      the caller's bool (1 byte, read volatile from the host), polled where
 *                   g2o polls terminate(): before every iteration (sparse_optimizer.cpp:376)
 *                   and after every LM trial (optimization_algorithm_levenberg.cpp:149); a
 *                   raised flag ends the call after the current trial with the estimates of
 *                   that point (an accepted trial's, or the pushed state after a rejected one),
 *                   report->terminated = 3 unless the LM itself terminated;
 *   post_iteration  called after each iteration (postIteration(i), sparse_optimizer.cpp:413,
 *                   the terminating one included), on the calling thread;
 *   post_trial      called after each trial's accept / reject (before the flag is polled);
 *   d_last_chi2     device [nedge]: every edge's chi2 from the last error pass the call ran --
 *                   what g2o's edges hold after optimize() (the last trial's _error, accepted or
 *                   not; LocalBundleAdjustment's outlier tests read it, Optimizer.cc:879-901).
 *                   Not written if no iteration ran (g2o computes no error then either).
 * The hooks run on the calling thread between trials (device work may still be queued). */
typedef struct {
    const volatile uint8_t *force_stop;
    void (*post_iteration)(void *user, int iteration);
    void (*post_trial)(void *user, int iteration, int trial);
    void *user;
    double *d_last_chi2;
} orbg_lm_control;
int orbg_ba_graph_optimize_ctl(orbg_ctx *ctx, orbg_ba_graph *graph, orbg_pose *d_poses,
                               double *d_points, int iterations, const orbg_lm_control *control,
                               orbg_lm_report *report);

/* The optimisation of Optimizer::LocalBundleAdjustment (Optimizer.cc:853-935) on one window,
 * host arrays in and out, everything between on the device (the window's graph, estimates and
 * LM in HBM):
 *   optimize(5) (:856-857) with the force-stop flag (:700-701);
 *   bDoMore = the flag is clear (:859-864);
 *   if bDoMore, the outlier pass (:868-901): for every edge whose map point is not bad,
 *     setLevel(1) if chi2 > 5.991 (mono) / 7.815 (stereo) or !isDepthPositive, and
 *     setRobustKernel(0) -- chi2 as g2o's edges hold it (the last error pass of optimize(5),
 *     orbg_lm_control.d_last_chi2), the depth test at the current estimates; then
 *     optimize(10) over the level-0 edges (:904-905);
 *   the vToErase test (:907-937): erase[e] = 1 for an edge whose map point is not bad with
 *     chi2 > threshold or !isDepthPositive -- chi2 again as g2o holds it: the last error pass
 *     of optimize(10) for its active edges, optimize(5)'s for the edges it did not optimise
 *     (g2o's computeActiveErrors skips level-1 edges), the depth test at the final estimates.
 * poses [npose] / points [npoint][3] (host) are the window (build_lba_window's order) and are
 * overwritten with the optimised estimates (Optimizer.cc:949-978 reads them).  edges as
 * orbg_ba_graph_create (active / robust as given: the reference starts with every edge at
 * level 0 with a Huber kernel).  control (NULL: none): force_stop is the caller's bool* (the
 * pbStopFlag both optimize calls poll), post_iteration / post_trial run in both optimize calls
 * (iterations counted from 0 in each), d_last_chi2 is ignored.  point_is_bad
 * (NULL: never): pMP->isBad(), called on the calling thread at the two places the reference
 * calls it (the outlier pass, the vToErase test).  erase [nedge] (host, required).  The caller
 * checks the flag before calling (Optimizer.cc:853-855 returns without any write-back); a flag
 * raised before optimize(5)'s first iteration leaves chi2 at the initial estimates' (g2o has
 * none: its _error is uninitialised then). */
typedef struct {
    orbg_lm_report lm[2];  /* optimize(5), optimize(10) (zeros when not run) */
    int32_t do_more;       /* bDoMore: the outlier pass and optimize(10) ran */
    int32_t n_outliers;    /* edges the outlier pass set to level 1 */
    int32_t n_erase;       /* edges with erase[e] = 1 */
    int32_t pad;
} orbg_lba_report;
int orbg_local_ba_optimize(orbg_ctx *ctx, orbg_pose *poses, int npose, double *points,
                           int npoint, const orbg_edge *edges, int nedge,
                           const orbg_lm_control *control,
                           int (*point_is_bad)(void *user, int point), void *user,
                           uint8_t *erase, orbg_lba_report *report);

/* g2o's per-trial error pass for the two LBA edge types: SparseOptimizer::
 * computeActiveErrors (Thirdparty/g2o/g2o/core/sparse_optimizer.cpp:61-76, computeError
 * types_six_dof_expmap.h:90-95, 122-127) and the terms activeRobustChi2 sums (:100-114,
 * RobustKernelHuber::robustify robust_kernel_impl.cpp:78-91), plus isDepthPositive
 * (types_six_dof_expmap.h:97-101, 129-133) for LocalBundleAdjustment's outlier test
 * (Optimizer.cc:871-901).  The LM calls this after every trial update, buildSystem
 * (orbg_ba_linearize) once per iteration.  For every edge given, active or not:
 *   err[3e .. 3e+2] the error (third entry 0 for mono; NULL: not stored),
 *   chi2[e] = e^T Omega e, rho0[e] = Huber rho[0](chi2) if edges[e].robust else chi2 (NULL:
 *   not stored), depth_ok[e] = camera-frame depth > 0 (NULL: not stored);
 * *active_robust_chi2 (NULL: not computed) = the sum of rho0 over the active edges in the
 * order given (pass them in g2o's _activeEdges order).  Host arrays. */
int orbg_ba_errors(orbg_ctx *ctx, const orbg_pose *poses, int npose, const double *points,
                   int npoint, const orbg_edge *edges, int nedge, double *err, double *chi2,
                   double *rho0, uint8_t *depth_ok, double *active_robust_chi2);
/* Device-resident form (no sum): every pointer device memory, enqueued on the context
 * stream; d_chi2 required, d_err / d_rho0 / d_depth_ok may be NULL. */
int orbg_ba_errors_device(orbg_ctx *ctx, const orbg_pose *d_poses, const double *d_points,
                          const orbg_edge *d_edges, int nedge, double *d_err, double *d_chi2,
                          double *d_rho0, uint8_t *d_depth_ok);

/* Whether orbg_ba_linearize_device stores the per-edge Jacobians eout.jp / eout.jt (g2o's
 * _jacobianOplusXi / Xj; default on).  Off, those fields are left as they are and every
 * other output is unchanged: the blocks, H_pl and orbg_ba_schur_solve do not read them. */
int orbg_ba_set_jacobians(orbg_ctx *ctx, int enable);
/* Whether orbg_ba_linearize_device stores the per-edge error terms eout.err / chi2 / rho1
 * (default on).  Off, they are left as they are and every other output is unchanged: g2o's
 * LM takes them from the per-trial error pass instead (orbg_ba_errors / _device, which the
 * outlier test of Optimizer.cc:871-901 reads too), so buildSystem's pass writes only H_pl
 * and the blocks. */
int orbg_ba_set_edge_errors(orbg_ctx *ctx, int enable);

/* g2o BlockSolver<6,3>::solve with the Schur complement (Thirdparty/g2o/g2o/core/
 * block_solver.hpp:354-486) for one LocalBundleAdjustment window, after setLambda(lambda):
 * inputs are orbg_ba_linearize's outputs (eout[e].hpl = H_pl^T of edge e) for the same
 * poses / edges; only active edges and non-fixed poses take part.  dx_pose[npose*6] (0 for
 * fixed poses), dx_point[npoint*3] (0 for points without an active edge); *ok = the linear
 * solver's success (0: increments are zero). */
int orbg_ba_schur_solve(orbg_ctx *ctx, const orbg_pose *poses, int npose, int npoint,
                        const orbg_edge *edges, int nedge, const orbg_edge_out *eout,
                        const double *hpose, const double *bpose, const double *hpoint,
                        const double *bpoint, double lambda, double *dx_pose, double *dx_point,
                        int *ok);

/* ---------------- DBoW2 vocabulary + transform (Frame::ComputeBoW) ---------------- */
/* WeightingType / ScoringType of Thirdparty/DBoW2/DBoW2/BowVector.h:36-53 */
#define ORBG_TF_IDF 0
#define ORBG_TF 1
#define ORBG_IDF 2
#define ORBG_BINARY 3
#define ORBG_L1_NORM 0
#define ORBG_L2_NORM 1
#define ORBG_CHI_SQUARE 2
#define ORBG_KL 3
#define ORBG_BHATTACHARYYA 4
#define ORBG_DOT_PRODUCT 5

typedef struct orbg_vocab orbg_vocab;   /* device-resident vocabulary tree (one GPU) */

/* The tree exactly as loadFromTextFile builds it: node 0 is the root, nodes 1..nnodes-1 in
 * file order with parent[i] < i; children of a node in node order; is_leaf[i] > 0 gives the
 * node the next word id (leaves numbered in node order).  desc[nnodes][32], weight[nnodes]
 * (the idf of a word; ignored for the root).  k, L, scoring, weighting as in the header line
 * (0 <= k <= 20, 1 <= L <= 10, scoring 0..5, weighting 0..3).  Uploads to ctx's device. */
int orbg_vocab_create(orbg_ctx *ctx, int k, int L, int scoring, int weighting, int nnodes,
                      const int32_t *parent, const uint8_t *is_leaf, const uint8_t *desc,
                      const double *weight, orbg_vocab **out);
/* Parses the ORBvoc.txt text format ("k L scoring weighting", then one "parent isLeaf d0..d31
 * weight" line per node).  Blank lines are skipped (the reference appends an uninitialised
 * stopped node under the root for a trailing newline).  ORBG_EINVAL on a
 * malformed file. */
int orbg_vocab_load_text(orbg_ctx *ctx, const char *path, orbg_vocab **out);
void orbg_vocab_destroy(orbg_vocab *v);
/* k, L, scoring, weighting, nnodes, nwords (any pointer may be NULL) */
int orbg_vocab_info(const orbg_vocab *v, int32_t *k, int32_t *L, int32_t *scoring,
                    int32_t *weighting, int32_t *nnodes, int32_t *nwords);

/* transform(descriptors, mBowVec, mFeatVec, levelsup) for n descriptors (n x 32 bytes, host):
 *   BowVector: bow_words[*nbow] ascending word ids, bow_weights[*nbow] (normalised per the
 *   scoring), FeatureVector: fv_nodes[*nfv] ascending node ids, feature indices
 *   fv_feats[fv_off[j] .. fv_off[j+1]) ascending.  Capacities: n for bow_*, fv_nodes, fv_feats;
 *   n + 1 for fv_off.  Bit-identical to the reference (doubles included). */
int orbg_bow_transform(orbg_ctx *ctx, const orbg_vocab *v, const uint8_t *desc, int n,
                       int levelsup, int32_t *bow_words, double *bow_weights, int *nbow,
                       int32_t *fv_nodes, int32_t *fv_off, int32_t *fv_feats, int *nfv);

/* Batched, device-resident: frame f's descriptors at desc + f * cap * 32, counts[f] of them
 * (cap <= 8192); outputs per frame at bow_words / bow_weights / fv_nodes / fv_feats + f * cap,
 * fv_off + f * (cap + 1), nbow[f], nfv[f].  Also word_of[f * cap + i] (word id of feature i,
 * -1 if stopped) and node_of[...] (its levelsup node) when non-NULL. */
int orbg_bow_transform_batch_device(orbg_ctx *ctx, const orbg_vocab *v, const uint8_t *desc,
                                    const int32_t *counts, int cap, int nframes, int levelsup,
                                    int32_t *bow_words, double *bow_weights, int32_t *nbow,
                                    int32_t *fv_nodes, int32_t *fv_off, int32_t *fv_feats,
                                    int32_t *nfv, int32_t *word_of, int32_t *node_of);

/* ---------------- ORBmatcher::SearchByBoW(KeyFrame*, Frame&) ---------------- */
/* One side of SearchByBoW pairs, device memory, in orbg_bow_transform_batch_device's layout
 * (frame f's rows at + f * cap, fv_off at + f * (cap + 1)): descriptors [cap][32], keypoints
 * [cap] (only .angle is read: the KeyFrame's mvKeysUn, the Frame's mvKeys), counts[f] = N,
 * the FeatureVector (fv_nodes / fv_off / fv_feats / nfv) and, on the KeyFrame side, valid
 * [cap] = "pMP && !pMP->isBad()" of mvpMapPoints (NULL: every feature has a good MapPoint;
 * ignored on the Frame side). */
typedef struct {
    const uint8_t *desc;
    const orbg_keypoint *kps;
    const int32_t *counts;
    const int32_t *fv_nodes, *fv_off, *fv_feats, *nfv;
    const uint8_t *valid;
} orbg_bow_frames;
/* ORBmatcher::SearchByBoW(KeyFrame *pKF, Frame &F, vector<MapPoint*> &vpMapPointMatches)
 * (src/ORBmatcher.cc:195-348; Tracking::TrackReferenceKeyFrame Tracking.cc:1069,
 * Relocalization :2009) for pairs p: KeyFrame kf_index[p] of `kf`, Frame f_index[p] of `f`
 * (device int arrays; the two sides may be the same batch).  match[p * cap + i] = the KeyFrame
 * feature whose MapPoint matched F's feature i (vpMapPointMatches[i] =
 * pKF->GetMapPointMatches()[match]), -1 if NULL, for i < N of the frame; nmatch[p] = the
 * return value.  nnratio = mfNNratio, check_ori = mbCheckOrientation.  On the match stream
 * (orbg_match_stream), ordered after the context stream (as orbg_batch_summary). */
int orbg_search_by_bow_batch_device(orbg_ctx *ctx, const orbg_bow_frames *kf,
                                    const orbg_bow_frames *f, int cap, const int32_t *d_kf_index,
                                    const int32_t *d_f_index, int npairs, float nnratio,
                                    int check_ori, int32_t *d_match, int32_t *d_nmatch);
/* The same for one pair from host arrays: the KeyFrame's n_kf descriptors, mvKeysUn angles
 * (kf_angle), valid flags (NULL: all) and FeatureVector; the Frame's n_f descriptors, mvKeys
 * angles and FeatureVector.  match[n_f] as above; *nmatches = the return value. */
int orbg_search_by_bow(orbg_ctx *ctx, const uint8_t *kf_desc, const float *kf_angle,
                       const uint8_t *kf_valid, int n_kf, const int32_t *kf_fv_nodes,
                       const int32_t *kf_fv_off, const int32_t *kf_fv_feats, int kf_nfv,
                       const uint8_t *f_desc, const float *f_angle, int n_f,
                       const int32_t *f_fv_nodes, const int32_t *f_fv_off,
                       const int32_t *f_fv_feats, int f_nfv, float nnratio, int check_ori,
                       int32_t *match, int *nmatches);

/* ORBmatcher(nnratio, checkOri).SearchByBoW(KeyFrame *pKF1, KeyFrame *pKF2, vpMatches12)
 * (src/ORBmatcher.cc:634-769; LoopClosing::ComputeSim3, LoopClosing.cc:485): pKF1's features with a good MapPoint
 * (valid1 = pMP && !isBad(), NULL: all) against pKF2's of the same node with a good MapPoint
 * (valid2) not yet matched; bestDist1 < TH_LOW (strict, unlike the KeyFrame-Frame form's
 * <=), the float ratio test, the rotation histogram over mvKeysUn angles.  match12[n1] = the
 * pKF2 feature matched to pKF1's feature i (vpMatches12[i] = pKF2->GetMapPointMatches()[
 * match12[i]]), -1 if NULL; *nmatches = the return value.  Host arrays: */
int orbg_search_by_bow_kf(orbg_ctx *ctx, const uint8_t *desc1, const float *angle1,
                          const uint8_t *valid1, int n1, const int32_t *fv_nodes1,
                          const int32_t *fv_off1, const int32_t *fv_feats1, int nfv1,
                          const uint8_t *desc2, const float *angle2, const uint8_t *valid2,
                          int n2, const int32_t *fv_nodes2, const int32_t *fv_off2,
                          const int32_t *fv_feats2, int nfv2, float nnratio, int check_ori,
                          int32_t *match12, int *nmatches);
/* Batched, device memory (orbg_bow_frames layout, the .valid arrays of both sides read):
 * d_match12[p * cap + i] for i < N of pKF1 = d_kf1_index[p]; on the match stream, ordered after
 * the context stream (as orbg_search_by_bow_batch_device). */
int orbg_search_by_bow_kf_batch_device(orbg_ctx *ctx, const orbg_bow_frames *kf1,
                                       const orbg_bow_frames *kf2, int cap,
                                       const int32_t *d_kf1_index, const int32_t *d_kf2_index,
                                       int npairs, float nnratio, int check_ori,
                                       int32_t *d_match12, int32_t *d_nmatch);

#ifdef __cplusplus
}
#endif
#endif /* ORBG_H */
