// orbg_api.hip -- host side of liborbg: the C ABI (include/orbg.h), context, HBM plan
// and kernel launches.  All reference tables are computed here exactly as the
// ORBextractor ctor does (ORBextractor.cc:432-521); geometry (levels, cells, quadtree
// roots) as ComputePyramid / ComputeKeyPointsOctTree / DistributeOctTree do.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdarg>
#include <cfloat>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <array>
#include <map>
#include <vector>

#include "../../include/orbg.h"
#include "orbg_internal.h"
#include "octree_args.h"
#include "track_args.h"
#include "schur_args.h"
#include "bow_args.h"
#include "pyramid_args.h"
#include "frame_device.h"

#pragma clang fp contract(off)

namespace orbg {
__global__ void k_resize(const uint8_t *, int64_t, int, int, uint8_t *, int64_t, int, int, int,
                         const int2 *, const int2 *, int, int);
__global__ void k_octree(const OrbgGeom *, const int32_t *, const uint2 *, uint32_t *,
                         uint32_t *, uint32_t *, uint8_t *, int4 *, uint32_t *, uint16_t *,
                         int32_t *, int32_t *, int);
hipError_t launch_octree_lds(bool small, dim3 grid, size_t lds, hipStream_t st, const OrbgGeom *g,
                             const int32_t *cell_cnt, const uint2 *cell_kp, uint32_t *lvl_kp,
                             uint16_t *lvl_idx, int32_t *lvl_cnt, int32_t *err_flag, OctLdsDims D);
hipError_t octree_lds_attr(int bytes);
// fast_kernels.hip
bool fast2_pitch_ok(int p4);
__global__ void k_pyramid(PyrArgs, const OrbgGeom *, const uint4 *, const int4 *, const int4 *,
                          const uint8_t *, int64_t, int, const uint8_t *, uint8_t *, uint8_t *,
                          int);
// blur_kernels.hip
int blur2_seg();
int blur2_tw(bool tiled);
hipError_t launch_blur2(hipStream_t st, const OrbgGeom *g, const int32_t *task_base,
                        const uint8_t *img0, int64_t img_fs, int img_pitch, const uint8_t *pyr,
                        uint8_t *blur, int t_begin, int t_count, int nframes);
// fast_rows_kernels.hip
int fast_rows_wave_bytes();
hipError_t launch_fast_rows(hipStream_t st, const OrbgGeom *g, const OrbgFastTile *tiles,
                            const uint8_t *img0, int64_t img_fs, int img_pitch,
                            const uint8_t *pyr, const uint32_t *ctab, int32_t *cell_cnt,
                            uint2 *cell_kp, int nframes, int t_begin, int t_count);
hipError_t launch_fast2(int p4, size_t lds, hipStream_t st, const OrbgGeom *g,
                        const OrbgCell *cells, const uint8_t *img0, int64_t img_fs,
                        int img_pitch, const uint8_t *pyr, const uint32_t *ctab,
                        int32_t *cell_cnt, uint2 *cell_kp, uint8_t *blur, int nframes,
                        int c_begin, int c_count);
hipError_t launch_blur_border(hipStream_t st, const OrbgGeom *g, int tasks_per_frame,
                              const uint8_t *img0, int64_t img_fs, int img_pitch,
                              const uint8_t *pyr, uint8_t *blur, int l0, int l1, int nframes);
struct OrbgKeypointDev;
hipError_t launch_orient_desc(bool bfma, bool tiled, dim3 grid, hipStream_t st, const OrbgGeom *g,
                              const uint8_t *img0, int64_t img_fs, int img_pitch,
                              const uint8_t *pyr, const uint8_t *blur, const uint4 *odtab,
                              const uint32_t *lvl_kp, const uint16_t *lvl_idx,
                              const int32_t *lvl_cnt, OrbgKeypointDev *kps, uint8_t *desc,
                              int32_t *counts, uint8_t *hc_base = nullptr,
                              const int32_t *hc_err = nullptr, size_t hc_okp = 0,
                              size_t hc_ods = 0, int32_t hc_tag = 0);
// match_kernels.hip
int launch_match_pairs(hipStream_t st, hipStream_t aux, hipEvent_t evf, hipEvent_t evj,
                       const uint8_t *desc, const orbg_keypoint *kps,
                       const int32_t *counts, int frame_cap, const int32_t *d_f1,
                       const int32_t *d_f2, int npairs, orbg_bounds b, int window, float nnratio,
                       int check_ori, int32_t *knn, int32_t *m12, int32_t *nm, uint32_t *topk,
                       int32_t *topk_n, void *prof, int serial, int cap0);
int launch_undistort(hipStream_t st, const orbg_camera &cam, const orbg_keypoint *kps,
                     const int32_t *counts, int fc, int nframes, orbg_keypoint *out);
int launch_frustum(hipStream_t st, const orbg_frustum_camera *cams, const orbg_map_point *mps,
                   const int32_t *counts, int cap, int nframes, float cos_limit,
                   orbg_map_projection *out, int32_t *nvisible);
int launch_tri_match(hipStream_t st, const orbg_keyframes &K, int cap, const int32_t *kf1,
                     const int32_t *kf2, const orbg_triangulation_pair *geo, int npairs,
                     const float *scale, const float *sigma2, int nlevels, int only_stereo,
                     int check_ori, int32_t *match, int32_t *nmatch);
int launch_ba_update(hipStream_t st, const orbg_pose *poses, int npose, const double *points,
                     int npoint, const double *dxp, const double *dxq, orbg_pose *pout,
                     double *qout);
int launch_lm_reduce(hipStream_t st, int mode, int n1, int n2, double lambda, const double *a1,
                     const double *a2, const double *b1, const double *b2,
                     const BaPackedEdge *edges, double *part, double *out);
int lm_reduce_groups();
int launch_tri_geometry(hipStream_t st, const orbg_kf_camera *cams, const int32_t *kf1,
                        const int32_t *kf2, int npairs, orbg_triangulation_pair *geo);
int launch_triangulate(hipStream_t st, const orbg_keyframes &K, const orbg_keypoint *kps_raw,
                       const float *depth, int cap, const orbg_kf_camera *cams, const int32_t *kf1,
                       const int32_t *kf2, const int32_t *m12, int npairs, const float *scale,
                       const float *sigma2, int nlevels, float scale_factor, float *x3d,
                       int8_t *status, int32_t *nnew);
int launch_fuse(hipStream_t st, const orbg_keyframes &K, int cap, const int32_t *kf,
                const orbg_frustum_camera *cams, const orbg_map_point *mps, const uint8_t *mdesc,
                const int32_t *mcounts, int mcap, int npairs, float th, const float *scale,
                const float *inv_sigma2, int nlevels, int sim3, int32_t *best_idx,
                int32_t *best_dist, int32_t *nfused, int32_t *err_flag);
int launch_search_by_sim3(hipStream_t st, const orbg_keyframes &K, int cap, const int32_t *kf1,
                          const int32_t *kf2, const orbg_sim3_pair *pairs,
                          const orbg_map_point *mps, const uint8_t *mdesc,
                          const uint8_t *matched1, const uint8_t *matched2, int npairs, float th,
                          const float *scale, int nlevels, int32_t *vn, int32_t *match12,
                          int32_t *nfound, int32_t *err_flag);
int launch_rgbd(hipStream_t st, const void *depth, int u16, float factor, int w, int h,
                size_t pitch, size_t istride, const orbg_keypoint *kps,
                const orbg_keypoint *kps_un, const int32_t *counts, int fc, int nframes,
                float mbf, float *uright, float *dout);
int launch_distinctive(hipStream_t st, const uint8_t *pool, const int32_t *rows,
                       const int32_t *off, int npoints, int32_t *best, uint8_t *desc_out);
int launch_pose_opt(hipStream_t st, const orbg_pose_edge *edges, const int32_t *counts, int cap,
                    const orbg_pose_camera *cams, const float *tcw_in, double *q_out,
                    double *t_out, float *tcw_out, uint8_t *outlier, int32_t *ninliers,
                    int nframes, void *prof);
int launch_match_pose(hipStream_t st, const orbg_keypoint *kps, const int32_t *counts, int fc,
                      const int32_t *f1, const int32_t *f2, const int32_t *m12, int npairs,
                      const orbg_pose_camera &cam, float depth, const float *inv_sigma2, int nlev,
                      orbg_pose_edge *edges, int32_t *ecount, orbg_pose_camera *cams,
                      float *tcw0, float *tcw_out, uint8_t *outlier, double *q_out,
                      double *t_out, int32_t *ninliers, void *prof);
int launch_match_export(hipStream_t st, const int32_t *m12, const int32_t *f1,
                        const int32_t *counts, int frame_cap, int npairs, int32_t *out);
int launch_knn2(hipStream_t st, const uint8_t *q, int nq, const uint8_t *t, int nt, int32_t *out,
                void *prof);
int launch_init_match_single(hipStream_t st, const orbg_keypoint *k1, const uint8_t *d1, int n1,
                             const orbg_keypoint *k2, const uint8_t *d2, int n2,
                             orbg_bounds b, const float *prev, float *prev_out, int32_t *m12,
                             int32_t *nm, int window, float nnratio, int check_ori, uint32_t *topk,
                             int32_t *topk_n, void *prof, int cap);
// bow_match_kernels.hip
int launch_bow_match(hipStream_t st, const orbg_bow_frames &kf, const orbg_bow_frames &f, int cap,
                     const int32_t *kf_index, const int32_t *f_index, int npairs, float nnratio,
                     int check_ori, int32_t *match, int32_t *nmatch, bool kfkf = false);
// ba_kernels.hip
int launch_ba(hipStream_t st, const orbg_pose *poses, int npose, const double *points,
              int npoint, const orbg_edge *edges, int nedge, const int32_t *pose_off,
              const int32_t *pose_edges, const int32_t *point_off, const int32_t *point_edges,
              orbg_edge_out *eout, double *hpose, double *bpose, double *hpoint, double *bpoint,
              void *scratch, void *prof);
int launch_ba_device(hipStream_t st, const orbg_pose *poses, int npose, const double *points,
                     int npoint, const orbg_edge *edges, int nedge, const int32_t *pose_off,
                     const int32_t *pose_edges, const int32_t *point_off,
                     const int32_t *point_edges, orbg_edge_out *eout, double *hpose,
                     double *bpose, double *hpoint, double *bpoint, double *scr, void *prof,
                     bool jacobians, bool errors, double *hpl);
size_t ba_rows_bytes(int nedge, int npose);
// stereo_kernels.hip
size_t stereo_scratch_bytes(int npairs, int frame_cap);
int launch_stereo(hipStream_t st, const OrbgGeom &g, const orbg_keypoint *kps,
                  const uint8_t *desc, const int32_t *counts, const int32_t *d_left,
                  const int32_t *d_right, int npairs, const uint8_t *img0, int64_t img_fs,
                  int img_pitch, const uint8_t *pyr, float bf, float min_z, void *scratch,
                  float *uright, float *depth, int32_t *nvalid, void *prof);
size_t ba_scratch_bytes(int npose, int npoint, int nedge);
int launch_ba_errors(hipStream_t st, const orbg_pose *poses, const double *points,
                     const orbg_edge *edges, int nedge, double *err, double *chi2, double *rho0,
                     uint8_t *depth_ok, void *prof);
int launch_ba_errors_packed(hipStream_t st, const orbg_pose *poses, const double *points,
                            const BaPackedEdge *edges, const BaCam *cam, const BaInfo *info,
                            int nedge, double *err, double *chi2, double *rho0,
                            uint8_t *depth_ok, void *prof);
int launch_ba_graph(hipStream_t st, const orbg_pose *poses, int npose, const double *points,
                    int npoint, const BaPackedEdge *edges, const BaCam *cam, const BaInfo *info,
                    int nedge, const int32_t *pose_off, const int32_t *pose_edges,
                    const int32_t *point_off, const int32_t *point_edges, const BaGraphDev &gd,
                    double *hpl, double *hpose, double *bpose, double *hpoint, double *bpoint,
                    void *prof);
}  // namespace orbg

using namespace orbg;

// ---------------------------------------------------------------------------
// errors
// ---------------------------------------------------------------------------
static thread_local std::string g_err;
static int set_err(int code, const char *fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}
#define HIPCHK(x)                                                                          \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess)                                                              \
            return set_err(ORBG_EIO, "%s failed: %s (%s:%d)", #x, hipGetErrorString(e_),   \
                           __FILE__, __LINE__);                                            \
    } while (0)

extern "C" const char *orbg_last_error(void) { return g_err.c_str(); }
extern "C" int orbg_abi_version(void) { return ORBG_ABI_VERSION; }

// ---------------------------------------------------------------------------
// profiling: HIP events around every launch on the context stream
// ---------------------------------------------------------------------------
namespace orbg {
struct ProfKind {
    const char *name;
    double total_ms = 0;
    int64_t launches = 0;
};
struct Prof {
    bool on = false;
    std::vector<ProfKind> kinds;
    struct Pending {
        int kind;
        hipEvent_t a, b;
    };
    std::vector<Pending> pending;
    std::vector<hipEvent_t> pool;
    hipEvent_t get()
    {
        if (!pool.empty()) {
            hipEvent_t e = pool.back();
            pool.pop_back();
            return e;
        }
        hipEvent_t e;
        hipEventCreate(&e);
        return e;
    }
    int kind(const char *n)
    {
        for (size_t i = 0; i < kinds.size(); i++)
            if (!strcmp(kinds[i].name, n)) return (int)i;
        kinds.push_back(ProfKind{n});
        return (int)kinds.size() - 1;
    }
    void begin(hipStream_t s, const char *n, hipEvent_t *a)
    {
        if (!on) return;
        *a = get();
        hipEventRecord(*a, s);
        (void)n;
    }
    void end(hipStream_t s, const char *n, hipEvent_t a)
    {
        if (!on) return;
        hipEvent_t b = get();
        hipEventRecord(b, s);
        pending.push_back(Pending{kind(n), a, b});
    }
    void collect()
    {
        for (auto &p : pending) {
            hipEventSynchronize(p.b);
            float ms = 0;
            hipEventElapsedTime(&ms, p.a, p.b);
            kinds[p.kind].total_ms += ms;
            kinds[p.kind].launches++;
            pool.push_back(p.a);
            pool.push_back(p.b);
        }
        pending.clear();
    }
};
}  // namespace orbg

// events on `st`, the stream the kernel is launched on (a local in every caller)
// Developer what-if knob ORBG_SKIP=<names> (developer builds only, `make DEV=1` defines
// ORBG_DEV_KNOBS): launches whose profile name is listed are not issued (their consumers
// read the previous batch's buffers), so a bench run shows what a kernel costs inside the
// overlapped pipeline.  Wrong results: a production build compiles it out and orbg_create
// warns when the variable is set.
#ifdef ORBG_DEV_KNOBS
static std::atomic<int> g_extract_batches{0};  // batches issued, all contexts (ORBG_SKIP_AFTER)
static bool prof_skip(const char *name)
{
    static const char *skip = getenv("ORBG_SKIP");
    static const int after = getenv("ORBG_SKIP_AFTER") ? atoi(getenv("ORBG_SKIP_AFTER")) : 0;
    if (!skip || g_extract_batches.load() <= after) return false;
    const size_t n = strlen(name);  // whole comma-separated names ("octree" != "octree_big")
    for (const char *p = skip; (p = strstr(p, name)); p += n)
        if ((p == skip || p[-1] == ',') && (p[n] == 0 || p[n] == ',')) return true;
    return false;
}
#else
static inline bool prof_skip(const char *) { return false; }
#endif
#define PROF_LAUNCH(ctxp, name, ...)                                                       \
    do {                                                                                   \
        if (prof_skip(name)) break;                                                        \
        hipEvent_t ev_a_ = nullptr;                                                        \
        (ctxp)->prof.begin(st, name, &ev_a_);                                              \
        __VA_ARGS__;                                                                       \
        (ctxp)->prof.end(st, name, ev_a_);                                                 \
    } while (0)

// ---------------------------------------------------------------------------
// context
// ---------------------------------------------------------------------------
struct orbg_ctx {
    int device = 0;
    orbg_params p{};
    hipStream_t stream = nullptr;
    hipStream_t own_stream = nullptr;
    // second stream for independent work inside one call (blur beside FAST+quadtree, knn2
    // beside SearchForInitialization); forked from / joined into `stream` with events
    hipStream_t aux_stream = nullptr;
    // quadtree stream (high priority, its own hardware queue): the quadtree runs beside the
    // GaussianBlur, fork after the FAST cells (ev_fast), join before k_octree (ev_oct).
    // oct_mode 0: everything on the extraction stream, 1: level 0 only, 2: all levels.
    hipStream_t ostream = nullptr;
    hipEvent_t ev_fast = nullptr, ev_oct = nullptr;
    // pipelined front, level 0 (FAST cells + GaussianBlur need only the input images) on
    // `fstream` beside the pyramid (ORBG_SIDE: 0 off, 1 normal priority, 2 high)
    hipStream_t fstream = nullptr;
    int side_mode = 1;
    hipEvent_t ev_f0[2] = {nullptr, nullptr}, ev_b0[2] = {nullptr, nullptr},
               ev_pfork[2] = {nullptr, nullptr}, ev_pyr[2] = {nullptr, nullptr};
    bool blur_side = false;  // ORBG_BLUR_SIDE
    // non-pipelined batches (the single-frame drop-in): k_octree, the fallback quadtree for
    // levels past k_octree_lds' capacity, on `fstream` beside the k_octree_lds launches once
    // every level's FAST cells are written (ev_big_a: level 0 on the quadtree stream, ev_big_b:
    // levels 1.. on the extraction stream), joined before k_orient_desc (ev_big); it only scans
    // the cell counts unless a level overflows.  ORBG_BIG_SIDE=1 (off by default: the single
    // frame measured 0.26 -> 0.32-0.36 ms, the level-1.. FAST launch 15 -> 51 us behind the
    // extra stream's waits, profiles/r05q_single_ab.txt)
    bool big_side = false;
    hipEvent_t ev_big_a = nullptr, ev_big_b = nullptr, ev_big = nullptr;
    // small batches: the side blur on `fstream` right behind k_pyramid (ORBG_BLUR_Q3), joined
    // before k_orient_desc
    bool blur_q3 = false;
    bool sblur = true;  // ORBG_SBLUR=0: small batches blur on the extraction stream (A/B)
    hipEvent_t ev_sblur = nullptr;
    // ORBG_OCT_GATE (read at orbg_create, default 1): the quadtree fallback launches of a
    // pipelined batch (the split level-0 pair's second launch, k_octree) exit at once unless an
    // earlier launch of the batch flagged a level for them (d_err[3], d_err[2]); 0 = they
    // always scan (A/B, and the parity test's ungated twin)
    bool oct_gate = true;
    bool fast_blur_env = false;  // ORBG_FAST_BLUR (read at orbg_create): the fused blur plan
    bool blur_tiled_env = true;  // ORBG_BLUR_TILED (read at orbg_create; 0: row-major blur)
    bool serial = false;     // orbg_set_serial: no stream overlap (isolated kernel timing)
    // orbg_extract's single-frame hipGraphs: the whole frame (H2D of the pinned input, the
    // extraction's launches on the context and quadtree streams, k_pack_frame, D2H of the
    // packed outputs) captured once per output slot and image size, then replayed with one
    // hipGraphLaunch.  ORBG_GRAPH=1|2|3 (graph_mode below); 0, the default, launches eagerly.
    int graph_mode = 0;
    hipGraphExec_t gexec[2] = {nullptr, nullptr};
    uint64_t gkey[2] = {0, 0};   // (plan generation, w, h) the graph was captured for
    int gwarm[2] = {0, 0};       // eager frames seen for gkey_next (capture after one)
    uint64_t gkey_seen[2] = {0, 0};
    uint64_t plan_gen = 0;
    uint8_t *h_gin = nullptr, *h_gout = nullptr;  // pinned graph input / output
    size_t gin_bytes = 0, gout_bytes = 0;
    bool ba_jacobians = true;  // orbg_ba_set_jacobians
    bool ba_edge_errors = true;  // orbg_ba_set_edge_errors
    int oct_mode = 0;
    int blur0_mode = 0;  // measured: 2.013 vs 2.025 ms per 256 frames with it on
    int fast0_mode = 1;  // level-0 FAST cells on `ostream` beside the resize chain (ORBG_FAST0)
    // Pipelined batches (orbg_set_pipeline): the front of a batch (pyramid, FAST cells,
    // GaussianBlur: image work) runs on `stream`, its back (quadtree, orientation +
    // descriptors, stereo: keypoint work) on `ostream`, so the front of batch k+1 overlaps
    // the back of batch k.  The per-batch intermediates (pyramid, blur, FAST cells) alternate
    // between two slots with the outputs: ev_cells[s] / ev_front[s] = slot s's FAST cells /
    // whole front written (on `stream`), ev_back[s] = slot s's last back reader done (on
    // `ostream`); the front into slot s waits for ev_back[s].
    int pipelined = 0;
    bool last_piped = false;  // the last batch took the pipelined path (back_stream)
    // stereo summary (orbg_stereo_summary) on the match stream: ev_sback = stereo outputs
    // written (back stream), ev_ssum = the summary's reads done (match stream; the next
    // stereo batch waits for it before overwriting d_snvalid / d_spairs)
    hipEvent_t ev_sback = nullptr, ev_ssum = nullptr;
    bool ssum_pending = false;
    // caller reads of the outputs (orbg_batch_acquire / orbg_batch_release): ev_rel[s] = the
    // caller's reads of output slot s issued so far, ev_srel = of the stereo outputs; the
    // slot's next extraction / the next stereo pass waits for them
    hipEvent_t ev_rel[2] = {nullptr, nullptr}, ev_srel = nullptr;
    bool rel_pending[2] = {false, false}, srel_pending = false;
    // entry points that write caller buffers on `mstream` (orbg_batch_summary /
    // orbg_batch_matches / orbg_match_pose_batch_device / orbg_stereo_summary) first order
    // `mstream` after the work queued on the context stream so far (ev_caller): a fill the
    // caller queued there before the call can never land after liborbg's write
    hipEvent_t ev_caller = nullptr;
    hipEvent_t ev_cells[2] = {nullptr, nullptr}, ev_front[2] = {nullptr, nullptr};
    hipEvent_t ev_back[2] = {nullptr, nullptr};
    bool back_pending[2] = {false, false};
    hipEvent_t ev_fork[2] = {nullptr, nullptr}, ev_join[2] = {nullptr, nullptr};
    // Batch matching and the trajectory summary run on `mstream`, so the matching of batch k
    // overlaps the extraction of batch k+1 on `stream`.  The per-frame outputs (kps, desc,
    // counts) alternate between two slots: ev_ext[s] = slot s written (on `stream`),
    // ev_mat[s] = slot s no longer read (on `mstream`); extraction into slot s waits for
    // ev_mat[s], matching of slot s waits for ev_ext[s].
    hipStream_t mstream = nullptr;
    hipEvent_t ev_ext[2] = {nullptr, nullptr}, ev_mat[2] = {nullptr, nullptr};
    bool mat_pending[2] = {false, false};
    int slot = 0;  // slot of the last extraction
    float scale[16], inv_scale[16], sigma2[16], inv_sigma2[16];
    int32_t fpl[16], umax[16];
    // plan
    int gw = 0, gh = 0, gbatch = 0;
    OrbgGeom geom{};
    std::vector<OrbgCell> cells;
    std::vector<int32_t> tile_base;  // k_blur2 tile bases (L + 1)
    // k_fast_rows strips (fast_rows_kernels.hip): fr_ok = every level's cells fit a strip
    // (wCell <= 32); ftile_base[l] = first strip of level l (L + 1 entries); fr_mode 0 forces
    // k_fast2 (ORBG_FAST_ROWS=0, developer A/B)
    OrbgFastTile *d_ftiles = nullptr;
    std::vector<int32_t> ftile_base;
    bool fr_ok = false;
    int fr_mode = 0;  // k_fast_rows opt-in (ORBG_FAST_ROWS=1) until it beats k_fast2
    OctLdsDims oct_dims[3] = {};  // levels 0, 1.., and level 0's batch first launch (kcap 0: none)
    // device
    OrbgGeom *d_geom = nullptr;
    OrbgCell *d_cells = nullptr;
    int32_t *d_tile_base = nullptr;
    int2 *d_rtab = nullptr;
    // k_pyramid (all levels in one launch): octet / row records and band closures; pyr_ok
    // = the plan passed k_pyramid's checks (else the k_resize chain)
    uint4 *d_ptab = nullptr;
    int4 *d_ytab4 = nullptr;
    int4 *d_bands = nullptr;
    PyrArgs pyr_args{};
    bool pyr_ok = false;
    int pyr_wg = 512;  // k_pyramid workgroup size (ORBG_PYR_WG)
    uint32_t *d_ctab = nullptr;  // quadtree path-code tables (xs | ys per level)
    uint4 *d_odtab = nullptr;    // k_orient_desc IC_Angle byte tables (make_od_tab)
    uint8_t *d_img = nullptr;
    size_t img_bytes = 0;
    uint8_t *d_pack = nullptr;  // orbg_download_frame: error word, count, kps, desc
    size_t pack_bytes = 0;
    // zero-copy host block (coherent pinned, device-mapped; ORBG_ZC, default 1): k_pack_frame
    // stores orbg_download_frame's packed outputs straight into it, and the
    // SearchForInitialization host entry's inputs are read from it by one copy kernel and its
    // outputs written into it by the resolver -- kernels instead of DMA submissions, whose
    // start latency (6-9 us each) the single-frame path otherwise waits for
    uint8_t *h_zc = nullptr, *h_zc_dev = nullptr;
    size_t zc_bytes = 0;
    // orbg_extract's image in coherent host memory, pulled by k_copy16 (ORBG_IMG_PULL)
    uint8_t *h_imz = nullptr, *h_imz_dev = nullptr;
    size_t imz_bytes = 0;
    int zc_mode = -1;  // -1: read ORBG_ZC on first use
    // orbg_extract's zero-copy outputs written by k_orient_desc itself (the packed block's
    // device pointer while launch_extract runs; null otherwise)
    uint8_t *hc_dst = nullptr;
    bool hc_done = false;  // the last extraction's frame 0 is already in the packed block
    // with hc_dst: k_octree (the fallback quadtree) not launched; a level it would have taken
    // shows in the packed header's word 3 and the frame is extracted again with it
    bool skip_big = false;
    // the single-frame skip path's fallback tag (OctLdsDims::tag; 0 = off) and its counter
    int32_t oct_tag = 0;
    int32_t sf_seq = 0;
    uint8_t *d_pyr = nullptr, *d_blur = nullptr;  // = pyr_slot[slot], blur_slot[slot]
    int32_t *d_cell_cnt = nullptr;                 // = cnt_slot[slot]
    uint2 *d_cell_kp = nullptr;                    // = ckp_slot[slot]
    uint8_t *pyr_slot[2] = {nullptr, nullptr}, *blur_slot[2] = {nullptr, nullptr};
    int32_t *cnt_slot[2] = {nullptr, nullptr};
    uint2 *ckp_slot[2] = {nullptr, nullptr};
    uint32_t *d_keys = nullptr, *d_knode = nullptr, *d_act = nullptr;
    uint8_t *d_qk = nullptr;
    int4 *d_nodes = nullptr;
    uint32_t *d_lvl_kp = nullptr;
    uint16_t *d_lvl_idx = nullptr;  // slot -> winner list position (octree -> orient)
    int32_t *d_lvl_cnt = nullptr;
    orbg_keypoint *d_kps = nullptr;  // = kps_slot[slot]
    uint8_t *d_desc = nullptr;        // = desc_slot[slot]
    int32_t *d_counts = nullptr;      // = counts_slot[slot]
    orbg_keypoint *kps_slot[2] = {nullptr, nullptr};
    uint8_t *desc_slot[2] = {nullptr, nullptr};
    int32_t *counts_slot[2] = {nullptr, nullptr};
    int32_t *d_err = nullptr;
    // last batch
    const uint8_t *last_img = nullptr;
    int64_t last_fs = 0;
    int last_pitch = 0;
    int last_n = 0;
    // matching (batch)
    int32_t *d_pairs = nullptr;
    int pair_cap = 0;
    std::vector<int32_t> h_pairs;  // last uploaded (f1, f2) lists
    int32_t *d_knn = nullptr, *d_m12 = nullptr, *d_nm = nullptr;
    uint32_t *d_topk = nullptr;
    int32_t *d_topk_n = nullptr;
    int last_npairs = 0;
    // stereo (ComputeStereoMatches) of the last batch
    int32_t *d_spairs = nullptr;
    std::vector<int32_t> h_spairs;  // last uploaded (left, right) lists
    float *d_uright = nullptr, *d_depth = nullptr;
    int32_t *d_snvalid = nullptr;
    void *d_sscr = nullptr;
    int stereo_cap = 0, last_nstereo = 0;
    // single-pair / host-data scratch
    void *d_scr = nullptr;
    size_t scr_bytes = 0;
    // pinned host staging of the host-data entry points (orbg_extract, orbg_download_frame,
    // orbg_search_for_initialization): one DMA per direction instead of pageable copies
    uint8_t *h_stage = nullptr;
    size_t stage_bytes = 0;
    // tracking matchers: K-lists of the queries
    void *d_trk = nullptr;
    size_t trk_bytes = 0;
    void *d_sim3 = nullptr;  // SearchBySim3's vnMatch1 / vnMatch2 scratch
    size_t sim3_bytes = 0;
    // batched-sequence pose stub (orbg_match_pose_batch_device): edges, counts, cameras, poses
    void *d_mpose = nullptr;
    size_t mpose_bytes = 0;
    // orbg_set_camera: distorted camera of the batched-sequence mode (has_cam: k1 != 0);
    // the batch matching undistorts into d_kps_un ([kps_un_frames][frame_cap], match stream)
    bool has_cam = false;
    orbg_camera cam{};
    orbg_keypoint *d_kps_un = nullptr;
    size_t kps_un_n = 0;
    bool kps_un_valid = false;
    Prof prof;
};

extern "C" void orbg_params_default(orbg_params *p)
{
    memset(p, 0, sizeof(*p));
    p->nfeatures = 2000;
    p->scale_factor = 1.2f;
    p->nlevels = 8;
    p->ini_th_fast = 20;
    p->min_th_fast = 7;
    p->resize_mode = ORBG_RESIZE_SIMD_16_8;
    const int32_t k[7] = {18, 34, 48, 56, 48, 34, 18};
    memcpy(p->gauss_k, k, sizeof(k));
    p->brief_fma = 0;
    p->max_batch = 1;
    p->sincos_mode = ORBG_SINCOS_GLIBC;
}

static int cv_round_f(float v) { return (int)lrintf(v); }
static int cv_floor_f(float v)
{
    int i = (int)v;
    return i - (i > v);
}

// ORBextractor ctor tables, ORBextractor.cc:437-520
static void make_tables(orbg_ctx *c)
{
    const orbg_params &p = c->p;
    const double sf = (double)p.scale_factor;
    c->scale[0] = 1.0f;
    c->sigma2[0] = 1.0f;
    for (int i = 1; i < p.nlevels; i++) {
        c->scale[i] = (float)((double)c->scale[i - 1] * sf);
        c->sigma2[i] = c->scale[i] * c->scale[i];
    }
    for (int i = 0; i < p.nlevels; i++) {
        c->inv_scale[i] = 1.0f / c->scale[i];
        c->inv_sigma2[i] = 1.0f / c->sigma2[i];
    }
    const float factor = (float)(1.0f / sf);
    float desired = (float)p.nfeatures * (1 - factor) /
                    (1 - (float)pow((double)factor, (double)p.nlevels));
    int sum = 0;
    for (int l = 0; l < p.nlevels - 1; l++) {
        c->fpl[l] = cv_round_f(desired);
        sum += c->fpl[l];
        desired *= factor;
    }
    c->fpl[p.nlevels - 1] = std::max(p.nfeatures - sum, 0);
    const int vmax = cv_floor_f(ORBG_HALF_PATCH * sqrtf(2.f) / 2 + 1);
    const int vmin = (int)ceilf(ORBG_HALF_PATCH * sqrtf(2.f) / 2);
    const double hp2 = ORBG_HALF_PATCH * ORBG_HALF_PATCH;
    int v, v0;
    for (v = 0; v <= vmax; ++v) c->umax[v] = (int)lrint(sqrt(hp2 - v * v));
    for (v = ORBG_HALF_PATCH, v0 = 0; v >= vmin; --v) {
        while (c->umax[v0] == c->umax[v0 + 1]) ++v0;
        c->umax[v] = v0;
        ++v0;
    }
}

static void free_plan(orbg_ctx *c)
{
    for (hipStream_t q : {c->stream, c->mstream, c->ostream, c->aux_stream, c->fstream})
        if (q) hipStreamSynchronize(q);
    c->mat_pending[0] = c->mat_pending[1] = false;
    c->back_pending[0] = c->back_pending[1] = false;
    for (hipEvent_t e : {c->ev_rel[0], c->ev_rel[1], c->ev_srel, c->ev_ssum})
        if (e) hipEventSynchronize(e);  // caller streams may still read the outputs
    c->rel_pending[0] = c->rel_pending[1] = c->srel_pending = c->ssum_pending = false;
    void *ptrs[] = {c->d_geom, c->d_cells, c->d_ftiles, c->d_tile_base, c->d_rtab, c->d_ctab, c->d_odtab,
                    c->pyr_slot[0], c->pyr_slot[1], c->blur_slot[0], c->blur_slot[1],
                    c->cnt_slot[0], c->cnt_slot[1], c->ckp_slot[0], c->ckp_slot[1], c->d_keys, c->d_knode, c->d_act, c->d_qk,
                    c->d_nodes, c->d_lvl_kp, c->d_lvl_idx, c->d_lvl_cnt, c->kps_slot[0], c->kps_slot[1],
                    c->desc_slot[0], c->desc_slot[1], c->counts_slot[0], c->counts_slot[1],
                    c->d_knn, c->d_m12, c->d_nm, c->d_topk, c->d_topk_n, c->d_pairs,
                    c->d_spairs, c->d_uright, c->d_depth, c->d_snvalid, c->d_sscr,
                    c->d_ptab, c->d_ytab4, c->d_bands};
    for (void *q : ptrs)
        if (q) hipFree(q);
    c->d_geom = nullptr;
    c->d_cells = nullptr;
    c->d_ftiles = nullptr;
    c->ftile_base.clear();
    c->fr_ok = false;
    c->d_tile_base = nullptr;
    c->d_rtab = nullptr;
    c->d_ptab = nullptr;
    c->d_ytab4 = nullptr;
    c->d_bands = nullptr;
    c->pyr_ok = false;
    c->d_ctab = nullptr;
    c->d_odtab = nullptr;
    c->d_pyr = c->d_blur = nullptr;
    c->d_cell_cnt = nullptr;
    c->d_cell_kp = nullptr;
    for (int i = 0; i < 2; i++) {
        c->pyr_slot[i] = c->blur_slot[i] = nullptr;
        c->cnt_slot[i] = nullptr;
        c->ckp_slot[i] = nullptr;
    }
    c->d_keys = c->d_knode = c->d_act = nullptr;
    c->d_qk = nullptr;
    c->d_nodes = nullptr;
    c->d_lvl_kp = nullptr;
    c->d_lvl_idx = nullptr;
    c->d_lvl_cnt = nullptr;
    c->d_kps = nullptr;
    c->d_desc = nullptr;
    c->d_counts = nullptr;
    for (int i = 0; i < 2; i++) {
        c->kps_slot[i] = nullptr;
        c->desc_slot[i] = nullptr;
        c->counts_slot[i] = nullptr;
    }
    c->d_knn = c->d_m12 = c->d_nm = nullptr;
    c->d_topk = nullptr;
    c->d_topk_n = nullptr;
    c->d_pairs = nullptr;
    c->pair_cap = 0;
    c->d_spairs = nullptr;
    c->h_spairs.clear();
    c->d_uright = c->d_depth = nullptr;
    c->d_snvalid = nullptr;
    c->d_sscr = nullptr;
    c->stereo_cap = c->last_nstereo = 0;
    c->last_npairs = 0;
    c->last_n = 0;
    c->h_pairs.clear();
    c->gw = c->gh = c->gbatch = 0;
}

// k_orient_desc's IC_Angle byte tables, [sh 0..3][weights, ones][w 0..92]: lane w holds
// bytes 16c .. 16c+15 (c = w % 3) of patch row r = w / 3 read from sh bytes before the row
// start, i.e. column u = 16c + b - sh - 15; inside the circle (|u| <= umax[|r - 15|],
// ORBextractor.cc:92-104) the weight byte is u + 15 and the one byte 1, else both 0.
static std::vector<uint4> make_od_tab(const int32_t *umax)
{
    std::vector<uint4> t(4 * ORBG_OD_TABW * 2);
    for (int sh = 0; sh < 4; sh++)
        for (int w = 0; w < ORBG_OD_TABW; w++) {
            const int r = w / 3, cw = w % 3, v = r - ORBG_HALF_PATCH;
            const int um = umax[v < 0 ? -v : v];
            uint32_t wt[4] = {0, 0, 0, 0}, on[4] = {0, 0, 0, 0};
            for (int b = 0; b < 16; b++) {
                const int u = 16 * cw + b - sh - ORBG_HALF_PATCH;
                if (u >= -um && u <= um) {
                    wt[b >> 2] |= (uint32_t)(u + ORBG_HALF_PATCH) << (8 * (b & 3));
                    on[b >> 2] |= 1u << (8 * (b & 3));
                }
            }
            // [sh][weights | ones][w]: a wave's lanes (consecutive w) read consecutive 16-byte
            // entries, conflict-free ds_read_b128
            t[(sh * 2) * ORBG_OD_TABW + w] = make_uint4(wt[0], wt[1], wt[2], wt[3]);
            t[(sh * 2 + 1) * ORBG_OD_TABW + w] = make_uint4(on[0], on[1], on[2], on[3]);
        }
    return t;
}

template <typename T>
static int dalloc(T **p, size_t n)
{
    if (n == 0) n = 1;
    hipError_t e = hipMalloc((void **)p, n * sizeof(T));
    if (e != hipSuccess)
        return set_err(ORBG_ENOMEM, "hipMalloc(%zu bytes): %s", n * sizeof(T),
                       hipGetErrorString(e));
    return ORBG_OK;
}

// pinned host staging buffer of at least `bytes` (grown on demand)
static int stage(orbg_ctx *c, size_t bytes, uint8_t **out)
{
    if (c->stage_bytes < bytes) {
        HIPCHK(hipStreamSynchronize(c->stream));
        if (c->h_stage) hipHostFree(c->h_stage);
        c->h_stage = nullptr;
        c->stage_bytes = 0;
        const size_t nb = std::max(bytes, (size_t)1 << 20);
        if (hipHostMalloc((void **)&c->h_stage, nb, hipHostMallocDefault) != hipSuccess)
            return set_err(ORBG_ENOMEM, "hipHostMalloc(%zu bytes)", nb);
        c->stage_bytes = nb;
    }
    *out = c->h_stage;
    return ORBG_OK;
}

static bool skip_big_enabled()
{
    static const int on = [] {
        const char *e = getenv("ORBG_SKIP_BIG");
        return e ? atoi(e) : 1;
    }();
    return on != 0;
}

// the single-frame skip path's fallback note as a per-call tag in d_err[4] (no clear ahead of
// the launch); ORBG_SF_TAG=0: d_err[2] cleared by a memset ahead of every frame (A/B)
static bool sf_tag_enabled()
{
    static const int on = [] {
        const char *e = getenv("ORBG_SF_TAG");
        return e ? atoi(e) : 1;
    }();
    return on != 0;
}

// small batches: k_pyramid launched ahead of the level-0 FAST cells' cross-stream wait and
// launch, so the critical chain's first kernel is submitted first (ORBG_PYR_FIRST=0: after, A/B)
static bool pyr_first_enabled()
{
    static const int on = [] {
        const char *e = getenv("ORBG_PYR_FIRST");
        return e ? atoi(e) : 1;
    }();
    return on != 0;
}

static bool hc_enabled()
{
    static const int on = [] {
        const char *e = getenv("ORBG_HC");
        return e ? atoi(e) : 1;
    }();
    return on != 0;
}

static bool use_zc(orbg_ctx *c)
{
    if (c->zc_mode < 0) {
        const char *e = getenv("ORBG_ZC");
        c->zc_mode = e ? atoi(e) != 0 : 1;
    }
    return c->zc_mode != 0;
}

// the zero-copy block (host pointer, device pointer), grown to `bytes`; the caller has drained
// every kernel that touched it (each user ends with sync_all / a stream synchronize).  The
// image upload stays a DMA: a k_copy16 pull of the image measured no faster (14.5 against
// 16.4 us, the frame a tie; profiles/r05r_single_ab.txt)
static int zc_buf(orbg_ctx *c, size_t bytes, uint8_t **h, uint8_t **d)
{
    if (c->zc_bytes < bytes) {
        HIPCHK(hipStreamSynchronize(c->stream));
        if (c->h_zc) hipHostFree(c->h_zc);
        c->h_zc = c->h_zc_dev = nullptr;
        c->zc_bytes = 0;
        const size_t nb = std::max(bytes, (size_t)1 << 20);
        if (hipHostMalloc((void **)&c->h_zc, nb, hipHostMallocCoherent) != hipSuccess)
            return set_err(ORBG_ENOMEM, "hipHostMalloc(%zu bytes, coherent)", nb);
        if (hipHostGetDevicePointer((void **)&c->h_zc_dev, c->h_zc, 0) != hipSuccess)
            return set_err(ORBG_EIO, "hipHostGetDevicePointer");
        c->zc_bytes = nb;
    }
    *h = c->h_zc;
    *d = c->h_zc_dev;
    return ORBG_OK;
}

// the image pull block (as zc_buf; the caller has drained the stream that reads it)
static int imz_buf(orbg_ctx *c, size_t bytes, uint8_t **h, uint8_t **d)
{
    if (c->imz_bytes < bytes) {
        if (c->h_imz) hipHostFree(c->h_imz);
        c->h_imz = c->h_imz_dev = nullptr;
        c->imz_bytes = 0;
        const size_t nb = std::max(bytes, (size_t)1 << 20);
        if (hipHostMalloc((void **)&c->h_imz, nb, hipHostMallocCoherent) != hipSuccess)
            return set_err(ORBG_ENOMEM, "hipHostMalloc(%zu bytes, coherent)", nb);
        if (hipHostGetDevicePointer((void **)&c->h_imz_dev, c->h_imz, 0) != hipSuccess)
            return set_err(ORBG_EIO, "hipHostGetDevicePointer");
        c->imz_bytes = nb;
    }
    *h = c->h_imz;
    *d = c->h_imz_dev;
    return ORBG_OK;
}

// orbg_extract's image upload: 1 = pulled from coherent host memory by k_copy16 on the
// extraction stream (the first kernel of the chain then follows a kernel, not an SDMA
// completion: ~13 us of queue hand-off on the single frame's critical path, r06as), 0 = the
// staged DMA
static bool img_pull_enabled()
{
    static const int on = [] {
        const char *e = getenv("ORBG_IMG_PULL");
        return e ? atoi(e) : 1;
    }();
    return on != 0;
}

// n16 16-byte words src -> dst (a host-mapped source: one PCIe read per word)
__global__ void k_copy16(const uint4 *__restrict__ src, uint4 *__restrict__ dst, size_t n16)
{
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16;
         i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

// k_pyramid tables (pyramid_args.h) from the cv::resize coefficient tables of every level.
// Returns false when a level falls outside what the kernel assumes (scale factors near 1.2:
// an octet's source bytes within 12, one output row completing per source row, at most
// PYR_NS source rows per 8 output rows); the k_resize chain then builds the pyramid.
static bool make_pyr_tables(const OrbgGeom &G, const std::vector<int2> &rtab, int nband,
                            std::vector<uint4> &ptab, std::vector<int4> &ytab,
                            std::vector<int4> &bands, PyrArgs &A, int fuse_blur)
{
    if (G.L < 2 || G.L > 16 || nband < 1) return false;
    A = PyrArgs{};
    A.L = G.L;
    A.nband = nband;
    A.pyr_frame = G.pyr_frame;
    for (int l = 1; l < G.L; l++) {
        const OrbgLevel &L = G.lv[l], &S = G.lv[l - 1];
        PyrLevelArgs &P = A.lv[l];
        P.sw = S.w;
        P.sh = S.h;
        P.dw = L.w;
        P.dh = L.h;
        P.spitch = S.pitch;
        P.dpitch = L.pitch;
        P.src_off = l >= 2 ? S.pyr_off : 0;
        P.dst_off = L.pyr_off;
        P.noct = (L.w + PYR_COLS - 1) / PYR_COLS;
        P.ptab_off = (int)ptab.size();
        P.ytab_off = (int)ytab.size();
        if (L.pitch % 64 || S.w < 2 || S.h < 2) return false;
        const int2 *xt = rtab.data() + L.xtab_off, *yt = rtab.data() + L.ytab_off;
        P.fix_oct = P.noct;
        P.clamp_row = L.h;
        P.guard_row = L.h;
        for (int dy = L.h - 1; dy >= 0; dy--) {
            if ((yt[dy].x & 0xFFFF) == (yt[dy].x >> 16)) P.clamp_row = dy;
            if ((yt[dy].x >> 16) == S.h - 1) P.guard_row = dy;
        }
        for (int q = 0; q < P.noct; q++) {
            const int dx0 = q * PYR_COLS, sx0 = xt[dx0].x;
            uint32_t sel[PYR_COLS], cf[PYR_COLS], smask = 0;
            for (int i = 0; i < PYR_COLS; i++) {
                const int dx = dx0 + i;
                sel[i] = 0x0c0c0c0cu;  // past the level's width: zeros, never stored
                cf[i] = 0;
                if (dx >= L.w) continue;
                const int sx = xt[dx].x, sx1 = std::min(sx + 1, S.w - 1);
                const int a0 = (int)(short)(xt[dx].y & 0xFFFF), a1 = (int)(short)(xt[dx].y >> 16);
                if (a0 < 0 || a1 < 0 || a0 > 4095 || a1 > 4095) return false;
                int r0 = sx - sx0, r1 = sx1 - sx0;
                if (i >= 4) {
                    r0 -= 4;
                    r1 -= 4;
                }
                if (r0 < 0 || r1 < 0 || r0 > 7 || r1 > 7) return false;
                sel[i] = (uint32_t)r0 | 0x0cu << 8 | (uint32_t)r1 << 16 | 0x0cu << 24;
                cf[i] = (uint32_t)(a0 << 4) | (uint32_t)(a1 << 4) << 16;
                if (dx >= L.bulk_end) smask |= 1u << i;
            }
            if ((smask || dx0 + PYR_COLS > L.w) && P.fix_oct == P.noct) P.fix_oct = q;
            ptab.push_back(make_uint4((uint32_t)sx0, smask, 0, 0));
            ptab.push_back(make_uint4(sel[0], sel[1], sel[2], sel[3]));
            ptab.push_back(make_uint4(sel[4], sel[5], sel[6], sel[7]));
            ptab.push_back(make_uint4(cf[0], cf[1], cf[2], cf[3]));
            ptab.push_back(make_uint4(cf[4], cf[5], cf[6], cf[7]));
        }
        for (int dy = 0; dy < L.h; dy++) {
            const int sy0 = yt[dy].x & 0xFFFF, sy1 = yt[dy].x >> 16;
            const int b0 = (int)(short)(yt[dy].y & 0xFFFF), b1 = (int)(short)(yt[dy].y >> 16);
            if (b0 < 0 || b1 < 0 || b0 > 4095 || b1 > 4095) return false;
            if (!(sy1 == sy0 + 1 || sy1 == sy0)) return false;
            if (dy > 0 && sy1 <= (yt[dy - 1].x >> 16)) return false;  // one row per source row
            if ((yt[std::min(dy + PYR_ROWS - 1, L.h - 1)].x >> 16) - sy0 + 1 > PYR_NS) return false;
            ytab.push_back(make_int4(sy0 | sy1 << 16, b0 << 8, b1 << 8, b0 | b1 << 16));
        }
    }
    // bands: own rows split evenly per level; the rows a band computes are its own rows (with
    // the fused blur, +-3 rows: the blur of its own rows reads them, REFLECT_101 inside the
    // level) plus the source rows of what it computes one level up (top-down closure)
    A.fuse_blur = fuse_blur;
    A.w0 = G.lv[0].w;
    A.h0 = G.lv[0].h;
    A.bpitch0 = G.lv[0].pitch;
    A.blur_frame = G.blur_frame;
    A.blur_off0 = G.lv[0].blur_off;
    for (int l = 1; l < G.L; l++) A.lv[l].blur_off = G.lv[l].blur_off;
    bands.assign((size_t)nband * G.L, make_int4(0, 0, 0, 0));
    for (int b = 0; b < nband; b++) {
        bands[(size_t)b * G.L] = make_int4(0, 0, (int)((int64_t)G.lv[0].h * b / nband),
                                           (int)((int64_t)G.lv[0].h * (b + 1) / nband));
        int lo = 0, hi = 0;  // computed rows of level l + 1
        for (int l = G.L - 1; l >= 1; l--) {
            const OrbgLevel &L = G.lv[l];
            const int own_lo = (int)((int64_t)L.h * b / nband), own_hi = (int)((int64_t)L.h * (b + 1) / nband);
            int olo = own_lo, ohi = own_hi;
            if (fuse_blur && own_hi > own_lo) {
                olo = std::max(own_lo - 3, 0);
                ohi = std::min(own_hi + 3, L.h);
            }
            if (l < G.L - 1 && hi > lo) {
                const int2 *yt = rtab.data() + G.lv[l + 1].ytab_off;
                const int slo = yt[lo].x & 0xFFFF, shi = (yt[hi - 1].x >> 16) + 1;
                if (ohi > olo) {
                    olo = std::min(olo, slo);
                    ohi = std::max(ohi, shi);
                } else {
                    olo = slo;
                    ohi = shi;
                }
            }
            bands[(size_t)b * G.L + l] = make_int4(olo, ohi, own_lo, own_hi);
            lo = olo;
            hi = ohi;
        }
    }
    return true;
}

// Build the geometry for an image size and allocate HBM for `batch` frames.
#ifndef ORBG_SIDE_BLUR_B
#define ORBG_SIDE_BLUR_B 8  // batches up to this size blur on the quadtree stream (launch_extract)
#endif
#ifndef ORBG_FC2_IL
#define ORBG_FC2_IL 1  // k_fast2 LDS layout (fast_kernels.hip): score rows interleaved with the tile rows
#endif

static int plan(orbg_ctx *c, int w, int h, int batch)
{
    if (c->gw == w && c->gh == h && c->gbatch >= batch) return ORBG_OK;
    const int want_batch = std::max(batch, c->gbatch);
    free_plan(c);
    c->plan_gen++;  // captured single-frame graphs hold the old buffers
    const orbg_params &p = c->p;
    OrbgGeom G{};
    G.L = p.nlevels;
    G.w = w;
    G.h = h;
    G.ini_th = std::min(std::max(p.ini_th_fast, 0), 255);
    G.min_th = std::min(std::max(p.min_th_fast, 0), 255);
    G.brief_fma = p.brief_fma;
    G.sincos_mode = p.sincos_mode;
#ifdef ORBG_DEV_KNOBS
    G.dbg = getenv("ORBG_DBG") ? atoi(getenv("ORBG_DBG")) : 0;  // phase-stop timing knob
#else
    G.dbg = 0;
#endif
    // error-path fault injection (tests): k_octree, the fallback for levels past
    // k_octree_lds' capacity, refuses every level, so such a level overflows and the batch's
    // sticky error flag fails the next check with ORBG_ENOTSUP (never a silent short output)
    if (const char *fi = getenv("ORBG_FAULT_INJECT"))
        if (!strcmp(fi, "octree_overflow")) G.dbg = 91;
    for (int i = 0; i < 7; i++) G.gk[i] = p.gauss_k[i];
    for (int i = 0; i < 16; i++) G.umax[i] = c->umax[i];
    std::vector<OrbgCell> cells;
    std::vector<int2> rtab;
    std::vector<uint32_t> ctab;
    int cell_cap = 1;
    int lw[16], lh[16];
    for (int l = 0; l < G.L; l++) {
        lw[l] = cv_round_f((float)w * c->inv_scale[l]);
        lh[l] = cv_round_f((float)h * c->inv_scale[l]);
        if (l > 0 && lw[l - 1] == 2 * lw[l] && lh[l - 1] == 2 * lh[l])
            return set_err(ORBG_ENOTSUP, "level %d is an exact 2x downscale: cv::resize would "
                                         "switch to INTER_AREA (not restated)", l);
        if (lw[l] - 2 * ORBG_MIN_BORDER >= 4096 || lh[l] - 2 * ORBG_MIN_BORDER >= 4096)
            return set_err(ORBG_ENOTSUP, "level %d too large (%dx%d)", l, lw[l], lh[l]);
    }
    // tiled blurred levels (blur_device.h blur2_tile TILED; k_orient_desc's rBRIEF loads):
    // k_blur2 must be the only writer -- the k_pyramid blur (ORBG_PYR_BLUR) and the fused
    // FAST-cell blur (opt-in ORBG_FAST_BLUR) write row-major
    {
        const char *pb = getenv("ORBG_PYR_BLUR");
        G.blur_tiled = c->blur_tiled_env && !c->fast_blur_env && !(pb && atoi(pb) != 0);
    }
    int64_t pyr_off = 0, blur_off = 0;
    int key_off = 0, node_off = 0, out_off = 0;
    std::vector<int32_t> tile_base, blur2_base;
    int blur2_tasks = 0;
    for (int l = 0; l < G.L; l++) {
        OrbgLevel &L = G.lv[l];
        L.w = lw[l];
        L.h = lh[l];
        L.pitch = (lw[l] + 63) & ~63;
        L.max_bx = lw[l] - ORBG_EDGE_THRESHOLD + 3;
        L.max_by = lh[l] - ORBG_EDGE_THRESHOLD + 3;
        const float width = (float)(L.max_bx - ORBG_MIN_BORDER);
        const float height = (float)(L.max_by - ORBG_MIN_BORDER);
        L.ncols = (int)(width / ORBG_CELL_W);
        L.nrows = (int)(height / ORBG_CELL_W);
        if (L.ncols <= 0 || L.nrows <= 0)
            return set_err(ORBG_ENOTSUP, "level %d (%dx%d) smaller than one 30-px cell: the "
                                         "reference divides by zero", l, lw[l], lh[l]);
        L.wcell = (int)ceilf(width / L.ncols);
        L.hcell = (int)ceilf(height / L.nrows);
        L.cell_base = (int)cells.size();
        for (int i = 0; i < L.nrows; i++) {
            const float iniY = (float)(ORBG_MIN_BORDER + i * L.hcell);
            float maxY = iniY + L.hcell + 6;
            if (iniY >= L.max_by - 3) continue;
            if (maxY > L.max_by) maxY = (float)L.max_by;
            for (int j = 0; j < L.ncols; j++) {
                const float iniX = (float)(ORBG_MIN_BORDER + j * L.wcell);
                float maxX = iniX + L.wcell + 6;
                if (iniX >= L.max_bx - 6) continue;
                if (maxX > L.max_bx) maxX = (float)L.max_bx;
                OrbgCell cl{};
                cl.level = (int16_t)l;
                cl.x0 = (int16_t)(int)iniX;
                cl.y0 = (int16_t)(int)iniY;
                cl.w = (int16_t)((int)maxX - (int)iniX);
                cl.h = (int16_t)((int)maxY - (int)iniY);
                cl.ci = (int16_t)i;
                cl.cj = (int16_t)j;
                if (cl.w > ORBG_MAX_WIN || cl.h > ORBG_MAX_WIN)
                    return set_err(ORBG_ENOTSUP, "FAST window %dx%d exceeds %d", cl.w, cl.h,
                                   ORBG_MAX_WIN);
                const int rw = std::max(cl.w - 6, 0), rh = std::max(cl.h - 6, 0);
                cell_cap = std::max(cell_cap, ((rw + 1) / 2) * ((rh + 1) / 2));
                cells.push_back(cl);
            }
        }
        L.ncells = (int)cells.size() - L.cell_base;
        L.nfeat = c->fpl[l];
        const int nini = (int)roundf((float)(L.max_bx - ORBG_MIN_BORDER) /
                                     (L.max_by - ORBG_MIN_BORDER));
        if (nini <= 0 || nini > 15)  // 4-bit root index of the quadtree path code
            return set_err(ORBG_ENOTSUP, "level %d aspect gives %d quadtree roots", l, nini);
        L.nini = nini;
        L.hx = (float)(L.max_bx - ORBG_MIN_BORDER) / nini;
        // Quadtree path codes (DistributeOctTree :705-724 roots, DivideNode :539-594).
        // A candidate's child at every depth depends on x and y separately: x decides
        // left/right along the halving of its root's [x0, x1), y top/bottom along
        // [0, rootH).  code = root << 28 | digit_d << (26 - 2d), digit = right | bottom << 1.
        {
            const int wrel = L.max_bx - ORBG_MIN_BORDER, hrel = L.max_by - ORBG_MIN_BORDER;
            L.xs_off = (int)ctab.size();
            for (int x = 0; x <= wrel; x++) {
                const int r = std::min((int)((float)x / L.hx), nini - 1);
                int x0 = (int)(L.hx * (float)r), x1 = (int)(L.hx * (float)(r + 1));
                uint32_t code = (uint32_t)r << 28;
                for (int d = 0; d < 14; d++) {
                    const int xm = x0 + (int)ceilf((float)(x1 - x0) / 2);
                    if (x >= xm) {
                        code |= 1u << (26 - 2 * d);
                        x0 = xm;
                    } else {
                        x1 = xm;
                    }
                }
                ctab.push_back(code);
            }
            L.ys_off = (int)ctab.size();
            for (int y = 0; y <= hrel; y++) {
                int y0 = 0, y1 = hrel;
                uint32_t code = 0;
                for (int d = 0; d < 14; d++) {
                    const int ym = y0 + (int)ceilf((float)(y1 - y0) / 2);
                    if (y >= ym) {
                        code |= 2u << (26 - 2 * d);
                        y0 = ym;
                    } else {
                        y1 = ym;
                    }
                }
                ctab.push_back(code);
            }
        }
        L.out_cap = std::max(L.nfeat + 3, 4 * nini + 1);
        if (L.out_cap > ORBG_OCT_ALIVE)
            return set_err(ORBG_ENOTSUP, "level %d wants %d features (> %d)", l, L.nfeat,
                           ORBG_OCT_ALIVE - 3);
        L.out_off = out_off;
        out_off += L.out_cap;
        L.node_cap = 20 * (L.nfeat + 3) + 20 * nini + 64;
        if (L.node_cap > 65535) L.node_cap = 65535;
        L.node_off = node_off;
        node_off += L.node_cap;
        L.scale = c->scale[l];
        L.patch_size = (int)(ORBG_PATCH * c->scale[l]);
        if (l > 0) {
            L.pyr_off = pyr_off;
            pyr_off += (int64_t)L.pitch * L.h;
        }
        L.blur_off = blur_off;  // rows rounded up to 8: the tiled layout's footprint
        blur_off += (int64_t)L.pitch * ((L.h + 7) & ~7);
        blur2_base.push_back(blur2_tasks);  // k_blur2 (blur_kernels.hip): 244 (tiled 240) x SEG wave tiles
        const int btw = blur2_tw(G.blur_tiled != 0);
        blur2_tasks += ((L.w + btw - 1) / btw) * ((L.h + blur2_seg() - 1) / blur2_seg());
        // resize coefficient tables (cv::resize, INTER_LINEAR)
        if (l > 0) {
            const int sw = lw[l - 1], sh = lh[l - 1], dw = lw[l], dh = lh[l];
            const double inv_sx = (double)dw / sw, inv_sy = (double)dh / sh;
            const double scale_x = 1. / inv_sx, scale_y = 1. / inv_sy;
            L.xtab_off = (int)rtab.size();
            for (int dx = 0; dx < dw; dx++) {
                float fx = (float)((dx + 0.5) * scale_x - 0.5);
                int sx = cv_floor_f(fx);
                fx -= sx;
                if (sx < 0) {
                    fx = 0;
                    sx = 0;
                }
                if (sx + 1 >= sw && sx >= sw - 1) {
                    fx = 0;
                    sx = sw - 1;
                }
                const int a0 = std::min(std::max(cv_round_f((1.f - fx) * 2048), -32768), 32767);
                const int a1 = std::min(std::max(cv_round_f(fx * 2048), -32768), 32767);
                rtab.push_back(make_int2(sx, (a0 & 0xFFFF) | (a1 << 16)));
            }
            L.ytab_off = (int)rtab.size();
            for (int dy = 0; dy < dh; dy++) {
                float fy = (float)((dy + 0.5) * scale_y - 0.5);
                int sy = cv_floor_f(fy);
                fy -= sy;
                const int b0 = std::min(std::max(cv_round_f((1.f - fy) * 2048), -32768), 32767);
                const int b1 = std::min(std::max(cv_round_f(fy * 2048), -32768), 32767);
                const int sy0 = sy < 0 ? 0 : (sy < sh ? sy : sh - 1);
                const int sy1 = sy + 1 < 0 ? 0 : (sy + 1 < sh ? sy + 1 : sh - 1);
                rtab.push_back(make_int2(sy0 | (sy1 << 16), (b0 & 0xFFFF) | (b1 << 16)));
            }
            int be = 0;
            if (p.resize_mode != ORBG_RESIZE_SCALAR) {
                const int step = p.resize_mode;
                int x = 0;
                for (; x <= dw - 16; x += 16) {
                }
                for (; x < dw - step; x += step) {
                }
                be = x;
            }
            L.bulk_end = be;
            // k_resize LDS staging extent (RZ_TW x RZ_TH output tiles)
            int span = 0, rows = 0;
            for (int c0 = 0; c0 < dw; c0 += 256) {
                const int c1 = std::min(c0 + 256, dw) - 1;
                const int lo = rtab[L.xtab_off + c0].x;
                const int hi = std::min(rtab[L.xtab_off + c1].x + 1, sw - 1);
                span = std::max(span, hi - lo + 1);
            }
            for (int r0 = 0; r0 < dh; r0 += 16) {
                const int r1 = std::min(r0 + 16, dh) - 1;
                rows = std::max(rows, (rtab[L.ytab_off + r1].x >> 16) -
                                          (rtab[L.ytab_off + r0].x & 0xFFFF) + 1);
            }
            L.rz_pitch = ((span + 3 + 15) / 16) * 16;  // whole 16-byte chunks per row
            L.rz_rows = rows;
            if ((int64_t)L.rz_pitch * rows > 64 * 1024 || rows * (L.rz_pitch / 16) > 256 * ORBG_RZ_FILL)
                return set_err(ORBG_ENOTSUP, "level %d resize tile needs %d x %d staged bytes", l,
                               rows, L.rz_pitch);
        }
    }
    blur2_base.push_back(blur2_tasks);
    // d_tile_base = k_blur2 tile bases (L + 1)
    tile_base = blur2_base;
    G.ncells = (int)cells.size();
    G.cell_cap = cell_cap;
    // k_fast_rows strips: consecutive cells of one cell row, at most 8 and 256 px of region
    // (lane l owns strip pixels 4l .. 4l+3); every level needs wCell <= 32 (a cell's bits of a
    // strip row fit one funnel-shifted dword), else the plan keeps k_fast2
    std::vector<OrbgFastTile> ftiles;
    std::vector<int32_t> ftile_base;
    bool fr_ok = true;
    for (int l = 0; l < G.L && fr_ok; l++) {
        const OrbgLevel &L = G.lv[l];
        if (L.wcell > 32) fr_ok = false;
        ftile_base.push_back((int)ftiles.size());
        const int cpt = std::min(8, 256 / std::max(L.wcell, 1));
        for (int a = L.cell_base; a < L.cell_base + L.ncells && fr_ok;) {
            int b = a;
            int tw = 0;
            while (b < L.cell_base + L.ncells && b - a < cpt && cells[b].ci == cells[a].ci) {
                tw += cells[b].w - 6;
                b++;
            }
            OrbgFastTile t{};
            t.level = (int16_t)l;
            t.ncell = (int16_t)(b - a);
            t.c0 = a;
            t.x0 = cells[a].x0;
            t.y0 = cells[a].y0;
            t.h = cells[a].h;
            t.tw = (int16_t)tw;
            if (tw > 256 || cells[a].h < 7 || cells[a].h - 6 > 64) fr_ok = false;  // region rows: one path code per lane
            for (int k = a; k < b; k++)
                if (cells[k].h != cells[a].h || cells[k].y0 != cells[a].y0 ||
                    cells[k].x0 != cells[a].x0 + (k - a) * L.wcell || (k + 1 < b && cells[k].w != L.wcell + 6))
                    fr_ok = false;
            ftiles.push_back(t);
            a = b;
        }
    }
    ftile_base.push_back((int)ftiles.size());
    {
        int wmax = 0, hmax = 0;
        for (const OrbgCell &cl : cells) {
            wmax = std::max(wmax, (int)cl.w);
            hmax = std::max(hmax, (int)cl.h);
        }
        const int rg = std::max(wmax - 6 + 3, 0) / 4;
        // 4-pixel unit groups per row of the cells (bank-spread cost of the LDS pitch)
        std::vector<int> rgs;
        for (const OrbgCell &cl : cells) {
            const int r = std::max((int)cl.w - 6 + 3, 0) / 4;
            if (r > 0 && std::find(rgs.begin(), rgs.end(), r) == rgs.end()) rgs.push_back(r);
        }
        // pretest survivor lists: two of one u16 (row << 8 | group) per unit of the largest cell
        int max_units = 0;
        for (const OrbgCell &cl : cells)
            max_units = std::max(max_units, std::max((int)cl.h - 6, 0) *
                                                ((std::max((int)cl.w - 6, 0) + 3) / 4));
        // k_fast2 (fast_kernels.hip): compile-time pitch P4 >= 4 * ceil((RG + 3) / 4) (its
        // 16-byte window chunks) among the instantiated ones; layout tA (hmax rows, stride
        // 2P, the score rows in the second half of each stride) | list (2 entries per unit).
        // Preferred: the most workgroups per CU by LDS, then the bank-spread cost.
        G.fc2_p4 = 0;
        {
            // tile rows: 4 * ceil-ish((rg + 6) / 4) dwords; score rows (P4 - 2 dwords) hold rg + 2
            const int need = std::max(4 * ((rg + 3 + 3) / 4), rg + 4);
            int best_c = 1 << 30, best_wg = 0;
            for (int wd = need; wd <= 32; wd++) {
                if (!fast2_pitch_ok(wd)) continue;
                const int P2 = 4 * wd;
#if ORBG_FC2_IL
                const int wb = (2 * hmax * P2 + 4 * max_units + 2 + 15) & ~15;
#else
                const int wb = (hmax * P2 + (std::max(hmax - 6, 0) + 2) * (P2 - 8) +
                                4 * max_units + 2 + 15) & ~15;
#endif
                const int wgs = std::min(8, 163840 / (4 * wb));
                int cost = 0;
                for (int r : rgs)
                    for (int k = 0; k < 3; k++)
                        for (int h = 0; h < 64; h += 32) {  // ds_read_b32: lane groups of 32, 32 banks
                            int hist[32] = {0}, mx = 0;
                            for (int lane = h; lane < h + 32; lane++) {
                                const int b = ((lane / r) * (ORBG_FC2_IL ? 2 : 1) * wd + lane % r + k) & 31;
                                mx = std::max(mx, ++hist[b]);
                            }
                            cost += mx;
                        }
                if (wgs > best_wg || (wgs == best_wg && cost < best_c)) {
                    best_wg = wgs;
                    best_c = cost;
                    G.fc2_p4 = wd;
                }
            }
            if (G.fc2_p4) {
                const int P2 = 4 * G.fc2_p4;
#if ORBG_FC2_IL
                G.fc2_sc_off = P2;  // score rows interleaved with the tile rows
                G.fc2_list_off = 2 * hmax * P2;
#else
                G.fc2_sc_off = hmax * P2;
                G.fc2_list_off = G.fc2_sc_off + (std::max(hmax - 6, 0) + 2) * (P2 - 8);  // score rows: P2 - 8 bytes
#endif
                G.fc2_list_cap = 2 * max_units;
#if ORBG_FC2_BITMAP
                // + k_fast2's spare entry (4 bytes with the alignment), + the corner-unit bitmap
                G.fc2_wave_bytes = (G.fc2_list_off + 2 * G.fc2_list_cap + 4 +
                                    4 * ((max_units + 31) / 32) + 15) & ~15;
#else
                G.fc2_wave_bytes = (G.fc2_list_off + 2 * G.fc2_list_cap + 2 + 15) & ~15;  // + k_fast2's spare entry
#endif
#ifdef ORBG_FC2_MIN_WAVE_BYTES  // developer A/B: LDS per wave padded (caps workgroups per CU)
                G.fc2_wave_bytes = std::max(G.fc2_wave_bytes, ORBG_FC2_MIN_WAVE_BYTES);
#endif
                if (4 * G.fc2_wave_bytes > 160 * 1024) G.fc2_p4 = 0;
            }
        }
        // every cell window the reference's 30-px grid makes (< 66 x 66) fits a pitch
        if (!G.fc2_p4)
            return set_err(ORBG_ENOTSUP, "FAST cell %dx%d fits no k_fast2 LDS pitch", wmax, hmax);
    }
    // GaussianBlur fused into k_fast2 (ORBG_FAST_BLUR=1, opt-in: measured slower, r06h --
    // fast_cells 1.97 -> 2.78 ms and the border pass 1.21 ms against k_blur2's 0.71 ms per
    // 1025 frames; the step is issue-bound, the pyramid re-read it saves was overlapped
    // anyway, profiles/r06h_fast_blur_ab.txt): every level's cells tile the
    // rectangle [16, gx1) x [16, gy1) with their detection regions, so the cells blur it
    // (dword-aligned on the right: [16, bx1)) from the window tiles they stage anyway, and
    // k_blur_border blurs the rest.  Needs: the regions tile the rectangle, every blurred
    // pixel's 7 x 7 sources inside the level (no REFLECT_101 in the fused part), the tile
    // pitch holding the window bytes the last output dword reads.  Not with the k_pyramid
    // blur (ORBG_PYR_BLUR) or k_fast_rows.
    G.fast_blur = 0;
    G.bt_total = 0;
    {
        const char *pb = getenv("ORBG_PYR_BLUR");
        bool ok = c->fast_blur_env && !(pb && atoi(pb) != 0) && !(fr_ok && c->fr_mode);
        for (int l = 0; l < G.L && ok; l++) {
            OrbgLevel &L = G.lv[l];
            int gx0 = 1 << 30, gy0 = 1 << 30, gx1 = 0, gy1 = 0;
            int64_t area = 0;
            for (int k = L.cell_base; k < L.cell_base + L.ncells && ok; k++) {
                const OrbgCell &cl = cells[k];
                const int X0 = cl.x0 + 3, Y0 = cl.y0 + 3, rw = cl.w - 6, rh = cl.h - 6;
                if (rw <= 0 || rh <= 0) ok = false;
                gx0 = std::min(gx0, X0);
                gy0 = std::min(gy0, Y0);
                gx1 = std::max(gx1, X0 + rw);
                gy1 = std::max(gy1, Y0 + rh);
                area += (int64_t)rw * rh;
                const int nb = 4 * ((X0 + rw + 3) >> 2) + 3 - cl.x0;  // k_fast2 decode()
                if (16 * ((nb + 15) >> 4) > 4 * G.fc2_p4) ok = false;
            }
            if (!ok) break;
            if (area != (int64_t)(gx1 - gx0) * (gy1 - gy0)) ok = false;  // no gaps, no overlaps
            L.bx0 = (gx0 + 3) & ~3;  // each cell blurs the dwords starting in its region
            L.by0 = gy0;
            L.bx1 = (gx1 + 3) & ~3;
            L.by1 = gy1;
            if (L.bx1 + 3 > L.w || L.by1 + 3 > L.h || gx0 < 3 || gy0 < 3) ok = false;
        }
        if (ok) {
            int off = 0;
            for (int l = 0; l < G.L; l++) {
                OrbgLevel &L = G.lv[l];
                const int nqw = (L.w + 3) / 4, sm = (L.by1 - L.by0 + 7) / 8;
                L.bt_off = off;
                L.bt_cnt = ((L.by0 + 7) / 8) * nqw + ((L.h - L.by1 + 7) / 8) * nqw +
                           sm * (L.bx0 / 4) + sm * (nqw - L.bx1 / 4);
                off += L.bt_cnt;
            }
            G.bt_total = off;
            G.fast_blur = 1;
        }
    }
    if (G.fast_blur && G.blur_tiled) return set_err(ORBG_EINVAL, "fused blur with tiled levels");
    for (int l = 0; l < G.L; l++) {
        G.lv[l].key_off = key_off;
        G.lv[l].key_cap = G.lv[l].ncells * cell_cap;
        key_off += G.lv[l].key_cap;
    }
    if ((int64_t)key_off * 1 >= (1 << 24))
        return set_err(ORBG_ENOTSUP, "candidate capacity %d exceeds 2^24", key_off);
    // k_octree_lds launches: level 0 alone with room for OCT_KEY_CAP candidates (one
    // workgroup per CU, one round at B <= 256 frames); levels 1.. sized for three
    // workgroups per CU.  A level whose candidates exceed its launch's kcap goes to k_octree.
    {
        auto dims = [&](int l0, int l1, int kcap_or_budget, bool budget) {
            OctLdsDims d{};
            d.level0 = l0;
            int acap = 0, cells = 0, roots = 0;
            for (int l = l0; l < l1; l++) {
                acap = std::max(acap, G.lv[l].out_cap);
                cells = std::max(cells, G.lv[l].ncells + 1);
                roots = std::max(roots, G.lv[l].nini);
            }
            d.acap = (acap + 63) & ~63;
            d.acap2 = (std::max(d.acap, cells) + 7) & ~7;
            d.nbw = 512 * roots;
            d.uni_bytes = std::max(d.nbw * 4, 3 * d.acap * 8);
            d.tile_sort = getenv("ORBG_OD_SORT") ? atoi(getenv("ORBG_OD_SORT")) != 0 : 0;  // measured: no gain
            if (budget) {
                const int room = kcap_or_budget - d.uni_bytes - 4 * d.acap2;
                d.kcap = std::min(OCT_KEY_CAP, std::max(0, room / 7) & ~63);
            } else {
                d.kcap = kcap_or_budget;
            }
            if (d.acap > ORBG_OCT_ALIVE) d.kcap = 0;  // k_octree only
            for (int l = l0; l < l1; l++) {
                G.lv[l].oct_kcap = d.kcap;
                G.lv[l].oct_acap2 = d.acap2;
            }
            return d;
        };
        // levels 1..: 3 workgroups per CU (160 KB / 3 minus the static header); level 0: the
        // rest of a CU beside one of them (it runs concurrently on the quadtree stream), at
        // most OCT_KEY_CAP candidates
        c->oct_dims[1] = dims(1, G.L, 163840 / 3 - (int)sizeof(OctLdsHdr) - 64, true);
        // Batches (B > ORBG_SIDE_BLUR_B) split level 0 in two launches: first at two workgroups
        // per CU (room for ~9.3k candidates; one workgroup's chain of barriers leaves a CU
        // idle), then the frames past that cap at one workgroup per CU.  ORBG_OCT_L0_WPC=n sets
        // the first launch's workgroups per CU (1: no split).  dims[2] first: level 0's
        // oct_kcap (k_octree's threshold) is the second launch's.
        const int l0_wpc = getenv("ORBG_OCT_L0_WPC") ? std::max(1, atoi(getenv("ORBG_OCT_L0_WPC"))) : 2;
        c->oct_dims[2] = OctLdsDims{};
        if (l0_wpc > 1) {
            c->oct_dims[2] = dims(0, 1, 163840 / l0_wpc - (int)sizeof(OctLdsHdr) - 64, true);
            c->oct_dims[2].first = 1;
        }
        c->oct_dims[0] = dims(0, 1, 163840 - (int)oct_lds_bytes(c->oct_dims[1]) -
                                        2 * (int)sizeof(OctLdsHdr) - 128, true);
        if (c->oct_dims[2].kcap >= c->oct_dims[0].kcap) c->oct_dims[2].kcap = 0;
        for (int k = 0; k < 3; k++) {
            const size_t b = oct_lds_bytes(c->oct_dims[k]);
            if (b + sizeof(OctLdsHdr) > 160 * 1024)
                return set_err(ORBG_ENOTSUP, "k_octree_lds needs %zu LDS bytes", b);
            // the attribute is per kernel, not per context: the whole CU's room, so a later
            // context (or the split pair's smaller launch) never lowers it under another's
            if (b > 64 * 1024) HIPCHK(octree_lds_attr(160 * 1024 - (int)sizeof(OctLdsHdr)));
        }
    }
    G.keys_frame = key_off;
    G.nodes_frame = node_off;
    G.out_frame = out_off;
    G.frame_cap = out_off;
    G.pyr_frame = (pyr_off + 255) & ~(int64_t)255;
    G.blur_frame = (blur_off + 255) & ~(int64_t)255;

    const std::vector<uint4> odtab = make_od_tab(G.umax);
    const size_t B = (size_t)want_batch;
    int rc;
    if (fr_ok && (rc = dalloc(&c->d_ftiles, ftiles.size()))) {
        free_plan(c);
        return rc;
    }
    if ((rc = dalloc(&c->d_geom, 1)) || (rc = dalloc(&c->d_cells, cells.size())) ||
        (rc = dalloc(&c->d_ctab, ctab.size())) || (rc = dalloc(&c->d_odtab, odtab.size())) ||
        (rc = dalloc(&c->d_tile_base, tile_base.size())) || (rc = dalloc(&c->d_rtab, rtab.size())) ||
        (rc = dalloc(&c->pyr_slot[0], B * G.pyr_frame)) ||
        (rc = dalloc(&c->pyr_slot[1], B * G.pyr_frame)) ||
        (rc = dalloc(&c->blur_slot[0], B * G.blur_frame)) ||
        (rc = dalloc(&c->blur_slot[1], B * G.blur_frame)) ||
        (rc = dalloc(&c->cnt_slot[0], B * G.ncells)) || (rc = dalloc(&c->cnt_slot[1], B * G.ncells)) ||
        (rc = dalloc(&c->ckp_slot[0], B * G.ncells * (size_t)cell_cap)) ||
        (rc = dalloc(&c->ckp_slot[1], B * G.ncells * (size_t)cell_cap)) ||
        (rc = dalloc(&c->d_keys, B * G.keys_frame)) || (rc = dalloc(&c->d_knode, B * G.keys_frame)) ||
        (rc = dalloc(&c->d_act, 2 * B * G.keys_frame)) || (rc = dalloc(&c->d_qk, B * G.keys_frame)) ||
        (rc = dalloc(&c->d_nodes, B * G.nodes_frame)) || (rc = dalloc(&c->d_lvl_kp, B * G.out_frame)) ||
        (rc = dalloc(&c->d_lvl_idx, B * G.out_frame)) ||
        (rc = dalloc(&c->d_lvl_cnt, B * G.L)) ||
        (rc = dalloc(&c->kps_slot[0], B * G.frame_cap)) ||
        (rc = dalloc(&c->kps_slot[1], B * G.frame_cap)) ||
        (rc = dalloc(&c->desc_slot[0], B * G.frame_cap * 32)) ||
        (rc = dalloc(&c->desc_slot[1], B * G.frame_cap * 32)) ||
        (rc = dalloc(&c->counts_slot[0], B)) || (rc = dalloc(&c->counts_slot[1], B))) {
        free_plan(c);
        return rc;
    }
    // resize tables are referenced by offset: fix up pointers through offsets at launch
    HIPCHK(hipMemcpy(c->d_geom, &G, sizeof(G), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(c->d_cells, cells.data(), cells.size() * sizeof(OrbgCell),
                     hipMemcpyHostToDevice));
    if (fr_ok)
        HIPCHK(hipMemcpy(c->d_ftiles, ftiles.data(), ftiles.size() * sizeof(OrbgFastTile),
                         hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(c->d_tile_base, tile_base.data(), tile_base.size() * sizeof(int32_t),
                     hipMemcpyHostToDevice));
    if (!rtab.empty())
        HIPCHK(hipMemcpy(c->d_rtab, rtab.data(), rtab.size() * sizeof(int2),
                         hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(c->d_ctab, ctab.data(), ctab.size() * sizeof(uint32_t),
                     hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(c->d_odtab, odtab.data(), odtab.size() * sizeof(uint4),
                     hipMemcpyHostToDevice));
    {
        // k_pyramid (ORBG_PYR=0: the k_resize chain, developer A/B; ORBG_PYR_NB: bands)
        const char *e = getenv("ORBG_PYR"), *nb = getenv("ORBG_PYR_NB");
        std::vector<uint4> pt;
        std::vector<int4> yt4;
        std::vector<int4> bd;
        PyrArgs A{};
        // ORBG_PYR_BLUR (A/B): 0 k_blur2 launches, 1 every level blurred inside k_pyramid,
        // 2 levels >= 1 inside k_pyramid and level 0 by k_blur2 (beside it on the side stream)
        const char *fb = getenv("ORBG_PYR_BLUR");
        // bands per frame: 4 fill the chip at bench batches; a small batch (the single-frame
        // drop-in) takes 16, the B = 1 optimum (profiles/r04k_single_frame_nband.txt: 4 bands
        // 0.247 ms per extraction, 16 0.229, 32 0.230, 48 0.233)
        const int nb_def = want_batch <= ORBG_SIDE_BLUR_B ? 16 : 4;
        c->pyr_ok = (!e || atoi(e)) && make_pyr_tables(G, rtab, nb ? atoi(nb) : nb_def, pt, yt4, bd,
                                                       A, fb ? atoi(fb) : 0);
        if (c->pyr_ok) {
            if ((rc = dalloc(&c->d_ptab, pt.size())) || (rc = dalloc(&c->d_ytab4, yt4.size())) ||
                (rc = dalloc(&c->d_bands, bd.size()))) {
                free_plan(c);
                return rc;
            }
            HIPCHK(hipMemcpy(c->d_ptab, pt.data(), pt.size() * sizeof(uint4), hipMemcpyHostToDevice));
            HIPCHK(hipMemcpy(c->d_ytab4, yt4.data(), yt4.size() * sizeof(int4), hipMemcpyHostToDevice));
            HIPCHK(hipMemcpy(c->d_bands, bd.data(), bd.size() * sizeof(int4), hipMemcpyHostToDevice));
            c->pyr_args = A;
            const char *wg = getenv("ORBG_PYR_WG");
            c->pyr_wg = wg ? std::min(std::max(atoi(wg) / 64 * 64, 64), 1024) : 512;
        }
    }
    HIPCHK(hipMemset(c->counts_slot[0], 0, B * sizeof(int32_t)));
    HIPCHK(hipMemset(c->counts_slot[1], 0, B * sizeof(int32_t)));
    c->slot = 0;
    c->d_kps = c->kps_slot[0];
    c->d_desc = c->desc_slot[0];
    c->d_counts = c->counts_slot[0];
    c->d_pyr = c->pyr_slot[0];
    c->d_blur = c->blur_slot[0];
    c->d_cell_cnt = c->cnt_slot[0];
    c->d_cell_kp = c->ckp_slot[0];
    c->geom = G;
    c->cells = cells;
    c->tile_base = tile_base;
    c->fr_ok = fr_ok;
    c->ftile_base = fr_ok ? ftile_base : std::vector<int32_t>();
    c->gw = w;
    c->gh = h;
    c->gbatch = want_batch;
    return ORBG_OK;
}

extern "C" int orbg_create(int device, const orbg_params *p, orbg_ctx **out)
{
    if (!out) return set_err(ORBG_EINVAL, "out is NULL");
    *out = nullptr;
    orbg_params prm;
    if (p)
        prm = *p;
    else
        orbg_params_default(&prm);
    if (prm.nlevels < 1 || prm.nlevels > ORBG_MAX_LEVELS)
        return set_err(ORBG_EINVAL, "nlevels %d out of [1, %d]", prm.nlevels, ORBG_MAX_LEVELS);
    if (!(prm.scale_factor > 1.0f))
        return set_err(ORBG_EINVAL, "scale_factor must be > 1");
    if (prm.nfeatures < 0) return set_err(ORBG_EINVAL, "nfeatures < 0");
    if (prm.resize_mode != ORBG_RESIZE_SCALAR && prm.resize_mode != ORBG_RESIZE_SSE2_16_4 &&
        prm.resize_mode != ORBG_RESIZE_SIMD_16_8)
        return set_err(ORBG_EINVAL, "resize_mode %d", prm.resize_mode);
    int ksum = 0;
    for (int i = 0; i < 7; i++) {
        if (prm.gauss_k[i] < 0) return set_err(ORBG_EINVAL, "gauss_k[%d] < 0", i);
        ksum += prm.gauss_k[i];
    }
    // 16-bit row sums in k_blur2's packed row pairs: sum(k) * 255 must fit (both OpenCV
    // tables: 256, 257)
    if (ksum > 257) return set_err(ORBG_EINVAL, "gauss_k sums to %d (> 257)", ksum);
    if (ksum == 0) {
        const int32_t k[7] = {18, 34, 48, 56, 48, 34, 18};
        memcpy(prm.gauss_k, k, sizeof(k));
    }
    if (prm.max_batch < 1) prm.max_batch = 1;
    if (prm.sincos_mode != ORBG_SINCOS_GLIBC && prm.sincos_mode != ORBG_SINCOS_PINNED)
        return set_err(ORBG_EINVAL, "sincos_mode %d", prm.sincos_mode);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return set_err(ORBG_EIO, "no HIP device visible (liborbg has no CPU fallback)");
    if (device < 0 || device >= ndev) return set_err(ORBG_EINVAL, "device %d of %d", device, ndev);
    HIPCHK(hipSetDevice(device));
    orbg_ctx *c = new orbg_ctx();
    c->device = device;
    c->p = prm;
    make_tables(c);
    if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return set_err(ORBG_EIO, "hipStreamCreate failed");
    }
    c->stream = c->own_stream;
    // sticky device error word {flags, first failing frame / pair}: OR of every launch since
    // it was last read (check_err), so a pipelined caller cannot lose an overflow.  It lives
    // as long as the context (a new extraction plan keeps pending flags), and every kernel
    // that may raise a flag -- the quadtree's and the device matchers' -- can write it.
    // Word [2] is not an error: k_octree_lds sets it when it leaves a level to k_octree, which
    // the pipelined batch's k_octree gate (and the single-frame path under ORBG_SF_TAG=0) reads.
    // Word [4]: the same note as a per-call tag (the single-frame path, OctLdsDims::tag).
    {
        const int32_t e0[8] = {0, INT32_MAX, 0, 0, 0, 0, 0, 0};
        if (hipMalloc(&c->d_err, sizeof(e0)) != hipSuccess ||
            hipMemcpy(c->d_err, e0, sizeof(e0), hipMemcpyHostToDevice) != hipSuccess) {
            if (c->d_err) hipFree(c->d_err);
            hipStreamDestroy(c->own_stream);
            delete c;
            return set_err(ORBG_ENOMEM, "device error word");
        }
    }
    // The matching streams run at low priority: a stream of another priority gets its own
    // hardware queue (at normal priority it can share one with the caller's stream and then
    // runs strictly after it), and the dispatcher hands the matching kernels the slots the
    // extraction leaves free (quadtree, kernel tails).  Measured: extract + match per 256
    // frames 2.24 -> 2.13 ms.  Developer A/B: ORBG_MATCH_PRIO=normal|high.
    int prio_lo = 0, prio_hi = 0;
    hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
    int mprio = prio_lo;
    if (const char *e = getenv("ORBG_MATCH_PRIO")) {
        if (!strcmp(e, "normal")) mprio = 0;
        if (!strcmp(e, "high")) mprio = prio_hi;
    }
    if (hipStreamCreateWithPriority(&c->aux_stream, hipStreamNonBlocking, mprio) != hipSuccess) {
        hipStreamDestroy(c->own_stream);
        delete c;
        return set_err(ORBG_EIO, "hipStreamCreate failed");
    }
    {
        const char *e = getenv("ORBG_OCT_STREAM");
        c->oct_mode = e ? atoi(e) : 1;
        const char *f0 = getenv("ORBG_FAST0");
        c->fast0_mode = f0 ? atoi(f0) : 1;
        const char *gm = getenv("ORBG_GRAPH");
        c->graph_mode = gm ? atoi(gm) : 0;
        const char *b0 = getenv("ORBG_BLUR0");
        c->blur0_mode = b0 ? atoi(b0) : 0;
        const char *bp = getenv("ORBG_BACK_PRIO");  // developer A/B: normal | high (default)
        const int oprio = (bp && !strcmp(bp, "normal")) ? 0 : prio_hi;
        if (c->oct_mode &&
            hipStreamCreateWithPriority(&c->ostream, hipStreamNonBlocking, oprio) == hipSuccess) {
            hipEventCreateWithFlags(&c->ev_fast, hipEventDisableTiming);
            hipEventCreateWithFlags(&c->ev_oct, hipEventDisableTiming);
        } else {
            c->ostream = nullptr;
            c->oct_mode = 0;
        }
    }
    {
        const char *e = getenv("ORBG_SIDE");
        c->side_mode = e ? atoi(e) : 1;  // normal priority: 1.596 vs 1.605 ms (high) after k_blur2
        if (c->side_mode && hipStreamCreateWithPriority(&c->fstream, hipStreamNonBlocking,
                                                        c->side_mode >= 2 ? prio_hi : 0) != hipSuccess) {
            c->fstream = nullptr;
            c->side_mode = 0;
        }
        for (int i = 0; i < 2; i++) {
            hipEventCreateWithFlags(&c->ev_f0[i], hipEventDisableTiming);
            hipEventCreateWithFlags(&c->ev_b0[i], hipEventDisableTiming);
            hipEventCreateWithFlags(&c->ev_pfork[i], hipEventDisableTiming);
            hipEventCreateWithFlags(&c->ev_pyr[i], hipEventDisableTiming);
        }
        const char *bs = getenv("ORBG_BLUR_SIDE");
        c->blur_side = bs ? atoi(bs) != 0 : false;
        const char *og = getenv("ORBG_OCT_GATE");
        c->oct_gate = !og || atoi(og) != 0;
        const char *fb = getenv("ORBG_FAST_BLUR");
        c->fast_blur_env = fb && atoi(fb) != 0;
        const char *bt = getenv("ORBG_BLUR_TILED");
        c->blur_tiled_env = !bt || atoi(bt) != 0;
        const char *sb = getenv("ORBG_SBLUR");
        c->sblur = !sb || atoi(sb) != 0;
        const char *bq = getenv("ORBG_BLUR_Q3");
        // off: 0.240 against 0.229 ms p50 single frame (r06av: a fourth busy stream past the
        // four hardware queues shares one with another stream)
        c->blur_q3 = c->fstream && (bq ? atoi(bq) != 0 : false) &&
                     hipEventCreateWithFlags(&c->ev_sblur, hipEventDisableTiming) == hipSuccess;
        const char *bg = getenv("ORBG_BIG_SIDE");
        c->big_side = c->fstream && (bg ? atoi(bg) != 0 : false);
        if (c->big_side)
            for (hipEvent_t *e : {&c->ev_big_a, &c->ev_big_b, &c->ev_big})
                if (hipEventCreateWithFlags(e, hipEventDisableTiming) != hipSuccess) c->big_side = false;
    }
    if (hipStreamCreateWithPriority(&c->mstream, hipStreamNonBlocking, mprio) != hipSuccess) {
        hipStreamDestroy(c->aux_stream);
        hipStreamDestroy(c->own_stream);
        delete c;
        return set_err(ORBG_EIO, "hipStreamCreate failed");
    }
    for (int i = 0; i < 2; i++) {
        hipEventCreateWithFlags(&c->ev_fork[i], hipEventDisableTiming);
        hipEventCreateWithFlags(&c->ev_join[i], hipEventDisableTiming);
        hipEventCreateWithFlags(&c->ev_ext[i], hipEventDisableTiming);
        hipEventCreateWithFlags(&c->ev_mat[i], hipEventDisableTiming);
        hipEventCreateWithFlags(&c->ev_cells[i], hipEventDisableTiming);
        hipEventCreateWithFlags(&c->ev_front[i], hipEventDisableTiming);
        hipEventCreateWithFlags(&c->ev_back[i], hipEventDisableTiming);
    }
    hipEventCreateWithFlags(&c->ev_sback, hipEventDisableTiming);
    hipEventCreateWithFlags(&c->ev_ssum, hipEventDisableTiming);
    hipEventCreateWithFlags(&c->ev_rel[0], hipEventDisableTiming);
    hipEventCreateWithFlags(&c->ev_rel[1], hipEventDisableTiming);
    hipEventCreateWithFlags(&c->ev_srel, hipEventDisableTiming);
    hipEventCreateWithFlags(&c->ev_caller, hipEventDisableTiming);
    if (const char *e = getenv("ORBG_PIPELINE")) c->pipelined = atoi(e) && c->ostream;
    if (const char *e = getenv("ORBG_FAST_ROWS")) c->fr_mode = atoi(e);
#ifdef ORBG_DEV_KNOBS
    if (getenv("ORBG_SKIP") || getenv("ORBG_DBG"))
        fprintf(stderr, "liborbg (developer build): ORBG_SKIP / ORBG_DBG set -- launches are "
                        "skipped or cut short, outputs are WRONG\n");
#else
    if (getenv("ORBG_SKIP") || getenv("ORBG_DBG"))
        fprintf(stderr, "liborbg: ORBG_SKIP / ORBG_DBG ignored (developer builds only, make "
                        "DEV=1)\n");
#endif
    if (const char *fi = getenv("ORBG_FAULT_INJECT"))
        fprintf(stderr, "liborbg: ORBG_FAULT_INJECT=%s set -- %s\n", fi,
                strcmp(fi, "octree_overflow") ? "unknown value, ignored"
                                              : "every quadtree level overflows, extractions fail "
                                                "with ORBG_ENOTSUP (error-path tests only)");
    *out = c;
    return ORBG_OK;
}

extern "C" void orbg_destroy(orbg_ctx *c)
{
    if (c && c->h_stage) hipHostFree(c->h_stage);
    if (!c) return;
    for (int i = 0; i < 2; i++)
        if (c->gexec[i]) hipGraphExecDestroy(c->gexec[i]);
    if (c->h_gin) hipHostFree(c->h_gin);
    if (c->h_gout) hipHostFree(c->h_gout);
    hipSetDevice(c->device);
    if (c->stream) hipStreamSynchronize(c->stream);
    c->prof.collect();
    for (hipEvent_t e : c->prof.pool) hipEventDestroy(e);
    free_plan(c);
    if (c->d_img) hipFree(c->d_img);
    if (c->d_pack) hipFree(c->d_pack);
    if (c->h_imz) hipHostFree(c->h_imz);
    if (c->h_zc) hipHostFree(c->h_zc);
    if (c->d_scr) hipFree(c->d_scr);
    if (c->d_trk) hipFree(c->d_trk);
    if (c->d_sim3) hipFree(c->d_sim3);
    if (c->d_err) hipFree(c->d_err);
    if (c->d_mpose) hipFree(c->d_mpose);
    if (c->d_kps_un) hipFree(c->d_kps_un);
    if (c->aux_stream) hipStreamSynchronize(c->aux_stream);
    if (c->ostream) hipStreamSynchronize(c->ostream);
    if (c->mstream) hipStreamSynchronize(c->mstream);
    for (int i = 0; i < 2; i++) {
        if (c->ev_fork[i]) hipEventDestroy(c->ev_fork[i]);
        if (c->ev_join[i]) hipEventDestroy(c->ev_join[i]);
        if (c->ev_ext[i]) hipEventDestroy(c->ev_ext[i]);
        if (c->ev_mat[i]) hipEventDestroy(c->ev_mat[i]);
        if (c->ev_cells[i]) hipEventDestroy(c->ev_cells[i]);
        if (c->ev_front[i]) hipEventDestroy(c->ev_front[i]);
        if (c->ev_back[i]) hipEventDestroy(c->ev_back[i]);
    }
    if (c->aux_stream) hipStreamDestroy(c->aux_stream);
    if (c->ostream) hipStreamDestroy(c->ostream);
    for (int i = 0; i < 2; i++)
        for (hipEvent_t e : {c->ev_f0[i], c->ev_b0[i], c->ev_pfork[i], c->ev_pyr[i]})
            if (e) hipEventDestroy(e);
    if (c->fstream) hipStreamDestroy(c->fstream);
    if (c->ev_sblur) hipEventDestroy(c->ev_sblur);
    for (hipEvent_t e : {c->ev_big_a, c->ev_big_b, c->ev_big})
        if (e) hipEventDestroy(e);
    if (c->ev_fast) hipEventDestroy(c->ev_fast);
    if (c->ev_oct) hipEventDestroy(c->ev_oct);
    for (hipEvent_t e : {c->ev_sback, c->ev_ssum, c->ev_rel[0], c->ev_rel[1], c->ev_srel,
                         c->ev_caller})
        if (e) hipEventDestroy(e);
    if (c->mstream) hipStreamDestroy(c->mstream);
    if (c->own_stream) hipStreamDestroy(c->own_stream);
    delete c;
}

extern "C" int orbg_get_scale_tables(const orbg_ctx *c, int32_t *nlevels, float *scale_factor,
                                     float *scale, float *inv_scale, float *sigma2,
                                     float *inv_sigma2, int32_t *fpl, int32_t *umax)
{
    if (!c) return set_err(ORBG_EINVAL, "ctx is NULL");
    const int L = c->p.nlevels;
    if (nlevels) *nlevels = L;
    if (scale_factor) *scale_factor = c->p.scale_factor;
    for (int i = 0; i < L; i++) {
        if (scale) scale[i] = c->scale[i];
        if (inv_scale) inv_scale[i] = c->inv_scale[i];
        if (sigma2) sigma2[i] = c->sigma2[i];
        if (inv_sigma2) inv_sigma2[i] = c->inv_sigma2[i];
        if (fpl) fpl[i] = c->fpl[i];
    }
    if (umax)
        for (int i = 0; i < 16; i++) umax[i] = c->umax[i];
    return ORBG_OK;
}

extern "C" int orbg_get_pattern(int32_t out[1024])
{
    static const int8_t pat[1024] = {
#define ORBG_PAIR(a, b, c, d) a, b, c, d,
#include "orb_pattern.inc"
#undef ORBG_PAIR
    };
    for (int i = 0; i < 1024; i++) out[i] = pat[i];
    return ORBG_OK;
}

// ---------------------------------------------------------------------------
// extraction
// ---------------------------------------------------------------------------
// ComputePyramid for B frames on `st`: k_pyramid (one launch, every level) when the plan
// passed its checks, else the k_resize chain (one launch per level)
static hipError_t launch_pyramid(orbg_ctx *c, hipStream_t st, const uint8_t *d_imgs, int B,
                                 int pitch, int64_t fs)
{
    const OrbgGeom &G = c->geom;
    if (G.L < 2) return hipSuccess;
    if (c->pyr_ok) {
        const OrbgLevel &L0 = G.lv[0];
        const uint8_t *img_end = d_imgs + (int64_t)(B - 1) * fs + (int64_t)(L0.h - 1) * pitch + L0.w;
        PROF_LAUNCH(c, "resize",
                    hipLaunchKernelGGL(k_pyramid, dim3(c->pyr_args.nband * B), dim3(c->pyr_wg), 0, st,
                                       c->pyr_args, c->d_geom, c->d_ptab, c->d_ytab4, c->d_bands,
                                       d_imgs, fs, pitch, img_end, c->d_pyr, c->d_blur, B));
        return hipGetLastError();
    }
    for (int l = 1; l < G.L; l++) {
        const OrbgLevel &L = G.lv[l], &P = G.lv[l - 1];
        const uint8_t *src = (l == 1) ? d_imgs : c->d_pyr + P.pyr_off;
        const int64_t sfs = (l == 1) ? fs : G.pyr_frame;
        const int spitch = (l == 1) ? pitch : P.pitch;
        dim3 grid((L.w + 255) / 256, (L.h + 16 * ORBG_RZ_NT - 1) / (16 * ORBG_RZ_NT), B);
        PROF_LAUNCH(c, "resize_chain",
                    hipLaunchKernelGGL(k_resize, grid, dim3(256), L.rz_pitch * L.rz_rows, st,
                                       src, sfs, spitch, P.w, c->d_pyr + L.pyr_off, G.pyr_frame,
                                       L.pitch, L.w, L.h, c->d_rtab + L.xtab_off,
                                       c->d_rtab + L.ytab_off, L.bulk_end, L.rz_pitch));
    }
    return hipGetLastError();
}

// GaussianBlur of levels [l0, l1) of every frame on `st`: k_blur2 (one wave per 244 x SEG
// output tile, blur_kernels.hip)
// level 0 of k_octree_lds: a batch's split pair (dims[2] then the frames past its cap at
// dims[0]), else one launch.  keep_cnt: k_octree runs concurrently (big_side) and owns the
// lvl_cnt entries of the levels left to it
static hipError_t launch_octree_l0(orbg_ctx *c, int B, hipStream_t st, bool keep_cnt = false)
{
    const bool small = B <= ORBG_SIDE_BLUR_B;
    OctLdsDims big = c->oct_dims[0];
    big.keep_cnt = keep_cnt;
    big.tag = c->oct_tag;
    if (!small && c->oct_dims[2].kcap > 0) {
        // d_err[3]: set by the first launch for a level it leaves to the second, which exits
        // at once while it is clear (ORBG_OCT_GATE=0: set, the second always scans)
        hipError_t e = hipMemsetAsync(c->d_err + 3, c->oct_gate ? 0 : 1, sizeof(int32_t), st);
        if (e != hipSuccess) return e;
        OctLdsDims first = c->oct_dims[2];
        first.keep_cnt = keep_cnt;
        first.tag = 0;
        e = launch_octree_lds(false, dim3(B, 1), oct_lds_bytes(first), st, c->d_geom,
                              c->d_cell_cnt, c->d_cell_kp, c->d_lvl_kp, c->d_lvl_idx,
                              c->d_lvl_cnt, c->d_err, first);
        if (e != hipSuccess) return e;
        big.kmin = c->oct_dims[2].kcap;
    }
    return launch_octree_lds(small, dim3(B, 1), oct_lds_bytes(big), st, c->d_geom, c->d_cell_cnt,
                             c->d_cell_kp, c->d_lvl_kp, c->d_lvl_idx, c->d_lvl_cnt, c->d_err, big);
}

// levels 1.. of k_octree_lds in one launch (keep_cnt as launch_octree_l0)
static hipError_t launch_octree_upper(orbg_ctx *c, int B, hipStream_t st, bool keep_cnt = false)
{
    OctLdsDims d = c->oct_dims[1];
    d.keep_cnt = keep_cnt;
    d.tag = c->oct_tag;
    return launch_octree_lds(B <= ORBG_SIDE_BLUR_B, dim3(B, c->geom.L - 1), oct_lds_bytes(d), st,
                             c->d_geom, c->d_cell_cnt, c->d_cell_kp, c->d_lvl_kp, c->d_lvl_idx,
                             c->d_lvl_cnt, c->d_err, d);
}

static hipError_t launch_blur_levels(orbg_ctx *c, hipStream_t st, const uint8_t *d_imgs, int B,
                                     int pitch, int64_t fs, int l0, int l1)
{
    const int32_t *b2 = c->tile_base.data();
    hipError_t e = hipSuccess;
    if (l1 <= l0) return e;
    const OrbgGeom &G = c->geom;
    if (G.fast_blur) {  // the FAST cells blurred the interior: the rest of levels [l0, l1)
        const int tpf = G.lv[l1 - 1].bt_off + G.lv[l1 - 1].bt_cnt - G.lv[l0].bt_off;
        PROF_LAUNCH(c, "blur",
                    e = launch_blur_border(st, c->d_geom, tpf, d_imgs, fs, pitch, c->d_pyr,
                                           c->d_blur, l0, l1, B));
        return e;
    }
    PROF_LAUNCH(c, "blur",
                e = launch_blur2(st, c->d_geom, c->d_tile_base, d_imgs, fs, pitch, c->d_pyr,
                                 c->d_blur, b2[l0], b2[l1] - b2[l0], B));
    return e;
}

// FAST cells [cb, cb + cn) of every frame on `st`: k_fast_rows over the strips of those
// levels (fast_rows_kernels.hip), k_fast2 (one wave per cell, fast_kernels.hip) when the plan has
// no strips or ORBG_FAST_ROWS=0.  cb and cb + cn are level boundaries (a level's cell_base).
static hipError_t launch_fast_cells(orbg_ctx *c, hipStream_t st, const uint8_t *d_imgs, int B,
                                    int pitch, int64_t fs, int cb, int cn)
{
    const OrbgGeom &G = c->geom;
    hipError_t e = hipSuccess;
    if (c->fr_ok && c->fr_mode) {
        int l0 = 0, l1 = G.L;
        while (l0 < G.L && G.lv[l0].cell_base < cb) l0++;
        while (l1 > l0 && G.lv[l1 - 1].cell_base >= cb + cn) l1--;
        const int t0 = c->ftile_base[l0], t1 = c->ftile_base[l1];
        PROF_LAUNCH(c, "fast_cells",
                    e = launch_fast_rows(st, c->d_geom, c->d_ftiles, d_imgs, fs, pitch, c->d_pyr,
                                         c->d_ctab, c->d_cell_cnt, c->d_cell_kp, B, t0, t1 - t0));
        return e;
    }
    PROF_LAUNCH(c, "fast_cells",
                e = launch_fast2(G.fc2_p4, 4 * G.fc2_wave_bytes, st, c->d_geom, c->d_cells, d_imgs,
                                 fs, pitch, c->d_pyr, c->d_ctab, c->d_cell_cnt, c->d_cell_kp,
                                 G.fast_blur ? c->d_blur : nullptr, B, cb, cn));
    return e;
}

// the packed frame block: header, keypoints at ORBG_PACK_OKP, descriptors at pack_ods
#define ORBG_PACK_OKP ((size_t)256)
static size_t pack_ods(int frame_cap)
{
    return ORBG_PACK_OKP + (((size_t)frame_cap * sizeof(orbg_keypoint) + 255) & ~(size_t)255);
}

// Pipelined batch into slot s (orbg_set_pipeline).  Front on `stream`: resize chain, FAST
// cells of every level (one launch), GaussianBlur.  Back on `ostream` (high priority):
// quadtree levels once the cells are written, k_octree, then orientation + descriptors once
// the blur is written.  The front of the next batch goes to the other slot, so it runs
// beside this back; the front into slot s waits until slot s's previous back is done.
// The back is in stream order on `ostream`, so the quadtree scratch (keys, lists, per-level
// outputs) is reused by consecutive batches without further events.  The input images
// must stay unchanged until the batch's outputs are complete (the back reads level 0).
static int launch_extract_pipe(orbg_ctx *c, const uint8_t *d_imgs, int B, int pitch, int64_t fs,
                               int s)
{
    const OrbgGeom &G = c->geom;
    {
        hipStream_t st = c->stream;
        if (c->back_pending[s]) {
            HIPCHK(hipStreamWaitEvent(st, c->ev_back[s], 0));
            c->back_pending[s] = false;
        }
        const bool side = c->fstream && G.L > 1;
        const int n0 = side ? G.lv[1].cell_base : 0;
        // fused: k_pyramid blurs levels >= 1 itself (fuse_blur 2) or every level (1)
        const int fz = c->pyr_ok ? c->pyr_args.fuse_blur : 0;
        const bool fused = fz != 0;
        if (side) {
            // level 0 beside the pyramid: FAST cells, then its GaussianBlur
            HIPCHK(hipEventRecord(c->ev_pfork[s], st));
            HIPCHK(hipStreamWaitEvent(c->fstream, c->ev_pfork[s], 0));
            {
                hipStream_t st = c->fstream;  // PROF_LAUNCH records on `st`
                HIPCHK(launch_fast_cells(c, st, d_imgs, B, pitch, fs, 0, n0));
                HIPCHK(hipEventRecord(c->ev_f0[s], st));
                if (fz != 1) HIPCHK(launch_blur_levels(c, st, d_imgs, B, pitch, fs, 0, 1));
                HIPCHK(hipEventRecord(c->ev_b0[s], st));
            }
        }
        HIPCHK(launch_pyramid(c, st, d_imgs, B, pitch, fs));
        // blur_side: levels 1.. of the GaussianBlur on the side stream too, beside the FAST
        // cells of levels 1.. (both need only the pyramid)
        const bool bside = side && c->blur_side && !fused;
        if (bside) {
            HIPCHK(hipEventRecord(c->ev_pyr[s], st));
            HIPCHK(hipStreamWaitEvent(c->fstream, c->ev_pyr[s], 0));
            hipStream_t st = c->fstream;
            HIPCHK(launch_blur_levels(c, st, d_imgs, B, pitch, fs, side ? 1 : 0, G.L));
            HIPCHK(hipEventRecord(c->ev_b0[s], st));
        }
        HIPCHK(launch_fast_cells(c, st, d_imgs, B, pitch, fs, n0, G.ncells - n0));
        if (side) HIPCHK(hipStreamWaitEvent(st, c->ev_f0[s], 0));
        HIPCHK(hipEventRecord(c->ev_cells[s], st));
        if (!bside && !fused) HIPCHK(launch_blur_levels(c, st, d_imgs, B, pitch, fs, side ? 1 : 0, G.L));
        if (!side && fz == 2) HIPCHK(launch_blur_levels(c, st, d_imgs, B, pitch, fs, 0, 1));
        if (side) HIPCHK(hipStreamWaitEvent(st, c->ev_b0[s], 0));
        HIPCHK(hipEventRecord(c->ev_front[s], st));
    }
    hipStream_t st = c->ostream;  // the back (PROF_LAUNCH records on `st`)
    HIPCHK(hipStreamWaitEvent(st, c->ev_cells[s], 0));
    // d_err[2] cleared ahead of this batch's quadtree launches: k_octree's workgroups exit at
    // once unless one of them left a level to it (the single-frame path clears it itself)
    HIPCHK(hipMemsetAsync(c->d_err + 2, 0, sizeof(int32_t), st));
    PROF_LAUNCH(c, "octree", launch_octree_l0(c, B, st));
    if (G.L > 1) PROF_LAUNCH(c, "octree", launch_octree_upper(c, B, st));
    PROF_LAUNCH(c, "octree_big",
                hipLaunchKernelGGL(k_octree, dim3(G.L, B), dim3(ORBG_OCT_THREADS), 0, st,
                                   c->d_geom, c->d_cell_cnt, c->d_cell_kp, c->d_keys, c->d_knode,
                                   c->d_act, c->d_qk, c->d_nodes, c->d_lvl_kp, c->d_lvl_idx, c->d_lvl_cnt,
                                   c->d_err, c->oct_gate ? 1 : 0));
    HIPCHK(hipStreamWaitEvent(st, c->ev_front[s], 0));
    if (c->mat_pending[s]) {  // the matching of the batch before last reads output slot s
        HIPCHK(hipStreamWaitEvent(st, c->ev_mat[s], 0));
        c->mat_pending[s] = false;
    }
    if (c->rel_pending[s]) {  // ... and so may the caller (orbg_batch_release)
        HIPCHK(hipStreamWaitEvent(st, c->ev_rel[s], 0));
        c->rel_pending[s] = false;
    }
    c->slot = s;
    c->d_kps = c->kps_slot[s];
    c->d_desc = c->desc_slot[s];
    c->d_counts = c->counts_slot[s];
    PROF_LAUNCH(c, "orient_desc",
                launch_orient_desc(G.brief_fma != 0, G.blur_tiled != 0,
                                   dim3((G.out_frame + 4 * ORBG_OD_KPW - 1) / (4 * ORBG_OD_KPW) * B),
                                   st, c->d_geom, d_imgs, fs, pitch, c->d_pyr,
                                   c->d_blur, c->d_odtab, c->d_lvl_kp, c->d_lvl_idx, c->d_lvl_cnt,
                                   (OrbgKeypointDev *)c->d_kps, c->d_desc, c->d_counts));
    HIPCHK(hipEventRecord(c->ev_ext[s], st));
    HIPCHK(hipEventRecord(c->ev_back[s], st));
    c->back_pending[s] = true;
    HIPCHK(hipGetLastError());
    c->last_img = d_imgs;
    c->last_fs = fs;
    c->last_pitch = pitch;
    c->last_n = B;
    return ORBG_OK;
}

// stream the last batch's per-frame outputs were written on (and stereo runs on): the back
// stream only if that batch actually took the pipelined path (orbg_set_serial on a
// pipelined context runs everything on the context stream)
static hipStream_t back_stream(orbg_ctx *c) { return c->last_piped ? c->ostream : c->stream; }

static int launch_extract(orbg_ctx *c, const uint8_t *d_imgs, int B, int pitch, int64_t fs)
{
    const OrbgGeom &G = c->geom;
    hipStream_t st = c->stream;
    // the match / stereo outputs of the previous batch are stale from here on
    c->last_npairs = 0;
    c->last_nstereo = 0;
    c->hc_done = false;
#ifdef ORBG_DEV_KNOBS
    g_extract_batches++;
#endif
    // d_err is not cleared here: it is sticky until check_err reads it
    // this batch's slot: intermediates (pyramid, blur, FAST cells) and per-frame outputs
    const int s = c->slot ^ 1;
    c->d_pyr = c->pyr_slot[s];
    c->d_blur = c->blur_slot[s];
    c->d_cell_cnt = c->cnt_slot[s];
    c->d_cell_kp = c->ckp_slot[s];
    c->last_piped = c->pipelined && !c->serial;
    if (c->last_piped) return launch_extract_pipe(c, d_imgs, B, pitch, fs, s);
    // serial (orbg_set_serial): every kernel on the caller's stream, one after the other
    const int oct_mode = c->serial ? 0 : c->oct_mode;
    // fast0: the level-0 FAST cells and quadtree need only the input images, so they run on
    // the quadtree stream beside the resize chain (latency-bound small launches)
    const bool fast0 = c->fast0_mode && oct_mode && G.L > 1;
    const int n0 = G.L > 1 ? G.lv[1].cell_base : G.ncells;
    // fused: k_pyramid blurs levels >= 1 itself (fuse_blur 2) or every level (1)
    const int fz = c->pyr_ok ? c->pyr_args.fuse_blur : 0;
    const bool fused = fz != 0;
    // blur0: the level-0 GaussianBlur follows them there (ORBG_BLUR0)
    const bool blur0 = fast0 && c->blur0_mode && fz != 1;
    // blur_side: small batches (the single-frame drop-in) blur every level on the quadtree
    // stream after the level-0 quadtree, so levels 1.. go FAST -> quadtree without waiting for
    // the blur on the extraction stream (at B = 1 the blur is ~9 us of a ~150 us chain)
    const bool blur_side = fast0 && oct_mode == 1 && !fused && !blur0 && B <= ORBG_SIDE_BLUR_B && c->sblur;
    auto launch_fast = [&](hipStream_t q, int cb, int cn) {
        return launch_fast_cells(c, q, d_imgs, B, pitch, fs, cb, cn);
    };
    // big_side: k_octree beside the quadtree launches (needs fast0's two FAST launches)
    const bool big_side = fast0 && c->big_side;
    // pyr_first (small batches): the resize chain is the frame's critical path, so k_pyramid is
    // submitted before the level-0 FAST cells' wait and launch (the wait still refers to the
    // event recorded ahead of k_pyramid: the images only)
    const bool pyr_first = fast0 && B <= ORBG_SIDE_BLUR_B && pyr_first_enabled();
    // early (with pyr_first): each quadtree launch is submitted right behind its FAST launch,
    // ahead of the side blur's wait and launch -- at B = 1 the host's launch sequence, not the
    // GPU, paced the quadtrees' starts (r06at: 9-12 us behind their FAST cells)
    const bool early = pyr_first && oct_mode == 1 && !big_side;
    if (fast0) {
        HIPCHK(hipEventRecord(c->ev_fast, st));
        if (pyr_first) HIPCHK(launch_pyramid(c, st, d_imgs, B, pitch, fs));
        HIPCHK(hipStreamWaitEvent(c->ostream, c->ev_fast, 0));
        HIPCHK(launch_fast(c->ostream, 0, n0));
        if (big_side) HIPCHK(hipEventRecord(c->ev_big_a, c->ostream));
        if (early) {
            hipStream_t st = c->ostream;  // PROF_LAUNCH records on `st`
            PROF_LAUNCH(c, "octree", launch_octree_l0(c, B, st, false));
        }
    }
    if (!pyr_first) HIPCHK(launch_pyramid(c, st, d_imgs, B, pitch, fs));
    if (blur_side) HIPCHK(hipEventRecord(c->ev_fast, st));  // pyramid written: the side blur
    if (fast0) {
        HIPCHK(launch_fast(st, n0, G.ncells - n0));
        if (early && G.L > 1) PROF_LAUNCH(c, "octree", launch_octree_upper(c, B, st, false));
        if (big_side) {
            HIPCHK(hipEventRecord(c->ev_big_b, st));
            HIPCHK(hipStreamWaitEvent(c->fstream, c->ev_big_a, 0));
            HIPCHK(hipStreamWaitEvent(c->fstream, c->ev_big_b, 0));
            hipStream_t st = c->fstream;  // PROF_LAUNCH records on `st`
            PROF_LAUNCH(c, "octree_big",
                        hipLaunchKernelGGL(k_octree, dim3(G.L, B), dim3(ORBG_OCT_THREADS), 0, st,
                                           c->d_geom, c->d_cell_cnt, c->d_cell_kp, c->d_keys,
                                           c->d_knode, c->d_act, c->d_qk, c->d_nodes, c->d_lvl_kp,
                                           c->d_lvl_idx, c->d_lvl_cnt, c->d_err, 0));
            HIPCHK(hipEventRecord(c->ev_big, st));
        }
    } else {
        HIPCHK(launch_fast(st, 0, G.ncells));
        if (oct_mode) {
            HIPCHK(hipEventRecord(c->ev_fast, st));
            HIPCHK(hipStreamWaitEvent(c->ostream, c->ev_fast, 0));
        }
    }
    {
        // PROF_LAUNCH records on `st`
        hipStream_t st = oct_mode ? c->ostream : c->stream;
        if (!early) PROF_LAUNCH(c, "octree", launch_octree_l0(c, B, st, big_side));
        if (oct_mode == 2 && G.L > 1) {
            // levels 1.. need their FAST cells (launched on the extraction stream under fast0)
            if (fast0) {
                HIPCHK(hipEventRecord(c->ev_fast, c->stream));
                HIPCHK(hipStreamWaitEvent(st, c->ev_fast, 0));
            }
            PROF_LAUNCH(c, "octree", launch_octree_upper(c, B, st, big_side));
        }
        if (blur0) HIPCHK(launch_blur_levels(c, st, d_imgs, B, pitch, fs, 0, 1));
        if (blur_side && c->blur_q3) {
            // a third queue (A/B, off): the blur needs only the pyramid, so k_orient_desc's
            // joins would be signalled well before the level-1.. quadtree ends
            HIPCHK(hipStreamWaitEvent(c->fstream, c->ev_fast, 0));
            HIPCHK(launch_blur_levels(c, c->fstream, d_imgs, B, pitch, fs, 0, G.L));
            HIPCHK(hipEventRecord(c->ev_sblur, c->fstream));
        } else if (blur_side) {
            HIPCHK(hipStreamWaitEvent(st, c->ev_fast, 0));
            HIPCHK(launch_blur_levels(c, st, d_imgs, B, pitch, fs, 0, G.L));
        }
        if (oct_mode) HIPCHK(hipEventRecord(c->ev_oct, st));
    }
    if (!fused && !blur_side)
        HIPCHK(launch_blur_levels(c, st, d_imgs, B, pitch, fs, blur0 ? 1 : 0, G.L));
    else if (fz == 2 && !blur0) HIPCHK(launch_blur_levels(c, st, d_imgs, B, pitch, fs, 0, 1));
    if (oct_mode != 2 && G.L > 1 && !early)
        PROF_LAUNCH(c, "octree", launch_octree_upper(c, B, st, big_side));
    if (oct_mode) HIPCHK(hipStreamWaitEvent(st, c->ev_oct, 0));
    if (blur_side && c->blur_q3) HIPCHK(hipStreamWaitEvent(st, c->ev_sblur, 0));
    if (big_side)
        HIPCHK(hipStreamWaitEvent(st, c->ev_big, 0));
    else if (!c->skip_big)
        PROF_LAUNCH(c, "octree_big",
                    hipLaunchKernelGGL(k_octree, dim3(G.L, B), dim3(ORBG_OCT_THREADS), 0, st,
                                       c->d_geom, c->d_cell_cnt, c->d_cell_kp, c->d_keys, c->d_knode,
                                       c->d_act, c->d_qk, c->d_nodes, c->d_lvl_kp, c->d_lvl_idx,
                                       c->d_lvl_cnt, c->d_err, 0));
    // per-frame outputs go to the other slot; wait until its last reader (matching of the
    // batch before last) is done
    if (c->mat_pending[s]) {
        HIPCHK(hipStreamWaitEvent(st, c->ev_mat[s], 0));
        c->mat_pending[s] = false;
    }
    if (c->rel_pending[s]) {
        HIPCHK(hipStreamWaitEvent(st, c->ev_rel[s], 0));
        c->rel_pending[s] = false;
    }
    c->slot = s;
    c->d_kps = c->kps_slot[s];
    c->d_desc = c->desc_slot[s];
    c->d_counts = c->counts_slot[s];
    PROF_LAUNCH(c, "orient_desc",
                launch_orient_desc(G.brief_fma != 0, G.blur_tiled != 0,
                                   dim3((G.out_frame + 4 * ORBG_OD_KPW - 1) / (4 * ORBG_OD_KPW) * B),
                                   st, c->d_geom, d_imgs, fs, pitch, c->d_pyr,
                                   c->d_blur, c->d_odtab, c->d_lvl_kp, c->d_lvl_idx, c->d_lvl_cnt, (OrbgKeypointDev *)c->d_kps,
                                   c->d_desc, c->d_counts,
                                   c->hc_dst, c->d_err, c->hc_dst ? ORBG_PACK_OKP : 0,
                                   c->hc_dst ? pack_ods(G.frame_cap) : 0, c->oct_tag));
    HIPCHK(hipEventRecord(c->ev_ext[s], st));
    HIPCHK(hipGetLastError());
    c->last_img = d_imgs;
    c->last_fs = fs;
    c->last_pitch = pitch;
    c->last_n = B;
    return ORBG_OK;
}

// the single-frame path's latency-critical waits (the frame's extraction, its
// SearchForInitialization).  ORBG_SPIN=1 polls the stream with hipStreamQuery first (the
// blocking synchronize wakes 6-8 us after the last kernel, r06au); measured no faster (0.2315
// against 0.2296 ms p50, r06aw: the traced gap to the next launch grew), so off by default
static int spin_sync(hipStream_t st)
{
    static const int on = [] {
        const char *e = getenv("ORBG_SPIN");
        return e ? atoi(e) : 0;
    }();
    if (on) {
        for (;;) {
            const hipError_t e = hipStreamQuery(st);
            if (e == hipSuccess) break;
            if (e != hipErrorNotReady) return set_err(ORBG_EIO, "hipStreamQuery: %s", hipGetErrorString(e));
        }
    }
    HIPCHK(hipStreamSynchronize(st));
    return ORBG_OK;
}

// both streams drained (host reads of any output)
static int sync_all(orbg_ctx *c)
{
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipStreamSynchronize(c->mstream));
    if (c->ostream) HIPCHK(hipStreamSynchronize(c->ostream));
    c->mat_pending[0] = c->mat_pending[1] = false;
    for (int i = 0; i < 2; i++)
        if (c->rel_pending[i]) HIPCHK(hipEventSynchronize(c->ev_rel[i]));
    if (c->srel_pending) HIPCHK(hipEventSynchronize(c->ev_srel));
    if (c->ssum_pending) HIPCHK(hipEventSynchronize(c->ev_ssum));
    c->rel_pending[0] = c->rel_pending[1] = c->srel_pending = c->ssum_pending = false;
    return ORBG_OK;
}

// the error a non-zero device error word maps to (check_err, orbg_download_frame)
static int err_from_flags(int32_t flags, int32_t first)
{
    if (flags & ORBG_DEVFLAG_COUNT)
        return set_err(ORBG_EINVAL, "a device matcher count exceeded its capacity (clamped; "
                                    "flags 0x%x, first pair %d since the last check)", flags, first);
    return set_err(ORBG_ENOTSUP, "quadtree capacity exceeded (flags 0x%x, first frame %d of "
                                 "a batch since the last check)", flags, first);
}

// Drains every stream, then reads and clears the sticky device error word: a non-zero flag
// means some frame since the last read lost a level (quadtree capacity exceeded) and its
// keypoints are incomplete, so the caller gets ORBG_ENOTSUP instead of short outputs; or
// that a device matcher was handed a count past its capacity (ORBG_DEVFLAG_COUNT: clamped,
// ORBG_EINVAL).
static int check_err(orbg_ctx *c)
{
    int rc = sync_all(c);
    if (rc) return rc;
    c->prof.collect();
    int32_t e[2] = {0, 0};
    HIPCHK(hipMemcpy(e, c->d_err, sizeof(e), hipMemcpyDeviceToHost));
    if (e[0]) {
        const int32_t e0[2] = {0, INT32_MAX};
        HIPCHK(hipMemcpy(c->d_err, e0, sizeof(e0), hipMemcpyHostToDevice));
        return err_from_flags(e[0], e[1]);
    }
    return ORBG_OK;
}

extern "C" int orbg_check_errors(orbg_ctx *c)
{
    if (!c) return set_err(ORBG_EINVAL, "ctx is NULL");
    return check_err(c);
}

extern "C" int orbg_extract_batch_device(orbg_ctx *c, const uint8_t *d_imgs, int nframes, int w,
                                         int h, size_t step, size_t frame_stride)
{
    if (!c || !d_imgs) return set_err(ORBG_EINVAL, "NULL argument");
    if (nframes <= 0 || w <= 0 || h <= 0 || step < (size_t)w)
        return set_err(ORBG_EINVAL, "bad batch shape");
    HIPCHK(hipSetDevice(c->device));
    int rc = plan(c, w, h, std::max(nframes, c->p.max_batch));
    if (rc) return rc;
    return launch_extract(c, d_imgs, nframes, (int)step, (int64_t)frame_stride);
}

extern "C" int orbg_batch_outputs(orbg_ctx *c, orbg_keypoint **d_kps, uint8_t **d_desc,
                                  int32_t **d_counts, int32_t *frame_cap)
{
    if (!c || !c->gw) return set_err(ORBG_EINVAL, "no batch extracted yet");
    if (d_kps) *d_kps = c->d_kps;
    if (d_desc) *d_desc = c->d_desc;
    if (d_counts) *d_counts = c->d_counts;
    if (frame_cap) *frame_cap = c->geom.frame_cap;
    return ORBG_OK;
}

// One frame's outputs gathered into one device block for a single DMA: [0..4) the sticky
// error word and the count, then the frame's keypoints and descriptors (count entries).
__global__ void k_pack_frame(const int32_t *__restrict__ err, const int32_t *__restrict__ counts,
                             const uint32_t *__restrict__ kps, const uint32_t *__restrict__ desc,
                             int frame, size_t fc, size_t okp, size_t ods,
                             uint32_t *__restrict__ pack)
{
    const int n = counts[frame];
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t kw = sizeof(orbg_keypoint) / 4, nk = (size_t)n * kw, nd = (size_t)n * 8;
    if (i < 4) pack[i] = i < 2 ? (uint32_t)err[i] : i == 2 ? (uint32_t)n : 0u;
    if (i < nk) pack[okp / 4 + i] = kps[(size_t)frame * fc * kw + i];
    if (i < nd) pack[ods / 4 + i] = desc[(size_t)frame * fc * 8 + i];
}

// drained: the caller (orbg_extract's optimistic path) drained every stream after the frame's
// last launch, and k_orient_desc filled the block: no second round of synchronisations
static int download_frame(orbg_ctx *c, int frame, orbg_keypoint *kps, uint8_t *desc, int cap,
                          int *n_out, bool drained);

extern "C" int orbg_download_frame(orbg_ctx *c, int frame, orbg_keypoint *kps, uint8_t *desc,
                                   int cap, int *n_out)
{
    return download_frame(c, frame, kps, desc, cap, n_out, false);
}

static int download_frame(orbg_ctx *c, int frame, orbg_keypoint *kps, uint8_t *desc, int cap,
                          int *n_out, bool drained)
{
    if (!c || !c->gw || frame < 0 || frame >= c->last_n)
        return set_err(ORBG_EINVAL, "bad frame index");
    static_assert(sizeof(orbg_keypoint) % 4 == 0, "keypoint records are whole words");
    // the error word, count, keypoints and descriptors in one pinned round trip: a packing
    // kernel behind the frame's last writer (the back stream), one DMA, then the streams are
    // drained as check_err does, so the error word covers every batch since the last read
    const size_t fc = (size_t)c->geom.frame_cap;
    const size_t okp = ORBG_PACK_OKP, ods = pack_ods(c->geom.frame_cap);
    const size_t bytes = ods + fc * 32;
    int rc;
    uint8_t *hs, *dst;
    // orbg_extract's k_orient_desc already stored frame 0's outputs into the block
    const bool packed = c->hc_done && frame == 0;
    c->hc_done = false;
    if (use_zc(c)) {
        if ((rc = zc_buf(c, bytes, &hs, &dst))) return rc;
    } else {
        if (c->pack_bytes < bytes) {
            if ((rc = sync_all(c))) return rc;
            if (c->d_pack) hipFree(c->d_pack);
            c->d_pack = nullptr;
            c->pack_bytes = 0;
            if ((rc = dalloc(&c->d_pack, bytes))) return rc;
            c->pack_bytes = bytes;
        }
        if ((rc = stage(c, bytes, &hs))) return rc;
        dst = c->d_pack;
    }
    hipStream_t st = back_stream(c);
    if (!packed) {
        const size_t words = std::max(fc * (sizeof(orbg_keypoint) / 4), fc * 8);
        hipLaunchKernelGGL(k_pack_frame, dim3((unsigned)((words + 255) / 256)), dim3(256), 0, st,
                           c->d_err, c->d_counts, (const uint32_t *)c->d_kps,
                           (const uint32_t *)c->d_desc, frame, fc, okp, ods, (uint32_t *)dst);
        HIPCHK(hipGetLastError());
    }
    if (!use_zc(c)) HIPCHK(hipMemcpyAsync(hs, c->d_pack, bytes, hipMemcpyDeviceToHost, st));
    if (!(drained && packed && use_zc(c)) && (rc = sync_all(c))) return rc;
    c->prof.collect();
    int32_t hdr[3];
    std::memcpy(hdr, hs, sizeof(hdr));
    if (hdr[0]) {  // check_err's reset and error
        const int32_t e0[2] = {0, INT32_MAX};
        HIPCHK(hipMemcpy(c->d_err, e0, sizeof(e0), hipMemcpyHostToDevice));
        return err_from_flags(hdr[0], hdr[1]);
    }
    const int32_t n = hdr[2];
    if (n_out) *n_out = n;
    if (n > cap) return set_err(ORBG_ERANGE, "capacity %d < %d keypoints", cap, n);
    if (kps && n) std::memcpy(kps, hs + okp, n * sizeof(orbg_keypoint));
    if (desc && n) std::memcpy(desc, hs + ods, (size_t)n * 32);
    return ORBG_OK;
}

static int extract_graph(orbg_ctx *c, const uint8_t *img, int w, int h, size_t step,
                         orbg_keypoint *kps, uint8_t *desc, int cap, int *n_out);
#ifndef ORBG_H2D_CHUNKS
#define ORBG_H2D_CHUNKS 1  // orbg_extract's image upload bands (4: +0.025 ms per frame, r05n: each DMA submission costs more than the overlap saves)
#endif

extern "C" int orbg_extract(orbg_ctx *c, const uint8_t *img, int w, int h, size_t step,
                            orbg_keypoint *kps, uint8_t *desc, int cap, int *n_out)
{
    if (!c) return set_err(ORBG_EINVAL, "ctx is NULL");
    if (w == 0 || h == 0 || img == nullptr) {  // _image.empty(): return (:1333-1334)
        if (n_out) *n_out = -1;
        return ORBG_OK;
    }
    if (w < 0 || h < 0 || step < (size_t)w) return set_err(ORBG_EINVAL, "bad image shape");
    HIPCHK(hipSetDevice(c->device));
    int rc = plan(c, w, h, c->p.max_batch);
    if (rc) return rc;
    const size_t bytes = (size_t)w * h;
    const size_t bytes16 = (bytes + 15) & ~(size_t)15;  // k_copy16's whole words
    if (c->img_bytes < bytes16) {
        if (c->d_img) hipFree(c->d_img);
        c->d_img = nullptr;
        c->img_bytes = 0;
        if ((rc = dalloc(&c->d_img, bytes16))) return rc;
        c->img_bytes = bytes16;
    }
    if (c->graph_mode && !c->prof.on && c->stream && !(c->pipelined && !c->serial) &&
        !c->mat_pending[c->slot ^ 1] && !c->rel_pending[c->slot ^ 1])
        return extract_graph(c, img, w, h, step, kps, desc, cap, n_out);
    // rows into pinned staging (a pageable 2-D copy of an odd-width image goes row by row:
    // ~3 ms for 1241 x 376), in ORBG_H2D_CHUNKS bands: the DMA of band k runs while the host
    // copies band k + 1
    uint8_t *hs;
    const bool pull = img_pull_enabled() && !c->graph_mode;
    if (pull) {
        uint8_t *ds;
        HIPCHK(hipStreamSynchronize(c->stream));  // the previous pull is done
        if ((rc = imz_buf(c, bytes16, &hs, &ds))) return rc;
        if (step == (size_t)w) {
            std::memcpy(hs, img, bytes);
        } else {
            for (int y = 0; y < h; y++) std::memcpy(hs + (size_t)y * w, img + (size_t)y * step, w);
        }
        const size_t n16 = bytes16 / 16;
        hipLaunchKernelGGL(k_copy16, dim3((unsigned)std::min<size_t>((n16 + 255) / 256, 1024)),
                           dim3(256), 0, c->stream, (const uint4 *)ds, (uint4 *)c->d_img, n16);
        HIPCHK(hipGetLastError());
    } else {
        if ((rc = stage(c, bytes, &hs))) return rc;
        HIPCHK(hipStreamSynchronize(c->stream));  // the staging buffer's previous DMA is done
    }
    const int nch = pull ? 0 : std::max(1, std::min(ORBG_H2D_CHUNKS, h));
    for (int k = 0; k < nch; k++) {
        const int y0 = (int)((int64_t)h * k / nch), y1 = (int)((int64_t)h * (k + 1) / nch);
        if (step == (size_t)w) {
            std::memcpy(hs + (size_t)y0 * w, img + (size_t)y0 * w, (size_t)(y1 - y0) * w);
        } else {
            for (int y = y0; y < y1; y++) std::memcpy(hs + (size_t)y * w, img + (size_t)y * step, w);
        }
        HIPCHK(hipMemcpyAsync(c->d_img + (size_t)y0 * w, hs + (size_t)y0 * w, (size_t)(y1 - y0) * w,
                              hipMemcpyHostToDevice, c->stream));
    }
    // zero-copy on the non-pipelined path: k_orient_desc stores the packed outputs itself
    // (ORBG_HC=0: k_pack_frame after it, A/B)
    uint8_t *hz = nullptr, *dz = nullptr;
    if (use_zc(c) && !(c->pipelined && !c->serial) && hc_enabled()) {
        const size_t pbytes = pack_ods(c->geom.frame_cap) + (size_t)c->geom.frame_cap * 32;
        if ((rc = zc_buf(c, pbytes, &hz, &dz))) return rc;
    }
    // optimistic: without k_octree when every level has an LDS quadtree launch (its early exits
    // flag d_err[2]; a flagged frame is extracted again with k_octree, ORBG_SKIP_BIG=0: never)
    const bool skip = dz && c->oct_dims[0].kcap > 0 && c->oct_dims[1].kcap > 0 && skip_big_enabled();
    // the flag is this frame's alone: an earlier batch (non-pipelined batches never clear it)
    // or an earlier rerun frame would otherwise force a needless second extraction.  Default:
    // a fresh tag per call, which the quadtree stores into d_err[4] and k_orient_desc compares
    // (nothing to clear: a memset ahead of the frame cost a blit and two queue gaps on the
    // critical chain); ORBG_SF_TAG=0: d_err[2] cleared ahead of the frame
    const bool tag = skip && sf_tag_enabled();
    if (tag) {
        c->sf_seq = c->sf_seq == INT32_MAX ? 1 : c->sf_seq + 1;
        c->oct_tag = c->sf_seq;
    } else if (skip) {
        HIPCHK(hipMemsetAsync(c->d_err + 2, 0, sizeof(int32_t), c->stream));
    }
    c->hc_dst = dz;
    c->skip_big = skip;
    rc = launch_extract(c, c->d_img, 1, w, (int64_t)bytes);
    c->hc_dst = nullptr;
    c->skip_big = false;
    c->oct_tag = 0;
    if (rc) return rc;
    bool drained = false;
    if (skip) {
        if ((rc = spin_sync(c->stream)) || (rc = sync_all(c))) return rc;
        drained = true;
        if (((const int32_t *)hz)[3]) {  // a level needed the fallback: again, with k_octree
            drained = false;
            const int32_t z = 0;
            if (!tag) HIPCHK(hipMemcpy(c->d_err + 2, &z, sizeof(z), hipMemcpyHostToDevice));
            c->hc_dst = dz;
            rc = launch_extract(c, c->d_img, 1, w, (int64_t)bytes);
            c->hc_dst = nullptr;
            if (rc) return rc;
        }
    }
    c->hc_done = dz != nullptr;
    return download_frame(c, 0, kps, desc, cap, n_out, drained);
}

// the context state launch_extract leaves for a non-pipelined batch into slot s (a graph
// replay sets it without the launches)
static void extract_state(orbg_ctx *c, int s, const uint8_t *d_imgs, int B, int pitch, int64_t fs)
{
    c->last_npairs = 0;
    c->last_nstereo = 0;
    c->d_pyr = c->pyr_slot[s];
    c->d_blur = c->blur_slot[s];
    c->d_cell_cnt = c->cnt_slot[s];
    c->d_cell_kp = c->ckp_slot[s];
    c->last_piped = false;
    c->slot = s;
    c->d_kps = c->kps_slot[s];
    c->d_desc = c->desc_slot[s];
    c->d_counts = c->counts_slot[s];
    c->last_img = d_imgs;
    c->last_fs = fs;
    c->last_pitch = pitch;
    c->last_n = B;
}

static int pinned(uint8_t **p, size_t *have, size_t bytes)
{
    if (*have >= bytes) return ORBG_OK;
    if (*p) hipHostFree(*p);
    *p = nullptr;
    *have = 0;
    if (hipHostMalloc((void **)p, bytes, hipHostMallocDefault) != hipSuccess)
        return set_err(ORBG_ENOMEM, "hipHostMalloc(%zu bytes)", bytes);
    *have = bytes;
    return ORBG_OK;
}

// orbg_extract through a captured hipGraph (graph_mode; plan, d_img and the caller checks done
// by orbg_extract).  The first frame of a (slot, size) runs eagerly (module loads, attribute
// setup happen outside any capture), the second is captured and every later one replayed.
static int extract_graph(orbg_ctx *c, const uint8_t *img, int w, int h, size_t step,
                         orbg_keypoint *kps, uint8_t *desc, int cap, int *n_out)
{
    const size_t bytes = (size_t)w * h;
    const size_t fc = (size_t)c->geom.frame_cap;
    const size_t okp = 256, ods = okp + ((fc * sizeof(orbg_keypoint) + 255) & ~(size_t)255);
    const size_t obytes = ods + fc * 32;
    int rc;
    if (c->pack_bytes < obytes) {
        if ((rc = sync_all(c))) return rc;
        if (c->d_pack) hipFree(c->d_pack);
        c->d_pack = nullptr;
        c->pack_bytes = 0;
        if ((rc = dalloc(&c->d_pack, obytes))) return rc;
        c->pack_bytes = obytes;
    }
    if ((rc = sync_all(c))) return rc;  // the pinned buffers' previous DMAs are done
    if (c->gin_bytes < bytes || c->gout_bytes < obytes) {
        for (int i = 0; i < 2; i++) {  // graphs hold the old host buffers
            if (c->gexec[i]) hipGraphExecDestroy(c->gexec[i]);
            c->gexec[i] = nullptr;
            c->gkey[i] = 0;
        }
        if ((rc = pinned(&c->h_gin, &c->gin_bytes, bytes))) return rc;
        if ((rc = pinned(&c->h_gout, &c->gout_bytes, obytes))) return rc;
    }
    if (step == (size_t)w) {
        std::memcpy(c->h_gin, img, bytes);
    } else {
        for (int y = 0; y < h; y++) std::memcpy(c->h_gin + (size_t)y * w, img + (size_t)y * step, w);
    }
    const int s = c->slot ^ 1;
    const uint64_t key = (c->plan_gen << 40) ^ ((uint64_t)w << 20) ^ (uint64_t)h;
    hipStream_t st = c->stream;
    // graph_mode 1: the copies inside the graph; 2: kernels only (the copies eager around the
    // launch); 3: as 2 with the extraction captured on the one context stream (a linear graph)
    const bool copies_in = c->graph_mode == 1;
    if (c->gexec[s] && c->gkey[s] == key) {
        extract_state(c, s, c->d_img, 1, w, (int64_t)bytes);
        if (!copies_in) HIPCHK(hipMemcpyAsync(c->d_img, c->h_gin, bytes, hipMemcpyHostToDevice, st));
        HIPCHK(hipGraphLaunch(c->gexec[s], st));
        if (!copies_in)
            HIPCHK(hipMemcpyAsync(c->h_gout, c->d_pack, obytes, hipMemcpyDeviceToHost, st));
    } else {
        if (c->gexec[s]) hipGraphExecDestroy(c->gexec[s]);
        c->gexec[s] = nullptr;
        const bool capture = c->gkey_seen[s] == key;
        c->gkey_seen[s] = key;
        rc = ORBG_OK;
        if (!copies_in &&
            hipMemcpyAsync(c->d_img, c->h_gin, bytes, hipMemcpyHostToDevice, st) != hipSuccess)
            rc = set_err(ORBG_EIO, "hipMemcpyAsync");
        if (capture) HIPCHK(hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed));
        if (!rc && copies_in &&
            hipMemcpyAsync(c->d_img, c->h_gin, bytes, hipMemcpyHostToDevice, st) != hipSuccess)
            rc = set_err(ORBG_EIO, "hipMemcpyAsync");
        const bool ser = c->serial;
        if (c->graph_mode == 3) c->serial = true;  // one stream: launch_extract's serial layout
        if (!rc) rc = launch_extract(c, c->d_img, 1, w, (int64_t)bytes);
        c->serial = ser;
        if (!rc) {
            const size_t words = std::max(fc * (sizeof(orbg_keypoint) / 4), fc * 8);
            hipLaunchKernelGGL(k_pack_frame, dim3((unsigned)((words + 255) / 256)), dim3(256), 0,
                               st, c->d_err, c->d_counts, (const uint32_t *)c->d_kps,
                               (const uint32_t *)c->d_desc, 0, fc, okp, ods, (uint32_t *)c->d_pack);
            if (hipGetLastError() != hipSuccess ||
                (copies_in && hipMemcpyAsync(c->h_gout, c->d_pack, obytes, hipMemcpyDeviceToHost,
                                             st) != hipSuccess))
                rc = set_err(ORBG_EIO, "k_pack_frame / D2H");
        }
        if (capture) {
            hipGraph_t g = nullptr;
            const hipError_t e = hipStreamEndCapture(st, &g);
            if (!rc && e != hipSuccess) rc = set_err(ORBG_EIO, "hipStreamEndCapture: %s", hipGetErrorString(e));
            if (!rc && hipGraphInstantiate(&c->gexec[s], g, nullptr, nullptr, 0) != hipSuccess)
                rc = set_err(ORBG_EIO, "hipGraphInstantiate");
            if (g) hipGraphDestroy(g);
            if (rc) {
                c->gexec[s] = nullptr;
                c->graph_mode = 0;  // fall back to eager launches for good
                return rc;
            }
            c->gkey[s] = key;
            HIPCHK(hipGraphLaunch(c->gexec[s], st));
        }
        if (rc) return rc;
        if (!copies_in)
            HIPCHK(hipMemcpyAsync(c->h_gout, c->d_pack, obytes, hipMemcpyDeviceToHost, st));
    }
    HIPCHK(hipEventRecord(c->ev_ext[s], st));
    if ((rc = sync_all(c))) return rc;
    int32_t hdr[3];
    std::memcpy(hdr, c->h_gout, sizeof(hdr));
    if (hdr[0]) {
        const int32_t e0[2] = {0, INT32_MAX};
        HIPCHK(hipMemcpy(c->d_err, e0, sizeof(e0), hipMemcpyHostToDevice));
        return err_from_flags(hdr[0], hdr[1]);
    }
    const int32_t n = hdr[2];
    if (n_out) *n_out = n;
    if (n > cap) return set_err(ORBG_ERANGE, "capacity %d < %d keypoints", cap, n);
    if (kps && n) std::memcpy(kps, c->h_gout + okp, n * sizeof(orbg_keypoint));
    if (desc && n) std::memcpy(desc, c->h_gout + ods, (size_t)n * 32);
    return ORBG_OK;
}

extern "C" int orbg_get_level(orbg_ctx *c, int frame, int level, uint8_t *dst, size_t dst_step,
                              int *lw, int *lh)
{
    if (!c || !c->gw) return set_err(ORBG_EINVAL, "nothing extracted yet");
    if (level < 0 || level >= c->geom.L || frame < 0 || frame >= c->last_n)
        return set_err(ORBG_EINVAL, "bad level/frame");
    const OrbgLevel &L = c->geom.lv[level];
    if (lw) *lw = L.w;
    if (lh) *lh = L.h;
    if (!dst) return ORBG_OK;
    if (dst_step < (size_t)L.w) return set_err(ORBG_EINVAL, "dst_step too small");
    int rc = sync_all(c);
    if (rc) return rc;
    if (level == 0)
        HIPCHK(hipMemcpy2D(dst, dst_step, c->last_img + frame * c->last_fs, c->last_pitch, L.w,
                           L.h, hipMemcpyDeviceToHost));
    else
        HIPCHK(hipMemcpy2D(dst, dst_step, c->d_pyr + frame * c->geom.pyr_frame + L.pyr_off,
                           L.pitch, L.w, L.h, hipMemcpyDeviceToHost));
    return ORBG_OK;
}

// the GaussianBlur of a pyramid level of the last batch (ORBextractor.cc:1375-1377: the
// image computeOrbDescriptor samples); a parity / debugging accessor, no reference member
extern "C" int orbg_get_blurred_level(orbg_ctx *c, int frame, int level, uint8_t *dst,
                                      size_t dst_step, int *lw, int *lh)
{
    if (!c || !c->gw) return set_err(ORBG_EINVAL, "nothing extracted yet");
    if (level < 0 || level >= c->geom.L || frame < 0 || frame >= c->last_n)
        return set_err(ORBG_EINVAL, "bad level/frame");
    const OrbgLevel &L = c->geom.lv[level];
    if (lw) *lw = L.w;
    if (lh) *lh = L.h;
    if (!dst) return ORBG_OK;
    if (dst_step < (size_t)L.w) return set_err(ORBG_EINVAL, "dst_step too small");
    int rc = sync_all(c);
    if (rc) return rc;
    const uint8_t *src = c->d_blur + frame * c->geom.blur_frame + L.blur_off;
    if (!c->geom.blur_tiled) {
        HIPCHK(hipMemcpy2D(dst, dst_step, src, L.pitch, L.w, L.h, hipMemcpyDeviceToHost));
        return ORBG_OK;
    }
    // tiled (blur2_tile TILED): the level's footprint, then its rows out of the tiles
    const int h8 = (L.h + 7) & ~7;
    std::vector<uint8_t> t((size_t)L.pitch * h8);
    HIPCHK(hipMemcpy(t.data(), src, t.size(), hipMemcpyDeviceToHost));
    for (int y = 0; y < L.h; y++)
        for (int x0 = 0; x0 < L.w; x0 += 16)
            memcpy(dst + (size_t)y * dst_step + x0,
                   t.data() + (size_t)(y >> 3) * 8 * L.pitch + (size_t)(x0 >> 4) * 128 + (y & 7) * 16,
                   std::min(16, L.w - x0));
    return ORBG_OK;
}

extern "C" int orbg_sync(orbg_ctx *c)
{
    if (!c) return set_err(ORBG_EINVAL, "ctx is NULL");
    return check_err(c);  // drains the streams and surfaces any device error flag
}

extern "C" void *orbg_stream(orbg_ctx *c) { return c ? (void *)c->stream : nullptr; }

extern "C" void *orbg_match_stream(orbg_ctx *c) { return c ? (void *)c->mstream : nullptr; }

extern "C" int orbg_set_stream(orbg_ctx *c, void *stream)
{
    if (!c) return set_err(ORBG_EINVAL, "ctx is NULL");
    int rc = sync_all(c);
    if (rc) return rc;
    c->prof.collect();
    c->stream = stream ? (hipStream_t)stream : c->own_stream;
    return ORBG_OK;
}

extern "C" int orbg_set_pipeline(orbg_ctx *c, int enable)
{
    if (!c) return set_err(ORBG_EINVAL, "ctx is NULL");
    if (enable && !c->ostream)
        return set_err(ORBG_ENOTSUP, "pipelined batches need the quadtree stream (ORBG_OCT_STREAM=0)");
    int rc = sync_all(c);
    if (rc) return rc;
    c->pipelined = enable ? 1 : 0;
    c->back_pending[0] = c->back_pending[1] = false;
    return ORBG_OK;
}

extern "C" int orbg_get_pipeline(const orbg_ctx *c) { return c ? c->pipelined : 0; }

extern "C" int orbg_set_serial(orbg_ctx *c, int enable)
{
    if (!c) return set_err(ORBG_EINVAL, "ctx is NULL");
    int rc = sync_all(c);
    if (rc) return rc;
    c->serial = enable != 0;
    c->back_pending[0] = c->back_pending[1] = false;
    return ORBG_OK;
}

extern "C" int orbg_get_quadtree_caps(const orbg_ctx *c, int32_t *first_cap, int32_t *level0_cap,
                                      int32_t *upper_cap)
{
    if (!c) return set_err(ORBG_EINVAL, "ctx is NULL");
    if (c->gw <= 0) return set_err(ORBG_EINVAL, "no image size planned yet");
    if (first_cap) *first_cap = c->oct_dims[2].kcap;
    if (level0_cap) *level0_cap = c->oct_dims[0].kcap;
    if (upper_cap) *upper_cap = c->oct_dims[1].kcap;
    return ORBG_OK;
}

extern "C" int orbg_get_blur_plan(const orbg_ctx *c, int32_t *fused, int64_t *interior_px,
                                  int64_t *border_px)
{
    if (!c) return set_err(ORBG_EINVAL, "ctx is NULL");
    if (c->gw <= 0) return set_err(ORBG_EINVAL, "no image size planned yet");
    const OrbgGeom &G = c->geom;
    int64_t in = 0, all = 0;
    for (int l = 0; l < G.L; l++) {
        all += (int64_t)G.lv[l].w * G.lv[l].h;
        if (G.fast_blur) in += (int64_t)(G.lv[l].bx1 - G.lv[l].bx0) * (G.lv[l].by1 - G.lv[l].by0);
    }
    if (fused) *fused = G.fast_blur;
    if (interior_px) *interior_px = in;
    if (border_px) *border_px = all - in;
    return ORBG_OK;
}

extern "C" int orbg_get_blur_layout(const orbg_ctx *c, int32_t *tiled)
{
    if (!c) return set_err(ORBG_EINVAL, "ctx is NULL");
    if (c->gw <= 0) return set_err(ORBG_EINVAL, "no image size planned yet");
    if (tiled) *tiled = c->geom.blur_tiled;
    return ORBG_OK;
}

extern "C" int orbg_batch_stats(orbg_ctx *c, int64_t *ncand, int64_t *nkp)
{
    if (!c || !c->gw || c->last_n <= 0) return set_err(ORBG_EINVAL, "no batch");
    int rc = check_err(c);
    if (rc) return rc;
    std::vector<int32_t> cc((size_t)c->last_n * c->geom.ncells), kc(c->last_n);
    HIPCHK(hipMemcpy(cc.data(), c->d_cell_cnt, cc.size() * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(kc.data(), c->d_counts, kc.size() * 4, hipMemcpyDeviceToHost));
    int64_t a = 0, b = 0;
    for (int32_t v : cc) a += v;
    for (int32_t v : kc) b += v;
    if (ncand) *ncand = a;
    if (nkp) *nkp = b;
    return ORBG_OK;
}

// `mstream` after everything queued on the context stream so far (ev_caller)
static hipError_t order_after_caller(orbg_ctx *c)
{
    hipError_t e = hipEventRecord(c->ev_caller, c->stream);
    if (e != hipSuccess) return e;
    return hipStreamWaitEvent(c->mstream, c->ev_caller, 0);
}

extern "C" int orbg_batch_summary(orbg_ctx *c, int32_t *d_out)
{
    if (!c || !c->gw || c->last_n <= 0 || !d_out) return set_err(ORBG_EINVAL, "no batch");
    const int s = c->slot;
    HIPCHK(order_after_caller(c));
    HIPCHK(hipStreamWaitEvent(c->mstream, c->ev_ext[s], 0));
    HIPCHK(hipMemcpyAsync(d_out, c->d_counts, c->last_n * sizeof(int32_t),
                          hipMemcpyDeviceToDevice, c->mstream));
    if (c->last_npairs > 0)
        HIPCHK(hipMemcpyAsync(d_out + c->last_n, c->d_nm, c->last_npairs * sizeof(int32_t),
                              hipMemcpyDeviceToDevice, c->mstream));
    HIPCHK(hipEventRecord(c->ev_mat[s], c->mstream));
    c->mat_pending[s] = true;
    return ORBG_OK;
}

extern "C" int orbg_batch_acquire(orbg_ctx *c, void *stream)
{
    if (!c || !c->gw || c->last_n <= 0) return set_err(ORBG_EINVAL, "no batch");
    const hipStream_t q = stream ? (hipStream_t)stream : c->mstream;
    HIPCHK(hipStreamWaitEvent(q, c->ev_ext[c->slot], 0));
    if (c->last_nstereo) HIPCHK(hipStreamWaitEvent(q, c->ev_sback, 0));
    return ORBG_OK;
}

extern "C" int orbg_batch_release(orbg_ctx *c, void *stream)
{
    if (!c || !c->gw || c->last_n <= 0) return set_err(ORBG_EINVAL, "no batch");
    const hipStream_t q = stream ? (hipStream_t)stream : c->mstream;
    const int s = c->slot;
    // a second reader stream of the same batch: chain the releases (q waits for the earlier
    // release's reads, then the one event covers both)
    if (c->rel_pending[s]) HIPCHK(hipStreamWaitEvent(q, c->ev_rel[s], 0));
    HIPCHK(hipEventRecord(c->ev_rel[s], q));
    c->rel_pending[s] = true;
    if (c->last_nstereo) {
        if (c->srel_pending) HIPCHK(hipStreamWaitEvent(q, c->ev_srel, 0));
        HIPCHK(hipEventRecord(c->ev_srel, q));
        c->srel_pending = true;
    }
    return ORBG_OK;
}

extern "C" int orbg_batch_matches(orbg_ctx *c, int32_t *d_out, int32_t *frame_cap)
{
    if (!c || !c->gw || c->last_n <= 0) return set_err(ORBG_EINVAL, "no batch");
    if (!c->last_npairs) return set_err(ORBG_EINVAL, "no match batch yet");
    if (frame_cap) *frame_cap = c->geom.frame_cap;
    if (!d_out) return ORBG_OK;
    const int s = c->slot;
    HIPCHK(order_after_caller(c));
    HIPCHK(hipStreamWaitEvent(c->mstream, c->ev_ext[s], 0));
    int rc = launch_match_export(c->mstream, c->d_m12, c->d_pairs, c->d_counts,
                                 c->geom.frame_cap, c->last_npairs, d_out);
    if (rc) return set_err(rc, "k_match_export launch failed");
    HIPCHK(hipEventRecord(c->ev_mat[s], c->mstream));
    c->mat_pending[s] = true;
    return ORBG_OK;
}

extern "C" int orbg_profile_enable(orbg_ctx *c, int enable)
{
    if (!c) return set_err(ORBG_EINVAL, "ctx is NULL");
    c->prof.on = enable != 0;
    return ORBG_OK;
}

extern "C" int orbg_profile_read(orbg_ctx *c, int i, const char **name, double *total_ms,
                                 int64_t *launches)
{
    if (!c) return set_err(ORBG_EINVAL, "ctx is NULL");
    c->prof.collect();
    const int n = (int)c->prof.kinds.size();
    if (i >= 0 && i < n) {
        if (name) *name = c->prof.kinds[i].name;
        if (total_ms) *total_ms = c->prof.kinds[i].total_ms;
        if (launches) *launches = c->prof.kinds[i].launches;
    }
    return n;
}

extern "C" int orbg_profile_reset(orbg_ctx *c)
{
    if (!c) return set_err(ORBG_EINVAL, "ctx is NULL");
    c->prof.collect();
    for (auto &k : c->prof.kinds) {
        k.total_ms = 0;
        k.launches = 0;
    }
    return ORBG_OK;
}

// ---------------------------------------------------------------------------
// matcher
// ---------------------------------------------------------------------------
extern "C" int orbg_descriptor_distance(const uint8_t *a, const uint8_t *b)
{
    int d = 0;
    for (int i = 0; i < 8; i++) {
        uint32_t x, y;
        memcpy(&x, a + 4 * i, 4);
        memcpy(&y, b + 4 * i, 4);
        d += __builtin_popcount(x ^ y);
    }
    return d;
}

static int scratch(orbg_ctx *c, size_t bytes, void **p)
{
    if (c->scr_bytes < bytes) {
        if (c->d_scr) hipFree(c->d_scr);
        c->d_scr = nullptr;
        c->scr_bytes = 0;
        hipError_t e = hipMalloc(&c->d_scr, bytes);
        if (e != hipSuccess) return set_err(ORBG_ENOMEM, "scratch %zu bytes", bytes);
        c->scr_bytes = bytes;
    }
    *p = c->d_scr;
    return ORBG_OK;
}

static size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

extern "C" int orbg_match_batch_device(orbg_ctx *c, const int32_t *f1, const int32_t *f2,
                                       int npairs, int window, float nnratio, int check_ori)
{
    if (!c || !c->gw || c->last_n <= 0) return set_err(ORBG_EINVAL, "no batch extracted");
    if (npairs <= 0 || !f1 || !f2) return set_err(ORBG_EINVAL, "no pairs");
    for (int i = 0; i < npairs; i++)
        if (f1[i] < 0 || f1[i] >= c->last_n || f2[i] < 0 || f2[i] >= c->last_n)
            return set_err(ORBG_EINVAL, "pair %d references a frame outside the batch", i);
    HIPCHK(hipSetDevice(c->device));
    const size_t fc = (size_t)c->geom.frame_cap;
    if (c->pair_cap < npairs) {
        int rs = sync_all(c);  // an earlier match may still read the buffers
        if (rs) return rs;
        c->h_pairs.clear();
        hipFree(c->d_pairs);
        hipFree(c->d_knn);
        hipFree(c->d_m12);
        hipFree(c->d_nm);
        hipFree(c->d_topk);
        hipFree(c->d_topk_n);
        c->d_pairs = nullptr;
        c->d_knn = c->d_m12 = c->d_nm = nullptr;
        c->d_topk = nullptr;
        c->d_topk_n = nullptr;
        c->pair_cap = 0;
        int rc;
        const size_t P = (size_t)std::max(npairs, c->gbatch);
        if ((rc = dalloc(&c->d_pairs, 2 * P)) || (rc = dalloc(&c->d_knn, P * fc * 3)) ||
            (rc = dalloc(&c->d_m12, P * fc)) || (rc = dalloc(&c->d_nm, P)) ||
            (rc = dalloc(&c->d_topk, P * fc * ORBG_MATCH_TOPK * 2)) ||
            (rc = dalloc(&c->d_topk_n, P * fc)))
            return rc;
        c->pair_cap = (int)P;
    }
    // upload the pair lists only when they change (the bench reuses them every step)
    std::vector<int32_t> hp(f1, f1 + npairs);
    hp.insert(hp.end(), f2, f2 + npairs);
    if (hp != c->h_pairs) {
        HIPCHK(hipStreamSynchronize(c->mstream));  // the previous match reads d_pairs
        HIPCHK(hipMemcpy(c->d_pairs, f1, npairs * sizeof(int32_t), hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(c->d_pairs + c->pair_cap, f2, npairs * sizeof(int32_t),
                         hipMemcpyHostToDevice));
        c->h_pairs.swap(hp);
    }
    const int s = c->slot;
    HIPCHK(hipStreamWaitEvent(c->mstream, c->ev_ext[s], 0));
    // mvKeysUn and the image bounds (Frame.cc:259, 575-611): the keypoints themselves and
    // (0, w, 0, h) unless orbg_set_camera gave a distorted camera
    const orbg_keypoint *kun = c->d_kps;
    orbg_bounds b{0.f, (float)c->geom.w, 0.f, (float)c->geom.h};
    c->kps_un_valid = false;
    if (c->has_cam) {
        const size_t need = (size_t)c->last_n * fc;
        if (c->kps_un_n < need) {
            HIPCHK(hipStreamSynchronize(c->mstream));  // an earlier match may still read it
            if (c->d_kps_un) hipFree(c->d_kps_un);
            c->d_kps_un = nullptr;
            c->kps_un_n = 0;
            int ra = dalloc(&c->d_kps_un, need);
            if (ra) return ra;
            c->kps_un_n = need;
        }
        int ru = 0;
        hipStream_t st = c->mstream;  // PROF_LAUNCH records on `st`
        PROF_LAUNCH(c, "undistort",
                    ru = launch_undistort(st, c->cam, c->d_kps, c->d_counts, (int)fc, c->last_n,
                                          c->d_kps_un));
        if (ru) return set_err(ORBG_EIO, "k_undistort launch failed");
        kun = c->d_kps_un;
        orbg_compute_image_bounds(&c->cam, c->geom.w, c->geom.h, &b);
        c->kps_un_valid = true;
    }
    int rc = launch_match_pairs(c->mstream, c->aux_stream, c->ev_fork[1], c->ev_join[1],
                                c->d_desc, kun, c->d_counts, (int)fc, c->d_pairs,
                                c->d_pairs + c->pair_cap, npairs, b, window,
                                nnratio, check_ori, c->d_knn, c->d_m12, c->d_nm, c->d_topk,
                                c->d_topk_n, &c->prof, c->serial || c->geom.dbg == 40,
                                c->geom.lv[0].out_cap);
    if (rc) return rc;
    HIPCHK(hipEventRecord(c->ev_mat[s], c->mstream));
    c->mat_pending[s] = true;
    c->last_npairs = npairs;
    return ORBG_OK;
}

extern "C" int orbg_match_pose_batch_device(orbg_ctx *c, const orbg_pose_camera *cam,
                                            float depth, double *d_q, double *d_t,
                                            int32_t *d_ninliers)
{
    if (!c || !c->gw || c->last_n <= 0) return set_err(ORBG_EINVAL, "no batch extracted");
    if (!c->last_npairs) return set_err(ORBG_EINVAL, "no match batch yet");
    if (!cam || !d_q || !d_t || !d_ninliers) return set_err(ORBG_EINVAL, "NULL argument");
    if (!(depth > 0) || !(cam->fx > 0) || !(cam->fy > 0))
        return set_err(ORBG_EINVAL, "depth, fx, fy must be > 0");
    HIPCHK(hipSetDevice(c->device));
    const int P = c->last_npairs;
    const size_t fc = (size_t)c->geom.frame_cap;
    size_t o = 0;
    const size_t oe = o;
    o += al256((size_t)P * fc * sizeof(orbg_pose_edge));
    const size_t on = o;
    o += al256((size_t)P * 4);
    const size_t oc = o;
    o += al256((size_t)P * sizeof(orbg_pose_camera));
    const size_t ot0 = o;
    o += al256((size_t)P * 48);
    const size_t ot1 = o;
    o += al256((size_t)P * 48);
    const size_t ool = o;
    o += al256((size_t)P * fc);
    if (c->mpose_bytes < o) {
        HIPCHK(hipStreamSynchronize(c->mstream));  // a previous pass may still read it
        if (c->d_mpose) hipFree(c->d_mpose);
        c->d_mpose = nullptr;
        c->mpose_bytes = 0;
        if (hipMalloc(&c->d_mpose, o) != hipSuccess)
            return set_err(ORBG_ENOMEM, "pose scratch %zu bytes", o);
        c->mpose_bytes = o;
    }
    uint8_t *b = (uint8_t *)c->d_mpose;
    const int s = c->slot;
    HIPCHK(order_after_caller(c));  // d_q / d_t / d_ninliers are the caller's
    HIPCHK(hipStreamWaitEvent(c->mstream, c->ev_ext[s], 0));  // (the matching already does)
    const int rc = launch_match_pose(
        c->mstream, c->kps_un_valid ? c->d_kps_un : c->d_kps, c->d_counts, (int)fc, c->d_pairs,
        c->d_pairs + c->pair_cap, c->d_m12, P, *cam, depth, c->inv_sigma2, c->p.nlevels, (orbg_pose_edge *)(b + oe),
        (int32_t *)(b + on), (orbg_pose_camera *)(b + oc), (float *)(b + ot0),
        (float *)(b + ot1), b + ool, d_q, d_t, d_ninliers, &c->prof);
    if (rc) return set_err(rc, "pose stub launch failed");
    HIPCHK(hipEventRecord(c->ev_mat[s], c->mstream));
    c->mat_pending[s] = true;
    return ORBG_OK;
}

extern "C" int orbg_stereo_batch_device(orbg_ctx *c, const int32_t *left, const int32_t *right,
                                        int npairs, float bf, float min_z)
{
    if (!c || !c->gw || c->last_n <= 0) return set_err(ORBG_EINVAL, "no batch extracted");
    if (npairs <= 0 || !left || !right) return set_err(ORBG_EINVAL, "no pairs");
    if (!(bf > 0)) return set_err(ORBG_EINVAL, "bf must be > 0");
    for (int i = 0; i < npairs; i++)
        if (left[i] < 0 || left[i] >= c->last_n || right[i] < 0 || right[i] >= c->last_n)
            return set_err(ORBG_EINVAL, "stereo pair %d references a frame outside the batch", i);
    HIPCHK(hipSetDevice(c->device));
    const size_t fc = (size_t)c->geom.frame_cap;
    if (c->stereo_cap < npairs) {
        int rs = sync_all(c);
        if (rs) return rs;
        hipFree(c->d_spairs);
        hipFree(c->d_uright);
        hipFree(c->d_depth);
        hipFree(c->d_snvalid);
        hipFree(c->d_sscr);
        c->h_spairs.clear();
        c->d_spairs = nullptr;
        c->d_uright = c->d_depth = nullptr;
        c->d_snvalid = nullptr;
        c->d_sscr = nullptr;
        c->stereo_cap = 0;
        const size_t P = (size_t)npairs;
        int rc;
        if ((rc = dalloc(&c->d_spairs, 2 * P)) || (rc = dalloc(&c->d_uright, P * fc)) ||
            (rc = dalloc(&c->d_depth, P * fc)) || (rc = dalloc(&c->d_snvalid, P)) ||
            (rc = dalloc((uint8_t **)&c->d_sscr, stereo_scratch_bytes(npairs, (int)fc))))
            return rc;
        c->stereo_cap = npairs;
    }
    // the kernels run on the extraction stream (they read this batch's pyramid, which the
    // next extraction overwrites); the pair lists are uploaded only when they change
    std::vector<int32_t> hp(left, left + npairs);
    hp.insert(hp.end(), right, right + npairs);
    const hipStream_t bs = back_stream(c);
    if (hp != c->h_spairs) {
        HIPCHK(hipStreamSynchronize(bs));  // a previous stereo pass may read them
        if (c->ssum_pending) HIPCHK(hipStreamSynchronize(c->mstream));  // ... or its summary
        if (c->srel_pending) HIPCHK(hipEventSynchronize(c->ev_srel));   // ... or the caller
        c->ssum_pending = c->srel_pending = false;
        HIPCHK(hipMemcpy(c->d_spairs, left, npairs * sizeof(int32_t), hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(c->d_spairs + c->stereo_cap, right, npairs * sizeof(int32_t),
                         hipMemcpyHostToDevice));
        c->h_spairs.swap(hp);
    }
    // the previous batch's summary (match stream) reads d_snvalid, which this pass rewrites
    if (c->ssum_pending) {
        HIPCHK(hipStreamWaitEvent(bs, c->ev_ssum, 0));
        c->ssum_pending = false;
    }
    if (c->srel_pending) {  // the caller's reads of the previous stereo outputs
        HIPCHK(hipStreamWaitEvent(bs, c->ev_srel, 0));
        c->srel_pending = false;
    }
    // pipelined: on the back stream after the batch's descriptors; the slot's next front
    // waits for it (ev_back)
    int rc = launch_stereo(bs, c->geom, c->d_kps, c->d_desc, c->d_counts, c->d_spairs,
                           c->d_spairs + c->stereo_cap, npairs, c->last_img, c->last_fs,
                           c->last_pitch, c->d_pyr, bf, min_z, c->d_sscr, c->d_uright,
                           c->d_depth, c->d_snvalid, &c->prof);
    if (rc) return set_err(rc, "stereo launch failed (level-0 height > 4096?)");
    if (c->last_piped) HIPCHK(hipEventRecord(c->ev_back[c->slot], c->ostream));
    HIPCHK(hipEventRecord(c->ev_sback, bs));
    c->last_nstereo = npairs;
    return ORBG_OK;
}

__global__ void k_stereo_summary(const int32_t *__restrict__ counts,
                                 const int32_t *__restrict__ left,
                                 const int32_t *__restrict__ nvalid, int npairs,
                                 int32_t *__restrict__ out)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < npairs) {
        out[i] = counts[left[i]];
        out[npairs + i] = nvalid[i];
    }
}

extern "C" int orbg_stereo_summary(orbg_ctx *c, int32_t *d_out)
{
    if (!c || !c->last_nstereo || !d_out) return set_err(ORBG_EINVAL, "no stereo batch yet");
    // on the match stream, as orbg_batch_summary: after the stereo pass (ev_sback); the
    // extraction that next rewrites this output slot waits for it (ev_mat), the next stereo
    // pass too (ev_ssum)
    const int s = c->slot;
    HIPCHK(order_after_caller(c));
    HIPCHK(hipStreamWaitEvent(c->mstream, c->ev_sback, 0));
    hipLaunchKernelGGL(k_stereo_summary, dim3((c->last_nstereo + 255) / 256), dim3(256), 0,
                       c->mstream, c->d_counts, c->d_spairs, c->d_snvalid, c->last_nstereo,
                       d_out);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(c->ev_mat[s], c->mstream));
    c->mat_pending[s] = true;
    HIPCHK(hipEventRecord(c->ev_ssum, c->mstream));
    c->ssum_pending = true;
    return ORBG_OK;
}

extern "C" int orbg_stereo_frame(orbg_ctx *c, const uint8_t *left, const uint8_t *right, int w,
                                 int h, size_t step, float bf, float min_z, orbg_keypoint *kps_l,
                                 uint8_t *desc_l, int cap_l, int *n_l, orbg_keypoint *kps_r,
                                 uint8_t *desc_r, int cap_r, int *n_r, float *uright,
                                 float *depth)
{
    if (!c) return set_err(ORBG_EINVAL, "ctx is NULL");
    if (!left || !right || w <= 0 || h <= 0 || step < (size_t)w)
        return set_err(ORBG_EINVAL, "bad stereo images");
    HIPCHK(hipSetDevice(c->device));
    int rc = plan(c, w, h, std::max(2, c->p.max_batch));
    if (rc) return rc;
    const size_t bytes = (size_t)w * h;
    if (c->img_bytes < 2 * bytes) {
        if (c->d_img) hipFree(c->d_img);
        c->d_img = nullptr;
        c->img_bytes = 0;
        if ((rc = dalloc(&c->d_img, 2 * bytes))) return rc;
        c->img_bytes = 2 * bytes;
    }
    // Frame.cc:110-113 extracts both images (two threads), then ComputeStereoMatches
    HIPCHK(hipMemcpy2DAsync(c->d_img, w, left, step, w, h, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpy2DAsync(c->d_img + bytes, w, right, step, w, h, hipMemcpyHostToDevice,
                            c->stream));
    if ((rc = launch_extract(c, c->d_img, 2, w, (int64_t)bytes))) return rc;
    const int32_t l0 = 0, r1 = 1;
    if ((rc = orbg_stereo_batch_device(c, &l0, &r1, 1, bf, min_z))) return rc;
    int nl = 0, nr = 0;
    rc = orbg_download_frame(c, 0, kps_l, desc_l, cap_l, &nl);
    if (n_l) *n_l = nl;
    if (rc) return rc;
    rc = orbg_download_frame(c, 1, kps_r, desc_r, cap_r, &nr);
    if (n_r) *n_r = nr;
    if (rc) return rc;
    return orbg_download_stereo(c, 0, uright, depth, nl, nullptr);
}

extern "C" int orbg_stereo_outputs(orbg_ctx *c, float **d_uright, float **d_depth,
                                   int32_t **d_nvalid, int32_t *frame_cap)
{
    if (!c || !c->last_nstereo) return set_err(ORBG_EINVAL, "no stereo batch yet");
    if (d_uright) *d_uright = c->d_uright;
    if (d_depth) *d_depth = c->d_depth;
    if (d_nvalid) *d_nvalid = c->d_snvalid;
    if (frame_cap) *frame_cap = c->geom.frame_cap;
    return ORBG_OK;
}

extern "C" int orbg_download_stereo(orbg_ctx *c, int pair, float *uright, float *depth, int cap,
                                    int32_t *nvalid)
{
    if (!c || pair < 0 || pair >= c->last_nstereo) return set_err(ORBG_EINVAL, "bad pair");
    int rc = sync_all(c);
    if (rc) return rc;
    const size_t fc = (size_t)c->geom.frame_cap;
    if (uright)
        HIPCHK(hipMemcpy(uright, c->d_uright + pair * fc, (size_t)cap * sizeof(float),
                         hipMemcpyDeviceToHost));
    if (depth)
        HIPCHK(hipMemcpy(depth, c->d_depth + pair * fc, (size_t)cap * sizeof(float),
                         hipMemcpyDeviceToHost));
    if (nvalid)
        HIPCHK(hipMemcpy(nvalid, c->d_snvalid + pair, sizeof(int32_t), hipMemcpyDeviceToHost));
    return ORBG_OK;
}

extern "C" int orbg_match_outputs(orbg_ctx *c, int32_t **d_knn, int32_t **d_m12, int32_t **d_nm,
                                  int32_t *frame_cap)
{
    if (!c || !c->last_npairs) return set_err(ORBG_EINVAL, "no match batch yet");
    if (d_knn) *d_knn = c->d_knn;
    if (d_m12) *d_m12 = c->d_m12;
    if (d_nm) *d_nm = c->d_nm;
    if (frame_cap) *frame_cap = c->geom.frame_cap;
    return ORBG_OK;
}

extern "C" int orbg_download_matches(orbg_ctx *c, int pair, int32_t *knn, int32_t *m12, int cap,
                                     int32_t *nmatches)
{
    if (!c || pair < 0 || pair >= c->last_npairs) return set_err(ORBG_EINVAL, "bad pair");
    int rc0 = sync_all(c);
    if (rc0) return rc0;
    c->prof.collect();
    const size_t fc = (size_t)c->geom.frame_cap;
    const int n = std::min(cap, (int)fc);
    if (knn) HIPCHK(hipMemcpy(knn, c->d_knn + pair * fc * 3, (size_t)n * 3 * 4, hipMemcpyDeviceToHost));
    if (m12) HIPCHK(hipMemcpy(m12, c->d_m12 + pair * fc, (size_t)n * 4, hipMemcpyDeviceToHost));
    if (nmatches) HIPCHK(hipMemcpy(nmatches, c->d_nm + pair, 4, hipMemcpyDeviceToHost));
    return ORBG_OK;
}

extern "C" int orbg_hamming_knn2(orbg_ctx *c, const uint8_t *qdesc, int nq, const uint8_t *tdesc,
                                 int nt, int32_t *best_idx, int32_t *best_dist,
                                 int32_t *second_dist)
{
    if (!c) return set_err(ORBG_EINVAL, "ctx is NULL");
    if (nq < 0 || nt < 0) return set_err(ORBG_EINVAL, "negative size");
    if (nq == 0) return ORBG_OK;
    HIPCHK(hipSetDevice(c->device));
    // the MFMA kernel keys train indices in 13 bits: train sets past that run in chunks of
    // KNN_CHUNK, merged here in chunk order (lowest index wins ties, as in the in-order scan)
    const int KNN_CHUNK = 8191;
    const int nch = std::max(1, (nt + KNN_CHUNK - 1) / KNN_CHUNK);
    const size_t oq = 0, ot = al256((size_t)nq * 32), oo = ot + al256((size_t)std::max(nt, 1) * 32);
    const size_t bytes = oo + al256((size_t)nq * 12 * nch);
    void *s;
    int rc = scratch(c, bytes, &s);
    if (rc) return rc;
    uint8_t *b = (uint8_t *)s;
    HIPCHK(hipMemcpyAsync(b + oq, qdesc, (size_t)nq * 32, hipMemcpyHostToDevice, c->stream));
    if (nt) HIPCHK(hipMemcpyAsync(b + ot, tdesc, (size_t)nt * 32, hipMemcpyHostToDevice, c->stream));
    for (int k = 0; k < nch; k++) {
        const int t0 = k * KNN_CHUNK, tn = std::min(KNN_CHUNK, nt - t0);
        if ((rc = launch_knn2(c->stream, b + oq, nq, b + ot + (size_t)t0 * 32, std::max(tn, 0),
                              (int32_t *)(b + oo) + (size_t)k * nq * 3, &c->prof)))
            return rc;
    }
    std::vector<int32_t> out((size_t)nq * 3 * nch);
    HIPCHK(hipMemcpyAsync(out.data(), b + oo, out.size() * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    c->prof.collect();
    for (int i = 0; i < nq; i++) {
        int bi = out[3 * i], bd = out[3 * i + 1], sd = out[3 * i + 2];
        for (int k = 1; k < nch; k++) {
            const int32_t *o = &out[((size_t)k * nq + i) * 3];
            if (o[1] < bd) {  // a later chunk's best is strictly better
                sd = std::min(bd, o[2]);
                bd = o[1];
                bi = o[0] + k * KNN_CHUNK;
            } else {
                sd = std::min(sd, o[1]);
            }
        }
        if (best_idx) best_idx[i] = bi;
        if (best_dist) best_dist[i] = bd;
        if (second_dist) second_dist[i] = sd;
    }
    return ORBG_OK;
}

extern "C" int orbg_search_for_initialization(orbg_ctx *c, const orbg_keypoint *kps1,
                                              const uint8_t *desc1, int n1,
                                              const orbg_keypoint *kps2, const uint8_t *desc2,
                                              int n2, const orbg_bounds *bounds2,
                                              float *prev_xy, int32_t *matches12, int window,
                                              float nnratio, int check_ori, int *nmatches)
{
    if (!c || !bounds2) return set_err(ORBG_EINVAL, "NULL argument");
    if (n1 < 0 || n2 < 0) return set_err(ORBG_EINVAL, "negative size");
    if (nmatches) *nmatches = 0;
    if (n1 == 0) return ORBG_OK;
    HIPCHK(hipSetDevice(c->device));
    // the search reads level-0 keypoints only (ORBmatcher.cc:509-512): the kernels work on
    // indices up to the last level-0 keypoint of either frame (the level-major extractor
    // order puts them first; any order is handled), so only those rows go up and only their
    // vbPrevMatched entries come back (the rest are not read or written)
    int last0 = 0;
    for (int i = n1 - 1; i >= 0; i--)
        if (kps1[i].octave == 0) {
            last0 = std::max(last0, i + 1);
            break;
        }
    for (int i = n2 - 1; i >= 0; i--)
        if (kps2[i].octave == 0) {
            last0 = std::max(last0, i + 1);
            break;
        }
    last0 = std::max(last0, 1);
    const size_t m1 = (size_t)n1, l1 = (size_t)std::min(n1, last0);
    const size_t l2 = (size_t)std::max(std::min(n2, last0), 1);
    size_t o = 0;
    const size_t ok1 = o;
    o += al256(l1 * sizeof(orbg_keypoint));
    const size_t od1 = o;
    o += al256(l1 * 32);
    const size_t ok2 = o;
    o += al256(l2 * sizeof(orbg_keypoint));
    const size_t od2 = o;
    o += al256(l2 * 32);
    const size_t opv = o;
    o += al256(l1 * 8);
    const size_t om = o;
    o += al256(m1 * 4 + 4);
    const size_t otk = o;
    o += al256(l1 * 8 * ORBG_MATCH_TOPK);
    const size_t otn = o;
    o += al256(l1 * 4);
    void *s;
    int rc = scratch(c, o, &s);
    if (rc) return rc;
    uint8_t *b = (uint8_t *)s;
    // inputs packed into pinned staging with the device layout, one DMA each way; zero-copy:
    // the staging is the coherent host block, uploaded by k_copy16, and the resolver writes
    // vnMatches12, the count and vbPrevMatched straight back into it
    const bool zc = use_zc(c);
    uint8_t *hs, *hd = nullptr;
    if ((rc = zc ? zc_buf(c, otk, &hs, &hd) : stage(c, otk, &hs))) return rc;
    HIPCHK(hipStreamSynchronize(c->stream));  // the staging buffer's previous user is done
    std::memcpy(hs + ok1, kps1, l1 * sizeof(orbg_keypoint));
    std::memcpy(hs + od1, desc1, l1 * 32);
    if (n2) {
        const size_t c2 = (size_t)std::min(n2, last0);
        std::memcpy(hs + ok2, kps2, c2 * sizeof(orbg_keypoint));
        std::memcpy(hs + od2, desc2, c2 * 32);
    }
    std::memcpy(hs + opv, prev_xy, l1 * 8);
    if (zc) {
        const size_t n16 = om / 16;  // om: a multiple of 256
        hipLaunchKernelGGL(k_copy16, dim3((unsigned)std::min<size_t>((n16 + 255) / 256, 256)),
                           dim3(256), 0, c->stream, (const uint4 *)hd, (uint4 *)b, n16);
        HIPCHK(hipGetLastError());
    } else {
        HIPCHK(hipMemcpyAsync(b, hs, om, hipMemcpyHostToDevice, c->stream));
    }
    // outputs: device copies behind one D2H, or the host block itself (zc)
    uint8_t *ob = zc ? hd : b;
    rc = launch_init_match_single(c->stream, (const orbg_keypoint *)(b + ok1), b + od1, n1,
                                  (const orbg_keypoint *)(b + ok2), b + od2, n2, *bounds2,
                                  (const float *)(b + opv), (float *)(ob + opv), (int32_t *)(ob + om),
                                  (int32_t *)(ob + om + m1 * 4), window, nnratio, check_ori,
                                  (uint32_t *)(b + otk), (int32_t *)(b + otn), &c->prof, last0);
    if (rc) return rc;
    int32_t nm = 0;
    if (!zc) HIPCHK(hipMemcpyAsync(hs + opv, b + opv, otk - opv, hipMemcpyDeviceToHost, c->stream));
    if ((rc = spin_sync(c->stream))) return rc;
    std::memcpy(matches12, hs + om, m1 * 4);
    std::memcpy(&nm, hs + om + m1 * 4, 4);
    std::memcpy(prev_xy, hs + opv, l1 * 8);
    c->prof.collect();
    if (nmatches) *nmatches = nm;
    return ORBG_OK;
}

// ---------------------------------------------------------------------------
// local BA
// ---------------------------------------------------------------------------
static int ba_check_edges(const orbg_edge *edges, int nedge, int npose, int npoint)
{
    for (int i = 0; i < nedge; i++)
        if (edges[i].pose < 0 || edges[i].pose >= npose || edges[i].point < 0 ||
            edges[i].point >= npoint)
            return set_err(ORBG_EINVAL, "edge %d references a missing vertex", i);
    return ORBG_OK;
}

extern "C" int orbg_ba_linearize(orbg_ctx *c, const orbg_pose *poses, int npose,
                                 const double *points, int npoint, const orbg_edge *edges,
                                 int nedge, orbg_edge_out *eout, double *hpose, double *bpose,
                                 double *hpoint, double *bpoint)
{
    if (!c) return set_err(ORBG_EINVAL, "ctx is NULL");
    if (npose < 0 || npoint < 0 || nedge < 0) return set_err(ORBG_EINVAL, "negative size");
    if (int rc0 = ba_check_edges(edges, nedge, npose, npoint)) return rc0;
    HIPCHK(hipSetDevice(c->device));
    // edge lists per pose and per point (CSR): MFMA pose blocks, summed point blocks
    std::vector<int32_t> off(npose + 1, 0), pe(nedge > 0 ? nedge : 1);
    std::vector<int32_t> qoff(npoint + 1, 0), qe(nedge > 0 ? nedge : 1);
    for (int i = 0; i < nedge; i++) {
        off[edges[i].pose + 1]++;
        qoff[edges[i].point + 1]++;
    }
    for (int p = 0; p < npose; p++) off[p + 1] += off[p];
    for (int q = 0; q < npoint; q++) qoff[q + 1] += qoff[q];
    {
        std::vector<int32_t> fill(off.begin(), off.end() - 1), qfill(qoff.begin(), qoff.end() - 1);
        for (int i = 0; i < nedge; i++) {
            pe[fill[edges[i].pose]++] = i;
            qe[qfill[edges[i].point]++] = i;
        }
    }
    const size_t sb = ba_scratch_bytes(npose, npoint, nedge);
    void *s;
    int rc = scratch(c, sb, &s);
    if (rc) return rc;
    rc = launch_ba(c->stream, poses, npose, points, npoint, edges, nedge, off.data(), pe.data(),
                   qoff.data(), qe.data(), eout, hpose, bpose, hpoint, bpoint, s, &c->prof);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(c->stream));
    c->prof.collect();
    return ORBG_OK;
}

extern "C" int orbg_ba_errors(orbg_ctx *c, const orbg_pose *poses, int npose, const double *points,
                              int npoint, const orbg_edge *edges, int nedge, double *err,
                              double *chi2, double *rho0, uint8_t *depth_ok,
                              double *active_robust_chi2)
{
    if (!c) return set_err(ORBG_EINVAL, "ctx is NULL");
    if (npose < 0 || npoint < 0 || nedge < 0) return set_err(ORBG_EINVAL, "negative size");
    if (nedge && (!poses || !points || !edges)) return set_err(ORBG_EINVAL, "NULL array");
    int rc = ba_check_edges(edges, nedge, npose, npoint);
    if (rc) return rc;
    if (active_robust_chi2) *active_robust_chi2 = 0;
    if (nedge == 0) return ORBG_OK;
    HIPCHK(hipSetDevice(c->device));
    const size_t ne = (size_t)nedge;
    size_t o = 0;
    const size_t opo = o;
    o += al256((size_t)npose * sizeof(orbg_pose));
    const size_t opt = o;
    o += al256((size_t)npoint * 24);
    const size_t oed = o;
    o += al256(ne * sizeof(orbg_edge));
    const size_t oer = o;  // outputs: err, chi2, rho0, depth_ok (one D2H copy)
    o += al256(ne * 24);
    const size_t och = o;
    o += al256(ne * 8);
    const size_t orh = o;
    o += al256(ne * 8);
    const size_t odk = o;
    o += al256(ne);
    void *sp;
    if ((rc = scratch(c, o, &sp))) return rc;
    uint8_t *b = (uint8_t *)sp;
    HIPCHK(hipMemcpyAsync(b + opo, poses, (size_t)npose * sizeof(orbg_pose), hipMemcpyHostToDevice,
                          c->stream));
    HIPCHK(hipMemcpyAsync(b + opt, points, (size_t)npoint * 24, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(b + oed, edges, ne * sizeof(orbg_edge), hipMemcpyHostToDevice, c->stream));
    if ((rc = launch_ba_errors(c->stream, (const orbg_pose *)(b + opo), (const double *)(b + opt),
                               (const orbg_edge *)(b + oed), nedge, (double *)(b + oer),
                               (double *)(b + och), (double *)(b + orh), b + odk, &c->prof)))
        return set_err(ORBG_EIO, "k_ba_errors launch failed");
    std::vector<uint8_t> h(o - oer);
    HIPCHK(hipMemcpyAsync(h.data(), b + oer, h.size(), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    c->prof.collect();
    const double *herr = (const double *)h.data(), *hchi = (const double *)(h.data() + och - oer),
                 *hrho = (const double *)(h.data() + orh - oer);
    const uint8_t *hdk = h.data() + odk - oer;
    if (err) std::memcpy(err, herr, ne * 24);
    if (chi2) std::memcpy(chi2, hchi, ne * 8);
    if (rho0) std::memcpy(rho0, hrho, ne * 8);
    if (depth_ok) std::memcpy(depth_ok, hdk, ne);
    if (active_robust_chi2) {
        // activeRobustChi2's sum, in the caller's edge order (sparse_optimizer.cpp:100-114)
        double t = 0;
        for (int i = 0; i < nedge; i++)
            if (edges[i].active) t += hrho[i];
        *active_robust_chi2 = t;
    }
    return ORBG_OK;
}

extern "C" int orbg_ba_errors_device(orbg_ctx *c, const orbg_pose *d_poses,
                                     const double *d_points, const orbg_edge *d_edges, int nedge,
                                     double *d_err, double *d_chi2, double *d_rho0,
                                     uint8_t *d_depth_ok)
{
    if (!c) return set_err(ORBG_EINVAL, "ctx is NULL");
    if (nedge < 0) return set_err(ORBG_EINVAL, "negative size");
    if (nedge && (!d_poses || !d_points || !d_edges || !d_chi2))
        return set_err(ORBG_EINVAL, "NULL device array");
    HIPCHK(hipSetDevice(c->device));
    if (launch_ba_errors(c->stream, d_poses, d_points, d_edges, nedge, d_err, d_chi2, d_rho0,
                         d_depth_ok, &c->prof))
        return set_err(ORBG_EIO, "k_ba_errors launch failed");
    return ORBG_OK;
}

extern "C" int orbg_ba_set_jacobians(orbg_ctx *c, int enable)
{
    if (!c) return set_err(ORBG_EINVAL, "ctx is NULL");
    c->ba_jacobians = enable != 0;
    return ORBG_OK;
}

extern "C" int orbg_ba_set_edge_errors(orbg_ctx *c, int enable)
{
    if (!c) return set_err(ORBG_EINVAL, "ctx is NULL");
    c->ba_edge_errors = enable != 0;
    return ORBG_OK;
}

extern "C" int orbg_ba_linearize_device(orbg_ctx *c, const orbg_pose *d_poses, int npose,
                                        const double *d_points, int npoint,
                                        const orbg_edge *d_edges, int nedge,
                                        const int32_t *d_pose_off, const int32_t *d_pose_edges,
                                        const int32_t *d_point_off,
                                        const int32_t *d_point_edges, orbg_edge_out *d_eout,
                                        double *d_hpose, double *d_bpose, double *d_hpoint,
                                        double *d_bpoint)
{
    if (!c) return set_err(ORBG_EINVAL, "ctx is NULL");
    if (npose < 0 || npoint < 0 || nedge < 0) return set_err(ORBG_EINVAL, "negative size");
    if ((nedge && (!d_edges || !d_eout)) || (npose && (!d_poses || !d_pose_off || !d_pose_edges ||
                                                       !d_hpose || !d_bpose)) ||
        (npoint && (!d_points || !d_hpoint || !d_bpoint || !d_point_off || !d_point_edges)))
        return set_err(ORBG_EINVAL, "NULL device array");
    HIPCHK(hipSetDevice(c->device));
    void *s;
    int rc = scratch(c, ba_rows_bytes(nedge, npose), &s);
    if (rc) return rc;
    rc = launch_ba_device(c->stream, d_poses, npose, d_points, npoint, d_edges, nedge, d_pose_off,
                          d_pose_edges, d_point_off, d_point_edges, d_eout, d_hpose, d_bpose,
                          d_hpoint, d_bpoint, (double *)s, &c->prof, c->ba_jacobians,
                          c->ba_edge_errors, nullptr);
    if (rc) return set_err(ORBG_EIO, "BA kernel launch failed");
    return ORBG_OK;
}

extern "C" int orbg_ba_build_system_device(orbg_ctx *c, const orbg_pose *d_poses, int npose,
                                           const double *d_points, int npoint,
                                           const orbg_edge *d_edges, int nedge,
                                           const int32_t *d_pose_off, const int32_t *d_pose_edges,
                                           const int32_t *d_point_off,
                                           const int32_t *d_point_edges, double *d_hpl,
                                           double *d_hpose, double *d_bpose, double *d_hpoint,
                                           double *d_bpoint)
{
    if (!c) return set_err(ORBG_EINVAL, "ctx is NULL");
    if (npose < 0 || npoint < 0 || nedge < 0) return set_err(ORBG_EINVAL, "negative size");
    if ((nedge && (!d_edges || !d_hpl)) || (npose && (!d_poses || !d_pose_off || !d_pose_edges ||
                                                      !d_hpose || !d_bpose)) ||
        (npoint && (!d_points || !d_hpoint || !d_bpoint || !d_point_off || !d_point_edges)))
        return set_err(ORBG_EINVAL, "NULL device array");
    HIPCHK(hipSetDevice(c->device));
    void *s;
    int rc = scratch(c, ba_rows_bytes(nedge, npose), &s);
    if (rc) return rc;
    rc = launch_ba_device(c->stream, d_poses, npose, d_points, npoint, d_edges, nedge, d_pose_off,
                          d_pose_edges, d_point_off, d_point_edges, nullptr, d_hpose, d_bpose,
                          d_hpoint, d_bpoint, (double *)s, &c->prof, false, false, d_hpl);
    if (rc) return set_err(ORBG_EIO, "BA kernel launch failed");
    return ORBG_OK;
}

// ---------------------------------------------------------------------------
// orbg_ba_graph: a device-resident LBA edge set, packed (orbg_internal.h BaPackedEdge)
// ---------------------------------------------------------------------------
struct orbg_ba_graph {
    int device = 0, nedge = 0, npose = 0, npoint = 0;
    std::vector<BaPackedEdge> h;  // host copy (orbg_ba_graph_set_active rewrites the flags)
    // orbg_ba_graph_set_active uploads from pinned staging with no host synchronisation; the
    // next call waits for the previous upload (ev_up) before rewriting the staging buffer
    BaPackedEdge *h_pin = nullptr;
    hipEvent_t ev_up = nullptr;
    bool up_pending = false;
    BaPackedEdge *d_edges = nullptr;
    BaCam *d_cam = nullptr;
    BaInfo *d_info = nullptr;
    int32_t *d_off = nullptr, *d_pe = nullptr, *d_qoff = nullptr, *d_qe = nullptr;
    // the build's precomputed structure (BaGraphDev, orbg_internal.h)
    int32_t *d_special = nullptr, *d_slice_off = nullptr, *d_slice_pose = nullptr;
    double *d_part = nullptr;
    BaGraphDev gd{};
    // the Schur solve's structure (orbg_ba_graph_schur_plan), rebuilt by set_active
    bool schur_planned = false;
    std::vector<uint8_t> fixed;  // the plan's fixed-pose flags
    uint8_t *d_schur = nullptr;  // structure + scratch (schur_layout)
    size_t schur_bytes = 0;
    SchurArgs sa{};
    // orbg_ba_graph_optimize's workspace (allocated on first use): the system, the errors,
    // the increments, the pushed estimates and the reductions' scalars
    uint8_t *d_lm = nullptr;
};

static size_t schur_layout(const SchurPlanHost &P, int nedge, uint8_t *base, SchurArgs &A,
                           size_t *structure_bytes);
static int schur_upload(const SchurPlanHost &P, const SchurArgs &A, hipStream_t st);

// (re)build an orbg_ba_graph's Schur structure from its host edges and the stored fixed
// flags, and upload it in stream order (no host synchronisation unless the buffer grows)
static int ba_graph_schur_replan(orbg_ctx *c, orbg_ba_graph *g)
{
    const int ne = g->nedge;
    std::vector<int32_t> ep(std::max(ne, 1)), eq(std::max(ne, 1));
    std::vector<uint8_t> ea(std::max(ne, 1));
    for (int e = 0; e < ne; e++) {
        ep[e] = g->h[e].pose;
        eq[e] = g->h[e].point;
        ea[e] = (g->h[e].flags & 4u) ? 1 : 0;
    }
    SchurPlanHost P;
    build_schur_plan(g->npose, g->npoint, ne, ep.data(), eq.data(), ea.data(), g->fixed.data(), P);
    SchurArgs A{};
    const size_t bytes = schur_layout(P, ne, nullptr, A, nullptr);
    if (bytes > g->schur_bytes) {
        if (g->d_schur) {
            HIPCHK(hipStreamSynchronize(c->stream));  // a queued solve may still read it
            hipFree(g->d_schur);
        }
        g->d_schur = nullptr;
        g->schur_bytes = 0;
        if (hipMalloc((void **)&g->d_schur, bytes) != hipSuccess)
            return set_err(ORBG_ENOMEM, "Schur structure %zu bytes", bytes);
        g->schur_bytes = bytes;
    }
    schur_layout(P, ne, g->d_schur, A, nullptr);
    int rc = schur_upload(P, A, c->stream);
    if (rc) return rc;
    g->sa = A;
    g->schur_planned = true;
    return ORBG_OK;
}

static void ba_graph_free(orbg_ba_graph *g)
{
    if (!g) return;
    hipSetDevice(g->device);
    if (g->ev_up) {
        if (g->up_pending) hipEventSynchronize(g->ev_up);
        hipEventDestroy(g->ev_up);
    }
    if (g->h_pin) hipHostFree(g->h_pin);
    for (void *p : {(void *)g->d_edges, (void *)g->d_cam, (void *)g->d_info, (void *)g->d_off,
                    (void *)g->d_pe, (void *)g->d_qoff, (void *)g->d_qe, (void *)g->d_special,
                    (void *)g->d_slice_off, (void *)g->d_slice_pose, (void *)g->d_part,
                    (void *)g->d_schur, (void *)g->d_lm})
        if (p) hipFree(p);
    delete g;
}

extern "C" int orbg_ba_graph_create(orbg_ctx *c, const orbg_edge *edges, int nedge, int npose,
                                    int npoint, orbg_ba_graph **out)
{
    if (!c || !out) return set_err(ORBG_EINVAL, "ctx / out is NULL");
    *out = nullptr;
    if (npose < 0 || npoint < 0 || nedge < 0) return set_err(ORBG_EINVAL, "negative size");
    if (nedge && !edges) return set_err(ORBG_EINVAL, "edges is NULL");
    if (int rc0 = ba_check_edges(edges, nedge, npose, npoint)) return rc0;
    // dedup the camera and (information, Huber delta) values by their bits; the observations
    // must survive the f32 store exactly (the mono third entry is never read: stored as 0)
    std::map<std::array<uint64_t, 5>, int> cams;
    std::map<std::array<uint64_t, 2>, int> infos;
    std::vector<BaCam> hc;
    std::vector<BaInfo> hi;
    std::vector<BaPackedEdge> h((size_t)(nedge > 0 ? nedge : 1));
    auto bits = [](double v) {
        uint64_t u;
        memcpy(&u, &v, 8);
        return u;
    };
    for (int i = 0; i < nedge; i++) {
        const orbg_edge &e = edges[i];
        const std::array<uint64_t, 5> ck = {bits(e.fx), bits(e.fy), bits(e.cx), bits(e.cy), bits(e.bf)};
        auto ci = cams.find(ck);
        if (ci == cams.end()) {
            if ((int)hc.size() >= ORBG_BA_MAX_CAMS)
                return set_err(ORBG_ENOTSUP, "more than %d distinct cameras", ORBG_BA_MAX_CAMS);
            ci = cams.emplace(ck, (int)hc.size()).first;
            hc.push_back(BaCam{e.fx, e.fy, e.cx, e.cy, e.bf});
        }
        const std::array<uint64_t, 2> ik = {bits(e.inv_sigma2), bits(e.huber_delta)};
        auto ii = infos.find(ik);
        if (ii == infos.end()) {
            if ((int)hi.size() >= ORBG_BA_MAX_INFOS)
                return set_err(ORBG_ENOTSUP, "more than %d distinct (inv_sigma2, huber_delta)",
                               ORBG_BA_MAX_INFOS);
            ii = infos.emplace(ik, (int)hi.size()).first;
            hi.push_back(BaInfo{e.inv_sigma2, e.huber_delta});
        }
        BaPackedEdge &p = h[i];
        p.point = e.point;
        p.pose = e.pose;
        p.flags = (e.stereo ? 1u : 0u) | (e.robust ? 2u : 0u) | (e.active ? 4u : 0u) |
                  (uint32_t)ci->second << 8 | (uint32_t)ii->second << 16;
        const int nobs = e.stereo ? 3 : 2;
        for (int k = 0; k < 3; k++) {
            const double v = k < nobs ? e.obs[k] : 0.0;
            p.obs[k] = (float)v;
            if ((double)p.obs[k] != v)
                return set_err(ORBG_ENOTSUP, "edge %d observation %d is not f32-exact", i, k);
        }
    }
    // per-vertex edge lists (CSR), as orbg_ba_linearize
    std::vector<int32_t> off(npose + 1, 0), pe(nedge > 0 ? nedge : 1);
    std::vector<int32_t> qoff(npoint + 1, 0), qe(nedge > 0 ? nedge : 1);
    for (int i = 0; i < nedge; i++) {
        off[edges[i].pose + 1]++;
        qoff[edges[i].point + 1]++;
    }
    for (int p = 0; p < npose; p++) off[p + 1] += off[p];
    for (int q = 0; q < npoint; q++) qoff[q + 1] += qoff[q];
    {
        std::vector<int32_t> fill(off.begin(), off.end() - 1), qfill(qoff.begin(), qoff.end() - 1);
        for (int i = 0; i < nedge; i++) {
            pe[fill[edges[i].pose]++] = i;
            qe[qfill[edges[i].point]++] = i;
        }
    }
    // pose slices (ORBG_BA_SLICE edges of one pose each)
    std::vector<int32_t> soff(npose + 1, 0), spose;
    for (int p = 0; p < npose; p++) {
        const int n = (off[p + 1] - off[p] + ORBG_BA_SLICE - 1) / ORBG_BA_SLICE;
        soff[p + 1] = soff[p] + n;
        for (int k = 0; k < n; k++) spose.push_back(p);
    }
    const size_t nsl = spose.size();
    // special points: their point-major slots span two k_ba_edges workgroups, or no edge
    std::vector<int32_t> special;
    for (int q = 0; q < npoint; q++)
        if (qoff[q + 1] == qoff[q] ||
            qoff[q] / ORBG_BA_EDGES_TPB != (qoff[q + 1] - 1) / ORBG_BA_EDGES_TPB)
            special.push_back(q);
    HIPCHK(hipSetDevice(c->device));
    orbg_ba_graph *g = new orbg_ba_graph;
    g->device = c->device;
    g->nedge = nedge;
    g->npose = npose;
    g->npoint = npoint;
    int rc = 0;
    if ((rc = dalloc(&g->d_edges, h.size())) || (rc = dalloc(&g->d_cam, hc.size())) ||
        (rc = dalloc(&g->d_info, hi.size())) || (rc = dalloc(&g->d_off, off.size())) ||
        (rc = dalloc(&g->d_pe, pe.size())) || (rc = dalloc(&g->d_qoff, qoff.size())) ||
        (rc = dalloc(&g->d_qe, qe.size())) ||
        (rc = dalloc(&g->d_special, std::max<size_t>(special.size(), 1))) ||
        (rc = dalloc(&g->d_slice_off, soff.size())) ||
        (rc = dalloc(&g->d_slice_pose, std::max<size_t>(nsl, 1))) ||
        (rc = dalloc(&g->d_part, std::max<size_t>(nsl, 1) * 42))) {
        ba_graph_free(g);
        return rc;
    }
    g->gd.special = g->d_special;
    g->gd.nspecial = (int)special.size();
    g->gd.slice_off = g->d_slice_off;
    g->gd.slice_pose = g->d_slice_pose;
    g->gd.nslice = (int)nsl;
    g->gd.part = g->d_part;
    auto up = [&](void *d, const void *src, size_t n) {
        return n ? hipMemcpyAsync(d, src, n, hipMemcpyHostToDevice, c->stream) : hipSuccess;
    };
    if (up(g->d_edges, h.data(), (size_t)nedge * sizeof(BaPackedEdge)) != hipSuccess ||
        up(g->d_cam, hc.data(), hc.size() * sizeof(BaCam)) != hipSuccess ||
        up(g->d_info, hi.data(), hi.size() * sizeof(BaInfo)) != hipSuccess ||
        up(g->d_off, off.data(), off.size() * 4) != hipSuccess ||
        up(g->d_pe, pe.data(), (size_t)nedge * 4) != hipSuccess ||
        up(g->d_qoff, qoff.data(), qoff.size() * 4) != hipSuccess ||
        up(g->d_qe, qe.data(), (size_t)nedge * 4) != hipSuccess ||
        up(g->d_special, special.data(), special.size() * 4) != hipSuccess ||
        up(g->d_slice_off, soff.data(), soff.size() * 4) != hipSuccess ||
        up(g->d_slice_pose, spose.data(), nsl * 4) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess) {
        ba_graph_free(g);
        return set_err(ORBG_EIO, "graph upload failed");
    }
    g->h = std::move(h);
    *out = g;
    return ORBG_OK;
}

extern "C" int orbg_ba_graph_destroy(orbg_ba_graph *g)
{
    ba_graph_free(g);
    return ORBG_OK;
}

// rewrite flag bit `bit` of every packed edge from v[] and upload the edges in stream order
// after the builds that read the previous flags, from pinned staging: no host
// synchronisation (only the previous upload's, before the staging is rewritten)
static int ba_graph_set_flag(orbg_ctx *c, orbg_ba_graph *g, const uint8_t *v, uint32_t bit)
{
    if (!c || !g) return set_err(ORBG_EINVAL, "ctx / graph is NULL");
    if (g->nedge && !v) return set_err(ORBG_EINVAL, "flag array is NULL");
    if (g->device != c->device) return set_err(ORBG_EINVAL, "graph of another device");
    for (int i = 0; i < g->nedge; i++) g->h[i].flags = (g->h[i].flags & ~bit) | (v[i] ? bit : 0u);
    HIPCHK(hipSetDevice(c->device));
    if (g->nedge) {
        if (!g->h_pin) {
            if (hipHostMalloc((void **)&g->h_pin, (size_t)g->nedge * sizeof(BaPackedEdge),
                              hipHostMallocDefault) != hipSuccess)
                return set_err(ORBG_ENOMEM, "pinned staging of %d edges", g->nedge);
            HIPCHK(hipEventCreateWithFlags(&g->ev_up, hipEventDisableTiming));
        }
        if (g->up_pending) HIPCHK(hipEventSynchronize(g->ev_up));
        memcpy(g->h_pin, g->h.data(), (size_t)g->nedge * sizeof(BaPackedEdge));
        HIPCHK(hipMemcpyAsync(g->d_edges, g->h_pin, (size_t)g->nedge * sizeof(BaPackedEdge),
                              hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipEventRecord(g->ev_up, c->stream));
        g->up_pending = true;
    }
    return ORBG_OK;
}

extern "C" int orbg_ba_graph_set_active(orbg_ctx *c, orbg_ba_graph *g, const uint8_t *active)
{
    int rc = ba_graph_set_flag(c, g, active, 4u);
    if (rc) return rc;
    if (g->schur_planned) return ba_graph_schur_replan(c, g);  // the active set shapes it
    return ORBG_OK;
}

extern "C" int orbg_ba_graph_set_robust(orbg_ctx *c, orbg_ba_graph *g, const uint8_t *robust)
{
    return ba_graph_set_flag(c, g, robust, 2u);
}

extern "C" int orbg_ba_graph_schur_plan(orbg_ctx *c, orbg_ba_graph *g, const uint8_t *fixed)
{
    if (!c || !g) return set_err(ORBG_EINVAL, "ctx / graph is NULL");
    if (g->npose && !fixed) return set_err(ORBG_EINVAL, "fixed is NULL");
    if (g->device != c->device) return set_err(ORBG_EINVAL, "graph of another device");
    HIPCHK(hipSetDevice(c->device));
    g->fixed.assign(std::max(g->npose, 1), 0);
    for (int i = 0; i < g->npose; i++) g->fixed[i] = fixed[i] ? 1 : 0;
    return ba_graph_schur_replan(c, g);
}

extern "C" int orbg_ba_graph_schur_solve(orbg_ctx *c, orbg_ba_graph *g, double lambda,
                                         const double *d_hpl, const double *d_hpose,
                                         const double *d_bpose, const double *d_hpoint,
                                         const double *d_bpoint, double *d_dx_pose,
                                         double *d_dx_point, int32_t *d_ok)
{
    if (!c || !g) return set_err(ORBG_EINVAL, "ctx / graph is NULL");
    if (g->device != c->device) return set_err(ORBG_EINVAL, "graph of another device");
    if (!g->schur_planned) return set_err(ORBG_EINVAL, "orbg_ba_graph_schur_plan not called");
    if (!d_ok || (g->nedge && !d_hpl) || (g->npose && (!d_hpose || !d_bpose || !d_dx_pose)) ||
        (g->npoint && (!d_hpoint || !d_bpoint || !d_dx_point)))
        return set_err(ORBG_EINVAL, "NULL device array");
    HIPCHK(hipSetDevice(c->device));
    SchurArgs A = g->sa;
    A.hpl = d_hpl;
    A.hpl_stride = 18;  // the graph build's compact H_pl [nedge][3][6]
    A.hpose = d_hpose;
    A.bpose = d_bpose;
    A.hpoint = d_hpoint;
    A.bpoint = d_bpoint;
    A.lambda = lambda;
    A.ok = d_ok;
    A.dx_pose = d_dx_pose;
    A.dx_point = d_dx_point;
    const int rc = launch_schur(c->stream, A, &c->prof);
    if (rc) return set_err(rc, "schur launch failed");
    return ORBG_OK;
}

extern "C" int orbg_ba_graph_build_system(orbg_ctx *c, orbg_ba_graph *g, const orbg_pose *d_poses,
                                          const double *d_points, double *d_hpl, double *d_hpose,
                                          double *d_bpose, double *d_hpoint, double *d_bpoint)
{
    if (!c || !g) return set_err(ORBG_EINVAL, "ctx / graph is NULL");
    if (g->device != c->device) return set_err(ORBG_EINVAL, "graph of another device");
    if ((g->nedge && !d_hpl) || (g->npose && (!d_poses || !d_hpose || !d_bpose)) ||
        (g->npoint && (!d_points || !d_hpoint || !d_bpoint)))
        return set_err(ORBG_EINVAL, "NULL device array");
    HIPCHK(hipSetDevice(c->device));
    const int rc = launch_ba_graph(c->stream, d_poses, g->npose, d_points, g->npoint, g->d_edges,
                                   g->d_cam, g->d_info, g->nedge, g->d_off, g->d_pe, g->d_qoff,
                                   g->d_qe, g->gd, d_hpl, d_hpose, d_bpose, d_hpoint, d_bpoint,
                                   &c->prof);
    if (rc) return set_err(ORBG_EIO, "BA kernel launch failed");
    return ORBG_OK;
}

extern "C" int orbg_ba_graph_errors(orbg_ctx *c, orbg_ba_graph *g, const orbg_pose *d_poses,
                                    const double *d_points, double *d_err, double *d_chi2,
                                    double *d_rho0, uint8_t *d_depth_ok)
{
    if (!c || !g) return set_err(ORBG_EINVAL, "ctx / graph is NULL");
    if (g->device != c->device) return set_err(ORBG_EINVAL, "graph of another device");
    if (g->nedge && (!d_poses || !d_points || !d_chi2)) return set_err(ORBG_EINVAL, "NULL device array");
    HIPCHK(hipSetDevice(c->device));
    if (launch_ba_errors_packed(c->stream, d_poses, d_points, g->d_edges, g->d_cam, g->d_info,
                                g->nedge, d_err, d_chi2, d_rho0, d_depth_ok, &c->prof))
        return set_err(ORBG_EIO, "BA error kernel launch failed");
    return ORBG_OK;
}

// g2o's pow(2 rho - 1, 3) as the device's lm_cube (se3_device.h): the exact cube as a
// double-double, rounded once
static double lm_cube_host(double t)
{
    const double h = t * t;
    const double l = std::fma(t, t, -h);
    const double ph = h * t;
    const double pl = std::fma(h, t, -ph);
    return ph + (pl + l * t);
}

extern "C" int orbg_ba_update_device(orbg_ctx *c, const orbg_pose *d_poses, int npose,
                                     const double *d_points, int npoint, const double *d_dx_pose,
                                     const double *d_dx_point, orbg_pose *d_poses_out,
                                     double *d_points_out)
{
    if (!c) return set_err(ORBG_EINVAL, "ctx is NULL");
    if (npose < 0 || npoint < 0) return set_err(ORBG_EINVAL, "negative size");
    if ((npose && (!d_poses || !d_dx_pose || !d_poses_out)) ||
        (npoint && (!d_points || !d_dx_point || !d_points_out)))
        return set_err(ORBG_EINVAL, "NULL device array");
    HIPCHK(hipSetDevice(c->device));
    if (launch_ba_update(c->stream, d_poses, npose, d_points, npoint, d_dx_pose, d_dx_point,
                         d_poses_out, d_points_out))
        return set_err(ORBG_EIO, "k_ba_update launch failed");
    return ORBG_OK;
}

// g2o's SparseOptimizer::optimize(iterations) with OptimizationAlgorithmLevenberg over an
// orbg_ba_graph, the estimates in HBM (see include/orbg.h)
extern "C" int orbg_ba_graph_optimize(orbg_ctx *c, orbg_ba_graph *g, orbg_pose *d_poses,
                                      double *d_points, int iterations, orbg_lm_report *rep)
{
    return orbg_ba_graph_optimize_ctl(c, g, d_poses, d_points, iterations, nullptr, rep);
}

// ... with g2o's force-stop flag (terminate(): before each iteration, sparse_optimizer.cpp:376,
// and after each trial, optimization_algorithm_levenberg.cpp:149) and iteration actions
extern "C" int orbg_ba_graph_optimize_ctl(orbg_ctx *c, orbg_ba_graph *g, orbg_pose *d_poses,
                                          double *d_points, int iterations,
                                          const orbg_lm_control *ctl, orbg_lm_report *rep)
{
    if (!c || !g) return set_err(ORBG_EINVAL, "ctx / graph is NULL");
    if (g->device != c->device) return set_err(ORBG_EINVAL, "graph of another device");
    if (!g->schur_planned) return set_err(ORBG_EINVAL, "orbg_ba_graph_schur_plan not called");
    if ((g->npose && !d_poses) || (g->npoint && !d_points))
        return set_err(ORBG_EINVAL, "NULL device array");
    if (iterations < 0) return set_err(ORBG_EINVAL, "negative iterations");
    HIPCHK(hipSetDevice(c->device));
    const size_t ne = (size_t)std::max(g->nedge, 1), np = (size_t)std::max(g->npose, 1),
                 nq = (size_t)std::max(g->npoint, 1);
    size_t o = 0;
    auto take = [&](size_t bytes) {
        const size_t r = o;
        o += al256(bytes);
        return r;
    };
    const size_t o_hpl = take(ne * 18 * 8), o_hp = take(np * 36 * 8), o_bp = take(np * 6 * 8),
                 o_hq = take(nq * 9 * 8), o_bq = take(nq * 3 * 8), o_chi = take(ne * 8),
                 o_rho = take(ne * 8), o_dxp = take(np * 6 * 8), o_dxq = take(nq * 3 * 8),
                 o_sp = take(np * sizeof(orbg_pose)), o_sq = take(nq * 3 * 8),
                 o_part = take((size_t)lm_reduce_groups() * 8), o_sc = take(4 * 8);
    if (!g->d_lm) {
        hipError_t e = hipMalloc((void **)&g->d_lm, o);
        if (e != hipSuccess) return set_err(ORBG_ENOMEM, "LM workspace %zu bytes", o);
    }
    uint8_t *b = g->d_lm;
    double *hpl = (double *)(b + o_hpl), *hp = (double *)(b + o_hp), *bp = (double *)(b + o_bp),
           *hq = (double *)(b + o_hq), *bq = (double *)(b + o_bq), *chi = (double *)(b + o_chi),
           *rho = (double *)(b + o_rho), *dxp = (double *)(b + o_dxp), *dxq = (double *)(b + o_dxq),
           *sq = (double *)(b + o_sq), *part = (double *)(b + o_part), *sc = (double *)(b + o_sc);
    orbg_pose *sp = (orbg_pose *)(b + o_sp);
    // sc[0] active robust chi2, sc[1] computeScale, sc[2] max |H_jj|, sc[3] the solver's ok
    hipStream_t st = c->stream;
    int rc;
    auto fail = [&](int code, const char *what) { return set_err(code, "LM: %s", what); };
    auto chi2 = [&](double *out) -> int {
        if ((rc = orbg_ba_graph_errors(c, g, d_poses, d_points, nullptr, chi, rho, nullptr)))
            return rc;
        if (launch_lm_reduce(st, 0, g->nedge, 0, 0.0, rho, nullptr, nullptr, nullptr, g->d_edges,
                             part, out))
            return fail(ORBG_EIO, "reduction launch");
        return ORBG_OK;
    };
    auto read = [&](double *h, int n) -> int {
        HIPCHK(hipMemcpyAsync(h, sc, n * sizeof(double), hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        return ORBG_OK;
    };
    orbg_lm_report R{};
    const orbg_lm_control C0{};
    const orbg_lm_control &K = ctl ? *ctl : C0;
    auto terminate = [&]() { return K.force_stop && *K.force_stop != 0; };
    double currentChi = 0.0, lambda = 0.0, hs[4];
    int ni = 2, nBad = 0;
    bool ran = false;
    for (int it = 0; it < iterations && !terminate(); it++) {
        if (it == 0) {  // computeActiveErrors at the start (later: the last accepted trial's)
            if ((rc = chi2(sc)) || (rc = read(hs, 1))) return rc;
            currentChi = hs[0];
            R.initial_chi2 = currentChi;
        }
        ran = true;
        const double iniChi = currentChi;
        if ((rc = orbg_ba_graph_build_system(c, g, d_poses, d_points, hpl, hp, bp, hq, bq))) return rc;
        if (it == 0) {  // computeLambdaInit: tau * max |H_jj| (before any lambda)
            if (launch_lm_reduce(st, 2, 6 * g->npose, 3 * g->npoint, 0.0, hp, hq, nullptr, nullptr,
                                 nullptr, part, sc + 2) ||
                (rc = read(hs, 3)))
                return rc ? rc : fail(ORBG_EIO, "reduction launch");
            lambda = 1e-5 * hs[2];
            ni = 2;
            nBad = 0;
        }
        double rhoLM = 0.0;
        int qmax = 0;
        do {
            // push
            if (g->npose)
                HIPCHK(hipMemcpyAsync(sp, d_poses, (size_t)g->npose * sizeof(orbg_pose),
                                      hipMemcpyDeviceToDevice, st));
            if (g->npoint)
                HIPCHK(hipMemcpyAsync(sq, d_points, (size_t)g->npoint * 24, hipMemcpyDeviceToDevice, st));
            // setLambda + solve + update (the Schur solve adds lambda to its own copies of
            // the diagonal: no restoreDiagonal needed)
            if ((rc = orbg_ba_graph_schur_solve(c, g, lambda, hpl, hp, bp, hq, bq, dxp, dxq,
                                                (int32_t *)(sc + 3))))
                return rc;
            if (launch_ba_update(st, d_poses, g->npose, d_points, g->npoint, dxp, dxq, d_poses,
                                 d_points) ||
                launch_lm_reduce(st, 1, 6 * g->npose, 3 * g->npoint, lambda, dxp, dxq, bp, bq,
                                 nullptr, part, sc + 1))
                return fail(ORBG_EIO, "update / reduction launch");
            if ((rc = chi2(sc)) || (rc = read(hs, 4))) return rc;
            double tempChi = hs[0];
            const bool ok2 = *(const int32_t *)&hs[3] != 0;
            if (!ok2) tempChi = DBL_MAX;
            rhoLM = currentChi - tempChi;
            double scale = hs[1];
            scale += 1e-3;
            rhoLM /= scale;
            R.trials++;
            if (rhoLM > 0 && std::isfinite(tempChi)) {  // the step is good
                double alpha = 1. - lm_cube_host(2 * rhoLM - 1);
                alpha = std::min(alpha, 2. / 3.);
                const double scaleFactor = std::max(1. / 3., alpha);
                lambda *= scaleFactor;
                ni = 2;
                currentChi = tempChi;
            } else {  // pop
                lambda *= ni;
                ni *= 2;
                if (g->npose)
                    HIPCHK(hipMemcpyAsync(d_poses, sp, (size_t)g->npose * sizeof(orbg_pose),
                                          hipMemcpyDeviceToDevice, st));
                if (g->npoint)
                    HIPCHK(hipMemcpyAsync(d_points, sq, (size_t)g->npoint * 24,
                                          hipMemcpyDeviceToDevice, st));
            }
            qmax++;
            if (K.post_trial) K.post_trial(K.user, it, qmax - 1);
        } while (rhoLM < 0 && qmax < 10 && !terminate());
        R.iterations = it + 1;
        R.final_chi2 = currentChi;
        R.lambda = lambda;
        bool ok = true;  // solve() returned OK (not Terminate)
        if (qmax == 10 || rhoLM == 0) {
            R.terminated = 1;
            ok = false;
        } else {
            if ((iniChi - currentChi) * 1e3 < iniChi)
                nBad++;
            else
                nBad = 0;
            if (nBad >= 3) {
                R.terminated = 2;
                ok = false;
            }
        }
        if (K.post_iteration) K.post_iteration(K.user, it);
        if (!ok) break;
    }
    if (!ran) {  // no iteration: the report's chi2 at the given estimates (g2o computes none)
        if ((rc = chi2(sc)) || (rc = read(hs, 1))) return rc;
        R.initial_chi2 = R.final_chi2 = hs[0];
    } else if (K.d_last_chi2 && g->nedge) {
        HIPCHK(hipMemcpyAsync(K.d_last_chi2, chi, (size_t)g->nedge * 8, hipMemcpyDeviceToDevice, st));
    }
    if (R.terminated == 0 && terminate()) R.terminated = 3;
    HIPCHK(hipStreamSynchronize(st));
    if (rep) *rep = R;
    return ORBG_OK;
}

// Optimizer::LocalBundleAdjustment's optimisation (Optimizer.cc:853-935) on one window: see
// include/orbg.h.  The host takes the decisions the reference takes on the host (the flag, the
// outlier thresholds, isBad), every pass over the edges runs on the device.
extern "C" int orbg_local_ba_optimize(orbg_ctx *c, orbg_pose *poses, int npose, double *points,
                                      int npoint, const orbg_edge *edges, int nedge,
                                      const orbg_lm_control *control,
                                      int (*point_is_bad)(void *user, int point), void *user,
                                      uint8_t *erase, orbg_lba_report *rep)
{
    if (!c) return set_err(ORBG_EINVAL, "ctx is NULL");
    if (npose < 0 || npoint < 0 || nedge < 0) return set_err(ORBG_EINVAL, "negative size");
    if ((npose && !poses) || (npoint && !points) || (nedge && (!edges || !erase)))
        return set_err(ORBG_EINVAL, "NULL array");
    orbg_lba_report R{};
    if (nedge == 0) {  // initializeOptimization of an empty graph fails: nothing optimised
        if (rep) *rep = R;
        return ORBG_OK;
    }
    HIPCHK(hipSetDevice(c->device));
    orbg_ba_graph *g = nullptr;
    int rc = orbg_ba_graph_create(c, edges, nedge, npose, npoint, &g);
    if (rc) return rc;
    uint8_t *dmem = nullptr;
    struct Guard {
        orbg_ba_graph *g;
        uint8_t **m;
        ~Guard()
        {
            if (*m) hipFree(*m);
            if (g) orbg_ba_graph_destroy(g);
        }
    } guard{g, &dmem};
    const size_t ne = (size_t)nedge, np = (size_t)std::max(npose, 1), nq = (size_t)std::max(npoint, 1);
    const size_t o_p = 0, o_q = al256(np * sizeof(orbg_pose)), o_c5 = o_q + al256(nq * 24),
                 o_c10 = o_c5 + al256(ne * 8), o_ce = o_c10 + al256(ne * 8),
                 o_dk = o_ce + al256(ne * 8), o_end = o_dk + al256(ne);
    HIPCHK(hipMalloc((void **)&dmem, o_end));
    orbg_pose *d_poses = (orbg_pose *)(dmem + o_p);
    double *d_points = (double *)(dmem + o_q), *d_c5 = (double *)(dmem + o_c5),
           *d_c10 = (double *)(dmem + o_c10), *d_ce = (double *)(dmem + o_ce);
    uint8_t *d_dk = dmem + o_dk;
    hipStream_t st = c->stream;
    if (npose)
        HIPCHK(hipMemcpyAsync(d_poses, poses, (size_t)npose * sizeof(orbg_pose), hipMemcpyHostToDevice, st));
    if (npoint)
        HIPCHK(hipMemcpyAsync(d_points, points, (size_t)npoint * 24, hipMemcpyHostToDevice, st));
    std::vector<uint8_t> fixed((size_t)std::max(npose, 1), 0), active(ne), robust(ne);
    for (int i = 0; i < npose; i++) fixed[i] = poses[i].fixed ? 1 : 0;
    for (size_t e = 0; e < ne; e++) {
        active[e] = edges[e].active ? 1 : 0;
        robust[e] = edges[e].robust ? 1 : 0;
    }
    if ((rc = orbg_ba_graph_schur_plan(c, g, fixed.data()))) return rc;
    // the chi2 g2o's edges would hold if optimize(5) ran no iteration: the initial estimates'
    if ((rc = orbg_ba_graph_errors(c, g, d_poses, d_points, nullptr, d_c5, nullptr, nullptr))) return rc;
    orbg_lm_control K{};
    if (control) K = *control;
    const volatile uint8_t *force_stop = K.force_stop;
    K.d_last_chi2 = d_c5;
    if ((rc = orbg_ba_graph_optimize_ctl(c, g, d_poses, d_points, 5, &K, &R.lm[0]))) return rc;
    auto stopped = [&]() { return force_stop && *force_stop != 0; };
    auto bad = [&](int pt) { return point_is_bad && point_is_bad(user, pt) != 0; };
    auto over = [&](size_t e, double chi2) {
        return chi2 > (edges[e].stereo ? 7.815 : 5.991);
    };
    std::vector<double> chi(ne), tmp(ne);
    std::vector<uint8_t> depth(ne);
    auto depth_now = [&]() -> int {  // isDepthPositive at the current estimates
        int r = orbg_ba_graph_errors(c, g, d_poses, d_points, nullptr, d_ce, nullptr, d_dk);
        if (r) return r;
        HIPCHK(hipMemcpyAsync(depth.data(), d_dk, ne, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        return ORBG_OK;
    };
    HIPCHK(hipMemcpyAsync(chi.data(), d_c5, ne * 8, hipMemcpyDeviceToHost, st));
    R.do_more = stopped() ? 0 : 1;
    if (R.do_more) {
        if ((rc = depth_now())) return rc;
        for (size_t e = 0; e < ne; e++) {
            if (bad(edges[e].point)) continue;
            if (over(e, chi[e]) || !depth[e]) {
                if (active[e]) R.n_outliers++;
                active[e] = 0;  // setLevel(1)
            }
            robust[e] = 0;  // setRobustKernel(0)
        }
        // initializeOptimization(0): the level-0 edges (set_active rebuilds the Schur plan)
        if ((rc = orbg_ba_graph_set_active(c, g, active.data())) ||
            (rc = orbg_ba_graph_set_robust(c, g, robust.data())))
            return rc;
        K.d_last_chi2 = d_c10;
        if ((rc = orbg_ba_graph_optimize_ctl(c, g, d_poses, d_points, 10, &K, &R.lm[1]))) return rc;
        if (R.lm[1].trials > 0) {  // g2o recomputed the active edges' errors only
            HIPCHK(hipMemcpyAsync(tmp.data(), d_c10, ne * 8, hipMemcpyDeviceToHost, st));
            HIPCHK(hipStreamSynchronize(st));
            for (size_t e = 0; e < ne; e++)
                if (active[e]) chi[e] = tmp[e];
        }
    }
    if ((rc = depth_now())) return rc;
    for (size_t e = 0; e < ne; e++) {
        erase[e] = 0;
        if (bad(edges[e].point)) continue;
        if (over(e, chi[e]) || !depth[e]) {
            erase[e] = 1;
            R.n_erase++;
        }
    }
    if (npose)
        HIPCHK(hipMemcpyAsync(poses, d_poses, (size_t)npose * sizeof(orbg_pose), hipMemcpyDeviceToHost, st));
    if (npoint)
        HIPCHK(hipMemcpyAsync(points, d_points, (size_t)npoint * 24, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (rep) *rep = R;
    return ORBG_OK;
}

// profiling hook used by the other translation units
namespace orbg {
void prof_begin(void *prof, hipStream_t s, const char *n, hipEvent_t *a)
{
    ((Prof *)prof)->begin(s, n, a);
}
void prof_end(void *prof, hipStream_t s, const char *n, hipEvent_t a)
{
    ((Prof *)prof)->end(s, n, a);
}
bool prof_skip_name(const char *n) { return prof_skip(n); }
}  // namespace orbg

// ---------------------------------------------------------------------------
// tracking matchers (ORBmatcher::SearchByProjection x 2)
// ---------------------------------------------------------------------------
static int track_run(orbg_ctx *c, int mode, const orbg_track_batch *tb, int nframes)
{
    if (tb->frame_cap <= 0 || tb->query_cap <= 0 || tb->frame_cap > (1 << 20))
        return set_err(ORBG_EINVAL, "frame_cap / query_cap out of range");
    if (!tb->kps || !tb->desc || !tb->counts || !tb->bounds || !tb->queries || !tb->qdesc ||
        !tb->qcounts || !tb->match || !tb->nmatches)
        return set_err(ORBG_EINVAL, "NULL device array");
    if (mode == ORBG_TRACK_LASTFRAME && !tb->cams) return set_err(ORBG_EINVAL, "cams is NULL");
    if ((mode == ORBG_TRACK_RELOC || mode == ORBG_TRACK_LOOP) && !tb->fcams)
        return set_err(ORBG_EINVAL, "fcams is NULL");
    const size_t tk = al256((size_t)nframes * tb->query_cap * ORBG_MATCH_TOPK * 8);
    const size_t need = tk + al256((size_t)nframes * tb->query_cap * 4);
    if (c->trk_bytes < need) {
        HIPCHK(hipStreamSynchronize(c->stream));
        if (c->d_trk) hipFree(c->d_trk);
        c->d_trk = nullptr;
        c->trk_bytes = 0;
        if (hipMalloc(&c->d_trk, need) != hipSuccess)
            return set_err(ORBG_ENOMEM, "track scratch %zu bytes", need);
        c->trk_bytes = need;
    }
    TrackArgs A{};
    A.kps = tb->kps;
    A.desc = tb->desc;
    A.uright = tb->uright;
    A.taken0 = tb->taken0;
    A.counts = tb->counts;
    A.bounds = tb->bounds;
    A.fc = tb->frame_cap;
    A.q = tb->queries;
    A.qdesc = tb->qdesc;
    A.qcounts = tb->qcounts;
    A.qc = tb->query_cap;
    A.cams = tb->cams;
    for (int l = 0; l < ORBG_MAX_LEVELS; l++)
        A.scale[l] = l < c->p.nlevels ? c->scale[l] : 1.f;
    A.th = tb->th;
    A.nnratio = tb->nnratio;
    A.check_ori = tb->check_ori;
    A.topk = (unsigned long long *)c->d_trk;
    A.topn = (int32_t *)((uint8_t *)c->d_trk + tk);
    A.match = tb->match;
    A.nmatches = tb->nmatches;
    // fcams / orb_dist were appended to orbg_track_batch in round 4: a caller built against
    // the older header passes the shorter struct, so they are read only in the modes that
    // define them (ABI notes)
    if (mode == ORBG_TRACK_RELOC || mode == ORBG_TRACK_LOOP) {
        A.fcams = tb->fcams;
        A.orb_dist = tb->orb_dist;
    }
    if (mode == ORBG_TRACK_LOOP) A.check_ori = 0;
    const int rc = launch_track(c->stream, mode, A, nframes, &c->prof);
    if (rc == ORBG_ENOTSUP)
        return set_err(rc, "frame_cap %d / query_cap %d exceed the LDS budget", tb->frame_cap,
                       tb->query_cap);
    if (rc) return set_err(rc, "track launch failed");
    return ORBG_OK;
}

extern "C" int orbg_search_by_projection_batch_device(orbg_ctx *c, int mode,
                                                      const orbg_track_batch *tb, int nframes)
{
    if (!c || !tb) return set_err(ORBG_EINVAL, "NULL argument");
    if (mode < ORBG_TRACK_LASTFRAME || mode > ORBG_TRACK_LOOP)
        return set_err(ORBG_EINVAL, "mode %d", mode);
    if (nframes <= 0) return ORBG_OK;
    HIPCHK(hipSetDevice(c->device));
    return track_run(c, mode, tb, nframes);
}

// one frame from host arrays: upload, run, download
static int track_host(orbg_ctx *c, int mode, const orbg_keypoint *kps, const uint8_t *desc,
                      const float *uright, int n, const uint8_t *taken0, const orbg_bounds *bounds,
                      const void *q, size_t qrec, const uint8_t *qdesc, int nq,
                      const orbg_track_camera *cam, float th, float nnratio, int check_ori,
                      int32_t *match, int *nmatches, const orbg_frustum_camera *fcam = nullptr,
                      int orb_dist = 0)
{
    if (!c || !bounds || !match || (n > 0 && (!kps || !desc)) || (nq > 0 && (!q || !qdesc)))
        return set_err(ORBG_EINVAL, "NULL argument");
    if (n < 0 || nq < 0) return set_err(ORBG_EINVAL, "negative size");
    if (mode == ORBG_TRACK_LASTFRAME && !cam) return set_err(ORBG_EINVAL, "cam is NULL");
    if ((mode == ORBG_TRACK_RELOC || mode == ORBG_TRACK_LOOP) && !fcam)
        return set_err(ORBG_EINVAL, "cam is NULL");
    for (int i = 0; i < n; i++) match[i] = -1;
    if (nmatches) *nmatches = 0;
    if (n == 0 || nq == 0) return ORBG_OK;
    HIPCHK(hipSetDevice(c->device));
    const size_t fc = (size_t)n, qc = (size_t)nq;
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t o = off;
        off += al256(bytes);
        return o;
    };
    const size_t o_kps = take(fc * sizeof(orbg_keypoint)), o_desc = take(fc * 32);
    const size_t o_ur = uright ? take(fc * 4) : 0, o_tk = taken0 ? take(fc) : 0;
    const size_t o_cnt = take(8), o_b = take(sizeof(orbg_bounds)), o_q = take(qc * qrec);
    const size_t o_qd = take(qc * 32), o_cam = take(sizeof(orbg_track_camera));
    const size_t o_fcam = take(sizeof(orbg_frustum_camera));
    const size_t o_match = take(fc * 4), o_nm = take(4);
    void *s;
    int rc = scratch(c, off, &s);
    if (rc) return rc;
    uint8_t *b = (uint8_t *)s;
    const int32_t cnts[2] = {n, nq};
    HIPCHK(hipMemcpyAsync(b + o_kps, kps, fc * sizeof(orbg_keypoint), hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(b + o_desc, desc, fc * 32, hipMemcpyHostToDevice, c->stream));
    if (uright) HIPCHK(hipMemcpyAsync(b + o_ur, uright, fc * 4, hipMemcpyHostToDevice, c->stream));
    if (taken0) HIPCHK(hipMemcpyAsync(b + o_tk, taken0, fc, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(b + o_cnt, cnts, 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(b + o_b, bounds, sizeof(orbg_bounds), hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(b + o_q, q, qc * qrec, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(b + o_qd, qdesc, qc * 32, hipMemcpyHostToDevice, c->stream));
    if (cam)
        HIPCHK(hipMemcpyAsync(b + o_cam, cam, sizeof(*cam), hipMemcpyHostToDevice, c->stream));
    if (fcam)
        HIPCHK(hipMemcpyAsync(b + o_fcam, fcam, sizeof(*fcam), hipMemcpyHostToDevice, c->stream));
    orbg_track_batch tb{};
    tb.kps = (const orbg_keypoint *)(b + o_kps);
    tb.desc = b + o_desc;
    tb.uright = uright ? (const float *)(b + o_ur) : nullptr;
    tb.taken0 = taken0 ? b + o_tk : nullptr;
    tb.counts = (const int32_t *)(b + o_cnt);
    tb.bounds = (const orbg_bounds *)(b + o_b);
    tb.frame_cap = n;
    tb.queries = b + o_q;
    tb.qdesc = b + o_qd;
    tb.qcounts = (const int32_t *)(b + o_cnt) + 1;
    tb.query_cap = nq;
    tb.cams = cam ? (const orbg_track_camera *)(b + o_cam) : nullptr;
    tb.th = th;
    tb.nnratio = nnratio;
    tb.check_ori = check_ori;
    tb.match = (int32_t *)(b + o_match);
    tb.nmatches = (int32_t *)(b + o_nm);
    tb.fcams = fcam ? (const orbg_frustum_camera *)(b + o_fcam) : nullptr;
    tb.orb_dist = orb_dist;
    if ((rc = track_run(c, mode, &tb, 1))) return rc;
    int32_t nm = 0;
    HIPCHK(hipMemcpyAsync(match, b + o_match, fc * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(&nm, b + o_nm, 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    c->prof.collect();
    if (nmatches) *nmatches = nm;
    return ORBG_OK;
}

extern "C" int orbg_search_by_projection_lastframe(orbg_ctx *c, const orbg_keypoint *kps,
                                                   const uint8_t *desc, const float *uright,
                                                   int n, const uint8_t *taken0,
                                                   const orbg_bounds *bounds,
                                                   const orbg_lastframe_point *pts,
                                                   const uint8_t *pdesc, int np,
                                                   const orbg_track_camera *cam, float th,
                                                   int check_ori, int32_t *match, int *nmatches)
{
    return track_host(c, ORBG_TRACK_LASTFRAME, kps, desc, uright, n, taken0, bounds, pts,
                      sizeof(orbg_lastframe_point), pdesc, np, cam, th, 0.f, check_ori, match,
                      nmatches);
}

extern "C" int orbg_search_by_projection_local(orbg_ctx *c, const orbg_keypoint *kps,
                                               const uint8_t *desc, const float *uright, int n,
                                               const uint8_t *taken0, const orbg_bounds *bounds,
                                               const orbg_map_projection *mps,
                                               const uint8_t *mdesc, int nm, float th,
                                               float nnratio, int32_t *match, int *nmatches)
{
    return track_host(c, ORBG_TRACK_LOCAL, kps, desc, uright, n, taken0, bounds, mps,
                      sizeof(orbg_map_projection), mdesc, nm, nullptr, th, nnratio, 0, match,
                      nmatches);
}

extern "C" int orbg_search_by_projection_reloc(orbg_ctx *c, const orbg_keypoint *kps,
                                               const uint8_t *desc, int n, const uint8_t *taken0,
                                               const orbg_frustum_camera *cam,
                                               const orbg_reloc_point *pts, const uint8_t *pdesc,
                                               int np, float th, int orb_dist, int check_ori,
                                               int32_t *match, int *nmatches)
{
    if (!cam) return set_err(ORBG_EINVAL, "NULL argument");
    return track_host(c, ORBG_TRACK_RELOC, kps, desc, nullptr, n, taken0, &cam->bounds, pts,
                      sizeof(orbg_reloc_point), pdesc, np, nullptr, th, 0.f, check_ori, match,
                      nmatches, cam, orb_dist);
}

extern "C" int orbg_search_by_projection_sim3(orbg_ctx *c, const orbg_keypoint *kps,
                                              const uint8_t *desc, int n, const uint8_t *taken0,
                                              const orbg_frustum_camera *cam,
                                              const orbg_map_point *mps, const uint8_t *mdesc,
                                              int nm, int th, int32_t *match, int *nmatches)
{
    if (!cam) return set_err(ORBG_EINVAL, "NULL argument");
    return track_host(c, ORBG_TRACK_LOOP, kps, desc, nullptr, n, taken0, &cam->bounds, mps,
                      sizeof(orbg_map_point), mdesc, nm, nullptr, (float)th, 0.f, 0, match,
                      nmatches, cam, 0);
}

// ---------------------------------------------------------------------------
// Optimizer::PoseOptimization
// ---------------------------------------------------------------------------
extern "C" int orbg_pose_optimization_batch_device(orbg_ctx *c, const orbg_pose_edge *edges,
                                                   const int32_t *counts, int edge_cap,
                                                   const orbg_pose_camera *cams,
                                                   const float *tcw_in, double *q_out,
                                                   double *t_out, float *tcw_out,
                                                   uint8_t *outlier, int32_t *ninliers,
                                                   int nframes)
{
    if (!c) return set_err(ORBG_EINVAL, "ctx is NULL");
    if (nframes <= 0) return ORBG_OK;
    if (edge_cap < 0 || !edges || !counts || !cams || !tcw_in || !q_out || !t_out || !tcw_out ||
        !outlier || !ninliers)
        return set_err(ORBG_EINVAL, "NULL device array");
    HIPCHK(hipSetDevice(c->device));
    const int rc = launch_pose_opt(c->stream, edges, counts, edge_cap, cams, tcw_in, q_out,
                                   t_out, tcw_out, outlier, ninliers, nframes, &c->prof);
    return rc ? set_err(rc, "pose optimisation launch failed") : ORBG_OK;
}

extern "C" int orbg_pose_optimization(orbg_ctx *c, const orbg_pose_edge *edges, int n,
                                      const orbg_pose_camera *cam, const float tcw_in[12],
                                      double q_out[4], double t_out[3], float tcw_out[12],
                                      uint8_t *outlier, int *ninliers)
{
    if (!c || !cam || !tcw_in || !q_out || !t_out || !tcw_out || (n > 0 && (!edges || !outlier)))
        return set_err(ORBG_EINVAL, "NULL argument");
    if (n < 0) return set_err(ORBG_EINVAL, "negative size");
    HIPCHK(hipSetDevice(c->device));
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t o = off;
        off += al256(bytes);
        return o;
    };
    const size_t o_e = take((size_t)std::max(n, 1) * sizeof(orbg_pose_edge)), o_n = take(4);
    const size_t o_cam = take(sizeof(orbg_pose_camera)), o_tin = take(48), o_q = take(32);
    const size_t o_t = take(24), o_tout = take(48), o_out = take((size_t)std::max(n, 1));
    const size_t o_ni = take(4);
    void *s;
    int rc = scratch(c, off, &s);
    if (rc) return rc;
    uint8_t *b = (uint8_t *)s;
    const int32_t cnt = n;
    if (n) HIPCHK(hipMemcpyAsync(b + o_e, edges, (size_t)n * sizeof(orbg_pose_edge), hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(b + o_n, &cnt, 4, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(b + o_cam, cam, sizeof(*cam), hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(b + o_tin, tcw_in, 48, hipMemcpyHostToDevice, c->stream));
    if ((rc = launch_pose_opt(c->stream, (const orbg_pose_edge *)(b + o_e), (const int32_t *)(b + o_n),
                              std::max(n, 1), (const orbg_pose_camera *)(b + o_cam),
                              (const float *)(b + o_tin), (double *)(b + o_q), (double *)(b + o_t),
                              (float *)(b + o_tout), b + o_out, (int32_t *)(b + o_ni), 1,
                              &c->prof)))
        return set_err(rc, "pose optimisation launch failed");
    int32_t ni = 0;
    HIPCHK(hipMemcpyAsync(q_out, b + o_q, 32, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(t_out, b + o_t, 24, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(tcw_out, b + o_tout, 48, hipMemcpyDeviceToHost, c->stream));
    if (n) HIPCHK(hipMemcpyAsync(outlier, b + o_out, (size_t)n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(&ni, b + o_ni, 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    c->prof.collect();
    if (ninliers) *ninliers = ni;
    return ORBG_OK;
}

// ---------------------------------------------------------------------------
// LocalBundleAdjustment: BlockSolver<6,3>::solve (Schur complement)
// ---------------------------------------------------------------------------
// Device layout of a SchurPlanHost (structure) followed by the solve's scratch, from `base`
// (nullptr: sizes only); returns the bytes.  The structure arrays are uploaded once per plan.
static size_t schur_layout(const SchurPlanHost &P, int nedge, uint8_t *base, SchurArgs &A,
                           size_t *structure_bytes)
{
    size_t off = 0;
    auto take = [&](size_t bytes) -> uint8_t * {
        uint8_t *q = base ? base + off : nullptr;
        off += al256(std::max(bytes, (size_t)1));
        return q;
    };
    (void)nedge;
    A.pidx = (const int32_t *)take(P.pidx.size() * 4);
    A.free_pose = (const int32_t *)take(P.free_pose.size() * 4);
    A.pt_off = (const int32_t *)take(P.pt_off.size() * 4);
    A.pt_edges = (const int32_t *)take(P.pt_edges.size() * 4);
    A.slot_point = (const int32_t *)take(P.slot_point.size() * 4);
    A.slot_fidx = (const int32_t *)take(P.slot_fidx.size() * 4);
    A.edge_pose = (const int32_t *)take(P.edge_pose.size() * 4);
    A.blk_off = (const int32_t *)take(P.blk_off.size() * 4);
    A.blk_pairs = (const int2 *)take(P.blk_pairs.size() * 8);
    A.blk_i1 = (const int32_t *)take(P.blk_i1.size() * 4);
    A.blk_i2 = (const int32_t *)take(P.blk_i2.size() * 4);
    A.blk_seg = (const int32_t *)take(P.blk_seg.size() * 4);
    A.blk_order = (const int32_t *)take(P.blk_order.size() * 4);
    A.pose_off = (const int32_t *)take(P.pose_off.size() * 4);
    A.pose_slots = (const int32_t *)take(P.pose_slots.size() * 4);
    A.seg_lo = (const int32_t *)take(P.seg_lo.size() * 4);
    A.seg_soff = (const int64_t *)take(P.seg_soff.size() * 8);
    if (structure_bytes) *structure_bytes = off;
    const size_t nslot = (size_t)std::max(P.pt_off.back(), 1);
    A.rec = (double *)take((nslot + 256) * 24 * 8);  // k_schur_points' records (+ a workgroup's tail)
    A.S = (double *)take((size_t)std::max<int64_t>(P.seg_soff.back(), 1) * 8);
    A.x = (double *)take((size_t)std::max(6 * P.nfree, 1) * 8);
    A.nslot = P.pt_off.back();
    A.npose = P.npose;
    A.npoint = P.npoint;
    A.nfree = P.nfree;
    A.nblk = P.nblk;
    A.nseg = P.nseg;
    A.max_seg = P.max_seg;
    A.s_total = P.seg_soff.back();
    return off;
}

// the structure arrays of P to their places in A (stream-ordered copies from host memory)
static int schur_upload(const SchurPlanHost &P, const SchurArgs &A, hipStream_t st)
{
    auto up = [&](const void *dst, const void *src, size_t bytes) -> int {
        if (bytes) HIPCHK(hipMemcpyAsync((void *)dst, src, bytes, hipMemcpyHostToDevice, st));
        return ORBG_OK;
    };
    int rc;
    if ((rc = up(A.pidx, P.pidx.data(), P.pidx.size() * 4)) ||
        (rc = up(A.free_pose, P.free_pose.data(), P.free_pose.size() * 4)) ||
        (rc = up(A.pt_off, P.pt_off.data(), P.pt_off.size() * 4)) ||
        (rc = up(A.pt_edges, P.pt_edges.data(), P.pt_edges.size() * 4)) ||
        (rc = up(A.slot_point, P.slot_point.data(), P.slot_point.size() * 4)) ||
        (rc = up(A.slot_fidx, P.slot_fidx.data(), P.slot_fidx.size() * 4)) ||
        (rc = up(A.edge_pose, P.edge_pose.data(), P.edge_pose.size() * 4)) ||
        (rc = up(A.blk_off, P.blk_off.data(), P.blk_off.size() * 4)) ||
        (rc = up(A.blk_pairs, P.blk_pairs.data(), P.blk_pairs.size() * 8)) ||
        (rc = up(A.blk_i1, P.blk_i1.data(), P.blk_i1.size() * 4)) ||
        (rc = up(A.blk_i2, P.blk_i2.data(), P.blk_i2.size() * 4)) ||
        (rc = up(A.blk_seg, P.blk_seg.data(), P.blk_seg.size() * 4)) ||
        (rc = up(A.blk_order, P.blk_order.data(), P.blk_order.size() * 4)) ||
        (rc = up(A.pose_off, P.pose_off.data(), P.pose_off.size() * 4)) ||
        (rc = up(A.pose_slots, P.pose_slots.data(), P.pose_slots.size() * 4)) ||
        (rc = up(A.seg_lo, P.seg_lo.data(), P.seg_lo.size() * 4)) ||
        (rc = up(A.seg_soff, P.seg_soff.data(), P.seg_soff.size() * 8)))
        return rc;
    return ORBG_OK;
}

extern "C" int orbg_ba_schur_solve(orbg_ctx *c, const orbg_pose *poses, int npose, int npoint,
                                   const orbg_edge *edges, int nedge, const orbg_edge_out *eout,
                                   const double *hpose, const double *bpose,
                                   const double *hpoint, const double *bpoint, double lambda,
                                   double *dx_pose, double *dx_point, int *ok)
{
    if (!c || !ok || npose < 0 || npoint < 0 || nedge < 0)
        return set_err(ORBG_EINVAL, "NULL argument or negative size");
    if ((npose && (!poses || !hpose || !bpose || !dx_pose)) ||
        (npoint && (!hpoint || !bpoint || !dx_point)) || (nedge && (!edges || !eout)))
        return set_err(ORBG_EINVAL, "NULL array");
    for (int e = 0; e < nedge; e++)
        if (edges[e].pose < 0 || edges[e].pose >= npose || edges[e].point < 0 ||
            edges[e].point >= npoint)
            return set_err(ORBG_EINVAL, "edge %d references a missing vertex", e);
    HIPCHK(hipSetDevice(c->device));
    // the structure (built per call here: the graph entry points keep it across iterations)
    std::vector<int32_t> ep(std::max(nedge, 1)), eq(std::max(nedge, 1));
    std::vector<uint8_t> ea(std::max(nedge, 1)), fx(std::max(npose, 1));
    for (int e = 0; e < nedge; e++) {
        ep[e] = edges[e].pose;
        eq[e] = edges[e].point;
        ea[e] = edges[e].active ? 1 : 0;
    }
    for (int i = 0; i < npose; i++) fx[i] = poses[i].fixed ? 1 : 0;
    SchurPlanHost P;
    build_schur_plan(npose, npoint, nedge, ep.data(), eq.data(), ea.data(), fx.data(), P);
    SchurArgs A{};
    const size_t sb = schur_layout(P, nedge, nullptr, A, nullptr);
    size_t off = sb;
    auto take = [&](size_t bytes) {
        const size_t o = off;
        off += al256(std::max(bytes, (size_t)1));
        return o;
    };
    const size_t o_eout = take((size_t)nedge * sizeof(orbg_edge_out));
    const size_t o_hp = take((size_t)npose * 36 * 8), o_bpz = take((size_t)npose * 6 * 8);
    const size_t o_hq = take((size_t)npoint * 9 * 8), o_bq = take((size_t)npoint * 3 * 8);
    const size_t o_ok = take(4);
    const size_t o_dp = take((size_t)npose * 6 * 8), o_dq = take((size_t)npoint * 3 * 8);
    void *sp;
    int rc = scratch(c, off, &sp);
    if (rc) return rc;
    uint8_t *B = (uint8_t *)sp;
    schur_layout(P, nedge, B, A, nullptr);
    if ((rc = schur_upload(P, A, c->stream))) return rc;
    auto up = [&](size_t o, const void *src, size_t bytes) -> int {
        if (bytes) HIPCHK(hipMemcpyAsync(B + o, src, bytes, hipMemcpyHostToDevice, c->stream));
        return ORBG_OK;
    };
    if ((rc = up(o_eout, eout, (size_t)nedge * sizeof(orbg_edge_out))) ||
        (rc = up(o_hp, hpose, (size_t)npose * 36 * 8)) || (rc = up(o_bpz, bpose, (size_t)npose * 6 * 8)) ||
        (rc = up(o_hq, hpoint, (size_t)npoint * 9 * 8)) || (rc = up(o_bq, bpoint, (size_t)npoint * 3 * 8)))
        return rc;
    static_assert(sizeof(orbg_edge_out) % 8 == 0, "edge_out records are whole doubles");
    A.hpl = (const double *)(B + o_eout + offsetof(orbg_edge_out, hpl));
    A.hpl_stride = (int)(sizeof(orbg_edge_out) / 8);
    A.hpose = (const double *)(B + o_hp);
    A.bpose = (const double *)(B + o_bpz);
    A.hpoint = (const double *)(B + o_hq);
    A.bpoint = (const double *)(B + o_bq);
    A.lambda = lambda;
    A.ok = (int32_t *)(B + o_ok);
    A.dx_pose = (double *)(B + o_dp);
    A.dx_point = (double *)(B + o_dq);
    if ((rc = launch_schur(c->stream, A, &c->prof))) return set_err(rc, "schur launch failed");
    int32_t okv = 0;
    if (npose) HIPCHK(hipMemcpyAsync(dx_pose, B + o_dp, (size_t)npose * 6 * 8, hipMemcpyDeviceToHost, c->stream));
    if (npoint) HIPCHK(hipMemcpyAsync(dx_point, B + o_dq, (size_t)npoint * 3 * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(&okv, B + o_ok, 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    c->prof.collect();
    *ok = okv;
    return ORBG_OK;
}

// ---------------------------------------------------------------------------
// DBoW2 vocabulary (TemplatedVocabulary::loadFromTextFile) + transform (Frame::ComputeBoW)
// ---------------------------------------------------------------------------
struct orbg_vocab {
    int device = 0;
    int k = 0, L = 0, scoring = 0, weighting = 0, nnodes = 0, nwords = 0;
    int group = 16, root_c0 = 0, root_c1 = 0;
    BowSlot *d_slots = nullptr;
};

extern "C" int orbg_vocab_create(orbg_ctx *c, int k, int L, int scoring, int weighting,
                                 int nnodes, const int32_t *parent, const uint8_t *is_leaf,
                                 const uint8_t *desc, const double *weight, orbg_vocab **out)
{
    if (!c || !out) return set_err(ORBG_EINVAL, "NULL argument");
    *out = nullptr;
    // header checks of loadFromTextFile (TemplatedVocabulary.h:1359-1363)
    if (k < 0 || k > 20 || L < 1 || L > 10 || scoring < 0 || scoring > 5 || weighting < 0 ||
        weighting > 3)
        return set_err(ORBG_EINVAL, "k %d L %d scoring %d weighting %d outside the text format",
                       k, L, scoring, weighting);
    if (nnodes < 1) return set_err(ORBG_EINVAL, "a vocabulary has at least the root node");
    if (nnodes > 1 && (!parent || !is_leaf || !desc || !weight))
        return set_err(ORBG_EINVAL, "NULL node array");
    std::vector<int32_t> off(nnodes + 1, 0), word(nnodes, 0);
    int nwords = 0;
    for (int i = 1; i < nnodes; i++) {
        if (parent[i] < 0 || parent[i] >= i)
            return set_err(ORBG_EINVAL, "node %d: parent %d is not an earlier node", i, parent[i]);
        off[parent[i] + 1]++;
        if (is_leaf[i]) word[i] = nwords++;
    }
    int maxc = 0;
    for (int i = 0; i < nnodes; i++) {
        maxc = std::max(maxc, off[i + 1]);
        off[i + 1] += off[i];
    }
    if (maxc > 64) return set_err(ORBG_ENOTSUP, "a node with %d children (> 64)", maxc);
    std::vector<BowSlot> slots(std::max(nnodes - 1, 1));
    std::vector<int32_t> fill(off.begin(), off.end() - 1);
    for (int i = 1; i < nnodes; i++) {  // children in node (file) order
        BowSlot &s = slots[fill[parent[i]]++];
        memset(&s, 0, sizeof(s));
        memcpy(s.d, desc + (size_t)i * 32, 32);
        s.c0 = off[i];
        s.c1 = off[i + 1];
        s.node = i;
        s.word = word[i];
        s.weight = weight[i];
    }
    auto *v = new orbg_vocab();
    v->device = c->device;
    v->k = k;
    v->L = L;
    v->scoring = scoring;
    v->weighting = weighting;
    v->nnodes = nnodes;
    v->nwords = nwords;
    v->group = maxc <= 16 ? 16 : maxc <= 32 ? 32 : 64;
    v->root_c0 = off[0];
    v->root_c1 = off[1];
    hipError_t e = hipSetDevice(c->device);
    if (e == hipSuccess) e = hipMalloc(&v->d_slots, slots.size() * sizeof(BowSlot));
    if (e == hipSuccess)
        e = hipMemcpy(v->d_slots, slots.data(), slots.size() * sizeof(BowSlot), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        if (v->d_slots) hipFree(v->d_slots);
        delete v;
        return set_err(ORBG_ENOMEM, "vocabulary upload: %s", hipGetErrorString(e));
    }
    *out = v;
    return ORBG_OK;
}

extern "C" int orbg_vocab_load_text(orbg_ctx *c, const char *path, orbg_vocab **out)
{
    if (!c || !path || !out) return set_err(ORBG_EINVAL, "NULL argument");
    FILE *fp = fopen(path, "r");
    if (!fp) return set_err(ORBG_EINVAL, "cannot open %s", path);
    char *line = nullptr;
    size_t cap = 0;
    int k = 0, L = 0, n1 = 0, n2 = 0, rc = ORBG_OK;
    std::vector<int32_t> parent(1, 0);
    std::vector<uint8_t> leaf(1, 0), desc(32, 0);
    std::vector<double> weight(1, 0.0);
    if (getline(&line, &cap, fp) < 0 || sscanf(line, "%d %d %d %d", &k, &L, &n1, &n2) != 4) {
        rc = set_err(ORBG_EINVAL, "%s: missing header line", path);
    } else {
        long lineno = 1;
        while (getline(&line, &cap, fp) >= 0) {
            lineno++;
            char *p = line, *e;
            while (*p == ' ' || *p == '\t' || *p == '\r' || *p == '\n') p++;
            if (!*p) continue;  // blank line
            long vals[34];
            int nv = 0;
            for (; nv < 34; nv++) {
                vals[nv] = strtol(p, &e, 10);
                if (e == p) break;
                p = e;
            }
            const double w = strtod(p, &e);
            if (nv < 34 || e == p) {
                rc = set_err(ORBG_EINVAL, "%s:%ld: expected parent isLeaf 32 bytes weight", path,
                             lineno);
                break;
            }
            parent.push_back((int32_t)vals[0]);
            leaf.push_back(vals[1] > 0);
            for (int j = 0; j < 32; j++) desc.push_back((uint8_t)vals[2 + j]);
            weight.push_back(w);
        }
    }
    free(line);
    fclose(fp);
    if (rc) return rc;
    return orbg_vocab_create(c, k, L, n1, n2, (int)parent.size(), parent.data(), leaf.data(),
                             desc.data(), weight.data(), out);
}

extern "C" void orbg_vocab_destroy(orbg_vocab *v)
{
    if (!v) return;
    if (v->d_slots) {
        hipSetDevice(v->device);
        hipFree(v->d_slots);
    }
    delete v;
}

extern "C" int orbg_vocab_info(const orbg_vocab *v, int32_t *k, int32_t *L, int32_t *scoring,
                               int32_t *weighting, int32_t *nnodes, int32_t *nwords)
{
    if (!v) return set_err(ORBG_EINVAL, "vocabulary is NULL");
    if (k) *k = v->k;
    if (L) *L = v->L;
    if (scoring) *scoring = v->scoring;
    if (weighting) *weighting = v->weighting;
    if (nnodes) *nnodes = v->nnodes;
    if (nwords) *nwords = v->nwords;
    return ORBG_OK;
}

#define ORBG_BOW_MAX_CAP 8192   // k_bow_vectors sorts a frame's keys in LDS

static BowArgs bow_args(const orbg_vocab *v, int levelsup)
{
    BowArgs A{};
    A.slots = v->d_slots;
    A.root_c0 = v->root_c0;
    A.root_c1 = v->root_c1;
    A.group = v->group;
    A.nid_level = v->L - levelsup;
    A.scoring = v->scoring;
    A.weighting = v->weighting;
    A.empty = v->nwords == 0;
    return A;
}

extern "C" int orbg_bow_transform_batch_device(orbg_ctx *c, const orbg_vocab *v,
                                               const uint8_t *desc, const int32_t *counts,
                                               int cap, int nframes, int levelsup,
                                               int32_t *bow_words, double *bow_weights,
                                               int32_t *nbow, int32_t *fv_nodes,
                                               int32_t *fv_off, int32_t *fv_feats, int32_t *nfv,
                                               int32_t *word_of, int32_t *node_of)
{
    if (!c || !v) return set_err(ORBG_EINVAL, "NULL context or vocabulary");
    if (v->device != c->device) return set_err(ORBG_EINVAL, "vocabulary lives on another device");
    if (nframes <= 0) return ORBG_OK;
    if (cap < 1 || cap > ORBG_BOW_MAX_CAP)
        return set_err(ORBG_ENOTSUP, "cap %d outside 1..%d", cap, ORBG_BOW_MAX_CAP);
    if (!desc || !counts || !bow_words || !bow_weights || !nbow || !fv_nodes || !fv_off ||
        !fv_feats || !nfv)
        return set_err(ORBG_EINVAL, "NULL device array");
    HIPCHK(hipSetDevice(c->device));
    const size_t per = (size_t)nframes * cap;
    const size_t o_w = 0, o_n = al256(per * 4), o_x = o_n + al256(per * 4);
    void *s;
    int rc = scratch(c, o_x + al256(per * 8), &s);
    if (rc) return rc;
    BowArgs A = bow_args(v, levelsup);
    A.desc = desc;
    A.counts = counts;
    A.cap = cap;
    A.nframes = nframes;
    A.fword = word_of ? word_of : (int32_t *)((uint8_t *)s + o_w);
    A.fnode = node_of ? node_of : (int32_t *)((uint8_t *)s + o_n);
    A.fweight = (double *)((uint8_t *)s + o_x);
    A.bow_words = bow_words;
    A.bow_weights = bow_weights;
    A.nbow = nbow;
    A.fv_nodes = fv_nodes;
    A.fv_off = fv_off;
    A.fv_feats = fv_feats;
    A.nfv = nfv;
    if ((rc = launch_bow(c->stream, A, &c->prof))) return set_err(rc, "bow launch failed");
    return ORBG_OK;
}

extern "C" int orbg_bow_transform(orbg_ctx *c, const orbg_vocab *v, const uint8_t *desc, int n,
                                  int levelsup, int32_t *bow_words, double *bow_weights,
                                  int *nbow, int32_t *fv_nodes, int32_t *fv_off,
                                  int32_t *fv_feats, int *nfv)
{
    if (!c || !v || !nbow || !nfv || !fv_off) return set_err(ORBG_EINVAL, "NULL argument");
    if (n < 0) return set_err(ORBG_EINVAL, "negative size");
    if (n > ORBG_BOW_MAX_CAP) return set_err(ORBG_ENOTSUP, "%d descriptors (> %d)", n, ORBG_BOW_MAX_CAP);
    if (n > 0 && (!desc || !bow_words || !bow_weights || !fv_nodes || !fv_feats))
        return set_err(ORBG_EINVAL, "NULL array");
    *nbow = *nfv = 0;
    fv_off[0] = 0;
    if (n == 0) return ORBG_OK;
    HIPCHK(hipSetDevice(c->device));
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t o = off;
        off += al256(bytes);
        return o;
    };
    const size_t o_d = take((size_t)n * 32), o_c = take(4), o_fw = take((size_t)n * 4);
    const size_t o_fn = take((size_t)n * 4), o_fx = take((size_t)n * 8);
    const size_t o_bw = take((size_t)n * 4), o_bx = take((size_t)n * 8), o_nb = take(4);
    const size_t o_vn = take((size_t)n * 4), o_vo = take((size_t)(n + 1) * 4);
    const size_t o_vf = take((size_t)n * 4), o_nf = take(4);
    void *s;
    int rc = scratch(c, off, &s);
    if (rc) return rc;
    uint8_t *b = (uint8_t *)s;
    const int32_t cnt = n;
    HIPCHK(hipMemcpyAsync(b + o_d, desc, (size_t)n * 32, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(b + o_c, &cnt, 4, hipMemcpyHostToDevice, c->stream));
    BowArgs A = bow_args(v, levelsup);
    A.desc = b + o_d;
    A.counts = (const int32_t *)(b + o_c);
    A.cap = n;
    A.nframes = 1;
    A.fword = (int32_t *)(b + o_fw);
    A.fnode = (int32_t *)(b + o_fn);
    A.fweight = (double *)(b + o_fx);
    A.bow_words = (int32_t *)(b + o_bw);
    A.bow_weights = (double *)(b + o_bx);
    A.nbow = (int32_t *)(b + o_nb);
    A.fv_nodes = (int32_t *)(b + o_vn);
    A.fv_off = (int32_t *)(b + o_vo);
    A.fv_feats = (int32_t *)(b + o_vf);
    A.nfv = (int32_t *)(b + o_nf);
    if ((rc = launch_bow(c->stream, A, &c->prof))) return set_err(rc, "bow launch failed");
    int32_t nb = 0, nf = 0;
    HIPCHK(hipMemcpyAsync(&nb, b + o_nb, 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(&nf, b + o_nf, 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    // outputs are at most n long; copy what was produced
    HIPCHK(hipMemcpyAsync(bow_words, b + o_bw, (size_t)nb * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(bow_weights, b + o_bx, (size_t)nb * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(fv_nodes, b + o_vn, (size_t)nf * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(fv_off, b + o_vo, (size_t)(nf + 1) * 4, hipMemcpyDeviceToHost, c->stream));
    int32_t m = 0;
    HIPCHK(hipMemcpyAsync(&m, b + o_vo + (size_t)nf * 4, 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (m) HIPCHK(hipMemcpy(fv_feats, b + o_vf, (size_t)m * 4, hipMemcpyDeviceToHost));
    c->prof.collect();
    *nbow = nb;
    *nfv = nf;
    return ORBG_OK;
}

// ---------------------------------------------------------------------------
// ORBmatcher::SearchByBoW(KeyFrame*, Frame&) (bow_match_kernels.hip)
// ---------------------------------------------------------------------------
extern "C" int orbg_search_by_bow_kf_batch_device(orbg_ctx *c, const orbg_bow_frames *kf1,
                                                  const orbg_bow_frames *kf2, int cap,
                                                  const int32_t *d_kf1_index,
                                                  const int32_t *d_kf2_index, int npairs,
                                                  float nnratio, int check_ori,
                                                  int32_t *d_match12, int32_t *d_nmatch)
{
    if (!c || !kf1 || !kf2) return set_err(ORBG_EINVAL, "NULL argument");
    if (npairs < 0 || cap <= 0 || cap > 8192) return set_err(ORBG_EINVAL, "bad npairs / cap");
    if (npairs == 0) return ORBG_OK;
    if (!d_kf1_index || !d_kf2_index || !d_match12 || !d_nmatch || !kf1->desc || !kf1->kps ||
        !kf1->counts || !kf1->fv_nodes || !kf1->fv_off || !kf1->fv_feats || !kf1->nfv ||
        !kf2->desc || !kf2->kps || !kf2->fv_nodes || !kf2->fv_off || !kf2->fv_feats || !kf2->nfv)
        return set_err(ORBG_EINVAL, "NULL device array");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(order_after_caller(c));
    hipStream_t st = c->mstream;  // PROF_LAUNCH records on `st`
    int rc = 0;
    PROF_LAUNCH(c, "bow_match_kf",
                rc = launch_bow_match(st, *kf1, *kf2, cap, d_kf1_index, d_kf2_index, npairs,
                                      nnratio, check_ori, d_match12, d_nmatch, true));
    if (rc == ORBG_ENOTSUP) return set_err(ORBG_ENOTSUP, "SearchByBoW: more than 4096 features per frame");
    if (rc) return set_err(ORBG_EIO, "k_bow_match launch failed");
    return ORBG_OK;
}

extern "C" int orbg_search_by_bow_batch_device(orbg_ctx *c, const orbg_bow_frames *kf,
                                               const orbg_bow_frames *f, int cap,
                                               const int32_t *d_kf_index, const int32_t *d_f_index,
                                               int npairs, float nnratio, int check_ori,
                                               int32_t *d_match, int32_t *d_nmatch)
{
    if (!c || !kf || !f) return set_err(ORBG_EINVAL, "NULL argument");
    if (npairs < 0 || cap <= 0 || cap > 8192) return set_err(ORBG_EINVAL, "bad npairs / cap");
    if (npairs == 0) return ORBG_OK;
    if (!d_kf_index || !d_f_index || !d_match || !d_nmatch || !kf->desc || !kf->kps ||
        !kf->fv_nodes || !kf->fv_off || !kf->fv_feats || !kf->nfv || !f->desc || !f->kps ||
        !f->counts || !f->fv_nodes || !f->fv_off || !f->fv_feats || !f->nfv)
        return set_err(ORBG_EINVAL, "NULL device array");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(order_after_caller(c));
    hipStream_t st = c->mstream;  // PROF_LAUNCH records on `st`
    int rc = 0;
    PROF_LAUNCH(c, "bow_match",
                rc = launch_bow_match(st, *kf, *f, cap, d_kf_index, d_f_index, npairs, nnratio,
                                      check_ori, d_match, d_nmatch));
    if (rc == ORBG_ENOTSUP) return set_err(ORBG_ENOTSUP, "SearchByBoW: more than 4096 features per frame");
    if (rc) return set_err(ORBG_EIO, "k_bow_match launch failed");
    return ORBG_OK;
}

static int search_by_bow_host(orbg_ctx *c, const uint8_t *kf_desc, const float *kf_angle,
                                  const uint8_t *kf_valid, int n_kf, const int32_t *kf_fv_nodes,
                                  const int32_t *kf_fv_off, const int32_t *kf_fv_feats, int kf_nfv,
                                  const uint8_t *f_desc, const float *f_angle,
                                  const uint8_t *f_valid, int n_f,
                                  const int32_t *f_fv_nodes, const int32_t *f_fv_off,
                                  const int32_t *f_fv_feats, int f_nfv, float nnratio,
                                  int check_ori, int32_t *match, int *nmatches, bool kfkf)
{
    const int n_out = kfkf ? n_kf : n_f;  // KeyFrame-KeyFrame: vpMatches12 over pKF1
    if (!c || !match || !nmatches) return set_err(ORBG_EINVAL, "NULL argument");
    if (n_kf < 0 || n_f < 0 || kf_nfv < 0 || f_nfv < 0 || kf_nfv > std::max(n_kf, 0) ||
        f_nfv > std::max(n_f, 0))
        return set_err(ORBG_EINVAL, "bad sizes");
    if ((n_kf && (!kf_desc || !kf_angle)) || (n_f && (!f_desc || !f_angle)) ||
        (kf_nfv && (!kf_fv_nodes || !kf_fv_off || !kf_fv_feats)) ||
        (f_nfv && (!f_fv_nodes || !f_fv_off || !f_fv_feats)))
        return set_err(ORBG_EINVAL, "NULL input array");
    *nmatches = 0;
    for (int i = 0; i < n_out; i++) match[i] = -1;
    if (!n_f || !n_kf || !kf_nfv || !f_nfv) return ORBG_OK;
    for (int j = 0; j < kf_nfv; j++)
        for (int k = kf_fv_off[j]; k < kf_fv_off[j + 1]; k++)
            if (kf_fv_feats[k] < 0 || kf_fv_feats[k] >= n_kf)
                return set_err(ORBG_EINVAL, "KF feature index out of range");
    for (int j = 0; j < f_nfv; j++)
        for (int k = f_fv_off[j]; k < f_fv_off[j + 1]; k++)
            if (f_fv_feats[k] < 0 || f_fv_feats[k] >= n_f)
                return set_err(ORBG_EINVAL, "F feature index out of range");
    HIPCHK(hipSetDevice(c->device));
    // one buffer: two frames (KF = 0, F = 1) at cap = max(n_kf, n_f)
    const int cap = std::max(n_kf, n_f);
    if (cap > 8192) return set_err(ORBG_ENOTSUP, "more than 8192 features");
    const size_t cp = (size_t)cap;
    size_t o = 0;
    auto take = [&](size_t bytes) {
        const size_t r = o;
        o += al256(bytes);
        return r;
    };
    const size_t o_desc = take(2 * cp * 32), o_kps = take(2 * cp * sizeof(orbg_keypoint)),
                 o_cnt = take(2 * 4), o_nodes = take(2 * cp * 4), o_off = take(2 * (cp + 1) * 4),
                 o_feats = take(2 * cp * 4), o_nfv = take(2 * 4), o_val = take(2 * cp),
                 o_idx = take(2 * 4), o_match = take(cp * 4), o_nm = take(4);
    uint8_t *hs;
    int rc = stage(c, o, &hs);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(c->stream));
    memset(hs, 0, o);
    memcpy(hs + o_desc, kf_desc, (size_t)n_kf * 32);
    memcpy(hs + o_desc + cp * 32, f_desc, (size_t)n_f * 32);
    orbg_keypoint *hk = (orbg_keypoint *)(hs + o_kps);
    for (int i = 0; i < n_kf; i++) hk[i].angle = kf_angle[i];
    for (int i = 0; i < n_f; i++) hk[cp + i].angle = f_angle[i];
    int32_t *hc = (int32_t *)(hs + o_cnt);
    hc[0] = n_kf;
    hc[1] = n_f;
    memcpy(hs + o_nodes, kf_fv_nodes, (size_t)kf_nfv * 4);
    memcpy(hs + o_nodes + cp * 4, f_fv_nodes, (size_t)f_nfv * 4);
    memcpy(hs + o_off, kf_fv_off, (size_t)(kf_nfv + 1) * 4);
    memcpy(hs + o_off + (cp + 1) * 4, f_fv_off, (size_t)(f_nfv + 1) * 4);
    memcpy(hs + o_feats, kf_fv_feats, (size_t)kf_fv_off[kf_nfv] * 4);
    memcpy(hs + o_feats + cp * 4, f_fv_feats, (size_t)f_fv_off[f_nfv] * 4);
    int32_t *hn = (int32_t *)(hs + o_nfv);
    hn[0] = kf_nfv;
    hn[1] = f_nfv;
    if (kf_valid)
        memcpy(hs + o_val, kf_valid, (size_t)n_kf);
    else
        memset(hs + o_val, 1, (size_t)n_kf);
    if (f_valid)
        memcpy(hs + o_val + cp, f_valid, (size_t)n_f);
    else
        memset(hs + o_val + cp, 1, (size_t)n_f);
    int32_t *hi = (int32_t *)(hs + o_idx);
    hi[0] = 0;
    hi[1] = 1;
    void *d;
    if ((rc = scratch(c, o, &d))) return rc;
    uint8_t *db = (uint8_t *)d;
    HIPCHK(hipMemcpyAsync(db, hs, o, hipMemcpyHostToDevice, c->stream));
    orbg_bow_frames K{}, F{};
    K.desc = F.desc = db + o_desc;
    K.kps = F.kps = (const orbg_keypoint *)(db + o_kps);
    K.counts = F.counts = (const int32_t *)(db + o_cnt);
    K.fv_nodes = F.fv_nodes = (const int32_t *)(db + o_nodes);
    K.fv_off = F.fv_off = (const int32_t *)(db + o_off);
    K.fv_feats = F.fv_feats = (const int32_t *)(db + o_feats);
    K.nfv = F.nfv = (const int32_t *)(db + o_nfv);
    K.valid = F.valid = db + o_val;  // frame 0 (KF / pKF1) and frame 1 (F / pKF2) at + cap
    const int32_t *di = (const int32_t *)(db + o_idx);
    rc = launch_bow_match(c->stream, K, F, cap, di, di + 1, 1, nnratio, check_ori,
                          (int32_t *)(db + o_match), (int32_t *)(db + o_nm), kfkf);
    if (rc == ORBG_ENOTSUP) return set_err(ORBG_ENOTSUP, "SearchByBoW: more than 4096 features per frame");
    if (rc) return set_err(ORBG_EIO, "k_bow_match launch failed");
    HIPCHK(hipMemcpyAsync(hs + o_match, db + o_match, cp * 4 + 256, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    memcpy(match, hs + o_match, (size_t)n_out * 4);
    memcpy(nmatches, hs + o_nm, 4);
    return ORBG_OK;
}

extern "C" int orbg_search_by_bow(orbg_ctx *c, const uint8_t *kf_desc, const float *kf_angle,
                                  const uint8_t *kf_valid, int n_kf, const int32_t *kf_fv_nodes,
                                  const int32_t *kf_fv_off, const int32_t *kf_fv_feats, int kf_nfv,
                                  const uint8_t *f_desc, const float *f_angle, int n_f,
                                  const int32_t *f_fv_nodes, const int32_t *f_fv_off,
                                  const int32_t *f_fv_feats, int f_nfv, float nnratio,
                                  int check_ori, int32_t *match, int *nmatches)
{
    return search_by_bow_host(c, kf_desc, kf_angle, kf_valid, n_kf, kf_fv_nodes, kf_fv_off,
                              kf_fv_feats, kf_nfv, f_desc, f_angle, nullptr, n_f, f_fv_nodes,
                              f_fv_off, f_fv_feats, f_nfv, nnratio, check_ori, match, nmatches,
                              false);
}

extern "C" int orbg_search_by_bow_kf(orbg_ctx *c, const uint8_t *desc1, const float *angle1,
                                     const uint8_t *valid1, int n1, const int32_t *fv_nodes1,
                                     const int32_t *fv_off1, const int32_t *fv_feats1, int nfv1,
                                     const uint8_t *desc2, const float *angle2,
                                     const uint8_t *valid2, int n2, const int32_t *fv_nodes2,
                                     const int32_t *fv_off2, const int32_t *fv_feats2, int nfv2,
                                     float nnratio, int check_ori, int32_t *match12,
                                     int *nmatches)
{
    return search_by_bow_host(c, desc1, angle1, valid1, n1, fv_nodes1, fv_off1, fv_feats1, nfv1,
                              desc2, angle2, valid2, n2, fv_nodes2, fv_off2, fv_feats2, nfv2,
                              nnratio, check_ori, match12, nmatches, true);
}

// ---------------------------------------------------------------------------
// Frame / MapPoint geometry (frame_kernels.hip)
// ---------------------------------------------------------------------------
static bool cam_ok(const orbg_camera *cam)
{
    return cam && std::isfinite(cam->fx) && std::isfinite(cam->fy) && cam->fx != 0.f &&
           cam->fy != 0.f;
}

extern "C" int orbg_compute_image_bounds(const orbg_camera *cam, int w, int h, orbg_bounds *out)
{
    if (!cam || !out) return set_err(ORBG_EINVAL, "NULL argument");
    if (w < 0 || h < 0) return set_err(ORBG_EINVAL, "negative image size");
    if (cam->k1 != 0.0f) {
        if (!cam_ok(cam)) return set_err(ORBG_EINVAL, "fx / fy must be finite and nonzero");
        // the corners (0,0), (cols,0), (0,rows), (cols,rows), Frame.cc:579-600
        float o[8];
        const float in[8] = {0.f, 0.f, (float)w, 0.f, 0.f, (float)h, (float)w, (float)h};
        for (int i = 0; i < 4; i++) orbg::undistort_point(*cam, in[2 * i], in[2 * i + 1], &o[2 * i], &o[2 * i + 1]);
        out->min_x = std::min(o[0], o[4]);
        out->max_x = std::max(o[2], o[6]);
        out->min_y = std::min(o[1], o[3]);
        out->max_y = std::max(o[5], o[7]);
    } else {
        out->min_x = 0.0f;
        out->max_x = (float)w;
        out->min_y = 0.0f;
        out->max_y = (float)h;
    }
    return ORBG_OK;
}

extern "C" int orbg_set_camera(orbg_ctx *c, const orbg_camera *cam)
{
    if (!c) return set_err(ORBG_EINVAL, "NULL context");
    if (cam && cam->k1 != 0.0f && !cam_ok(cam))
        return set_err(ORBG_EINVAL, "fx / fy must be finite and nonzero");
    c->has_cam = cam && cam->k1 != 0.0f;
    if (cam) c->cam = *cam;
    return ORBG_OK;
}

extern "C" int orbg_batch_keys_un(orbg_ctx *c, orbg_keypoint **d_kps_un, int32_t *frame_cap)
{
    if (!c || !d_kps_un) return set_err(ORBG_EINVAL, "NULL argument");
    if (!c->gw || c->last_n <= 0) return set_err(ORBG_EINVAL, "no batch extracted");
    *d_kps_un = c->kps_un_valid ? c->d_kps_un : c->d_kps;
    if (frame_cap) *frame_cap = c->geom.frame_cap;
    return ORBG_OK;
}

extern "C" int orbg_undistort_batch_device(orbg_ctx *c, const orbg_camera *cam,
                                           const orbg_keypoint *d_kps, const int32_t *d_counts,
                                           int frame_cap, int nframes, orbg_keypoint *d_kps_un)
{
    if (!c || !cam) return set_err(ORBG_EINVAL, "NULL argument");
    if (nframes < 0 || frame_cap < 0) return set_err(ORBG_EINVAL, "negative size");
    if (nframes == 0 || frame_cap == 0) return ORBG_OK;
    if (!d_kps || !d_counts || !d_kps_un) return set_err(ORBG_EINVAL, "NULL device array");
    if (cam->k1 != 0.0f && !cam_ok(cam)) return set_err(ORBG_EINVAL, "fx / fy must be finite and nonzero");
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = c->stream;
    int rc = 0;
    PROF_LAUNCH(c, "undistort",
                rc = launch_undistort(st, *cam, d_kps, d_counts, frame_cap, nframes, d_kps_un));
    if (rc) return set_err(ORBG_EIO, "k_undistort launch failed");
    return ORBG_OK;
}

extern "C" int orbg_rgbd_stereo_batch_device(orbg_ctx *c, const void *d_depth, int depth_type,
                                             float factor, int w, int h, size_t pitch,
                                             size_t image_stride, const orbg_keypoint *d_kps,
                                             const orbg_keypoint *d_kps_un,
                                             const int32_t *d_counts, int frame_cap, int nframes,
                                             float mbf, float *d_uright, float *d_depth_out)
{
    if (!c) return set_err(ORBG_EINVAL, "NULL argument");
    if (depth_type != ORBG_DEPTH_F32 && depth_type != ORBG_DEPTH_U16)
        return set_err(ORBG_EINVAL, "depth_type %d", depth_type);
    if (nframes < 0 || frame_cap < 0 || w < 0 || h < 0) return set_err(ORBG_EINVAL, "negative size");
    if (nframes == 0 || frame_cap == 0) return ORBG_OK;
    const size_t px = depth_type == ORBG_DEPTH_U16 ? 2 : 4;
    if (pitch < (size_t)w * px) return set_err(ORBG_EINVAL, "pitch below the row width");
    if (nframes > 1 && image_stride < pitch * (size_t)h)
        return set_err(ORBG_EINVAL, "image_stride below one image");
    if (!d_depth || !d_kps || !d_kps_un || !d_counts || !d_uright || !d_depth_out)
        return set_err(ORBG_EINVAL, "NULL device array");
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = c->stream;
    int rc = 0;
    PROF_LAUNCH(c, "rgbd",
                rc = launch_rgbd(st, d_depth, depth_type == ORBG_DEPTH_U16, factor, w, h, pitch,
                                 image_stride, d_kps, d_kps_un, d_counts, frame_cap, nframes, mbf,
                                 d_uright, d_depth_out));
    if (rc) return set_err(ORBG_EIO, "k_rgbd launch failed");
    return ORBG_OK;
}

extern "C" int orbg_rgbd_stereo(orbg_ctx *c, const void *depth, int depth_type, float factor,
                                int w, int h, size_t pitch, const orbg_keypoint *kps,
                                const orbg_keypoint *kps_un, int n, float mbf, float *uright,
                                float *depth_out)
{
    if (!c) return set_err(ORBG_EINVAL, "NULL argument");
    if (depth_type != ORBG_DEPTH_F32 && depth_type != ORBG_DEPTH_U16)
        return set_err(ORBG_EINVAL, "depth_type %d", depth_type);
    if (n < 0 || w < 0 || h < 0) return set_err(ORBG_EINVAL, "negative size");
    if (n == 0) return ORBG_OK;
    if (!depth || !kps || !kps_un || !uright || !depth_out) return set_err(ORBG_EINVAL, "NULL array");
    const size_t px = depth_type == ORBG_DEPTH_U16 ? 2 : 4;
    if (pitch < (size_t)w * px) return set_err(ORBG_EINVAL, "pitch below the row width");
    HIPCHK(hipSetDevice(c->device));
    // only the keypoints' pixels are read: upload the image rows once (w x h), packed
    const size_t ib = al256((size_t)w * px * h), kb = al256((size_t)n * sizeof(orbg_keypoint));
    const size_t ob = al256((size_t)n * 4);
    const size_t o_img = 0, o_k = ib, o_ku = ib + kb, o_cnt = ib + 2 * kb, o_ur = o_cnt + 256,
                 o_d = o_ur + ob, tot = o_d + ob;
    uint8_t *hs;
    int rc = stage(c, tot, &hs);
    if (rc) return rc;
    void *dv;
    if ((rc = scratch(c, tot, &dv))) return rc;
    uint8_t *db = (uint8_t *)dv;
    HIPCHK(hipStreamSynchronize(c->stream));
    for (int y = 0; y < h; y++)
        memcpy(hs + o_img + (size_t)y * w * px, (const uint8_t *)depth + (size_t)y * pitch, (size_t)w * px);
    memcpy(hs + o_k, kps, (size_t)n * sizeof(orbg_keypoint));
    memcpy(hs + o_ku, kps_un, (size_t)n * sizeof(orbg_keypoint));
    const int32_t cnt = n;
    memcpy(hs + o_cnt, &cnt, 4);
    HIPCHK(hipMemcpyAsync(db, hs, o_ur, hipMemcpyHostToDevice, c->stream));
    rc = launch_rgbd(c->stream, db + o_img, depth_type == ORBG_DEPTH_U16, factor, w, h,
                     (size_t)w * px, 0, (const orbg_keypoint *)(db + o_k),
                     (const orbg_keypoint *)(db + o_ku), (const int32_t *)(db + o_cnt), n, 1, mbf,
                     (float *)(db + o_ur), (float *)(db + o_d));
    if (rc) return set_err(ORBG_EIO, "k_rgbd launch failed");
    HIPCHK(hipMemcpyAsync(hs + o_ur, db + o_ur, tot - o_ur, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    memcpy(uright, hs + o_ur, (size_t)n * 4);
    memcpy(depth_out, hs + o_d, (size_t)n * 4);
    return ORBG_OK;
}

extern "C" int orbg_undistort_keypoints(orbg_ctx *c, const orbg_camera *cam,
                                        const orbg_keypoint *kps, int n, orbg_keypoint *kps_un)
{
    if (!c || !cam) return set_err(ORBG_EINVAL, "NULL argument");
    if (n < 0) return set_err(ORBG_EINVAL, "negative size");
    if (n == 0) return ORBG_OK;
    if (!kps || !kps_un) return set_err(ORBG_EINVAL, "NULL array");
    if (cam->k1 != 0.0f && !cam_ok(cam)) return set_err(ORBG_EINVAL, "fx / fy must be finite and nonzero");
    HIPCHK(hipSetDevice(c->device));
    const size_t kb = al256((size_t)n * sizeof(orbg_keypoint));
    uint8_t *hs;
    int rc = stage(c, 2 * kb, &hs);
    if (rc) return rc;
    void *d;
    if ((rc = scratch(c, 2 * kb + 256, &d))) return rc;
    uint8_t *db = (uint8_t *)d;
    HIPCHK(hipStreamSynchronize(c->stream));  // the staging buffer may still feed a copy
    memcpy(hs, kps, (size_t)n * sizeof(orbg_keypoint));
    const int32_t cnt = n;
    memcpy(hs + kb, &cnt, 4);
    HIPCHK(hipMemcpyAsync(db, hs, kb + 4, hipMemcpyHostToDevice, c->stream));
    rc = launch_undistort(c->stream, *cam, (const orbg_keypoint *)db, (const int32_t *)(db + kb),
                          n, 1, (orbg_keypoint *)(db + kb + 256));
    if (rc) return set_err(ORBG_EIO, "k_undistort launch failed");
    HIPCHK(hipMemcpyAsync(hs, db + kb + 256, (size_t)n * sizeof(orbg_keypoint),
                          hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    memcpy(kps_un, hs, (size_t)n * sizeof(orbg_keypoint));
    return ORBG_OK;
}

extern "C" int orbg_is_in_frustum_batch_device(orbg_ctx *c, const orbg_frustum_camera *d_cams,
                                               const orbg_map_point *d_mps,
                                               const int32_t *d_counts, int cap, int nframes,
                                               float viewing_cos_limit,
                                               orbg_map_projection *d_proj, int32_t *d_nvisible)
{
    if (!c) return set_err(ORBG_EINVAL, "NULL context");
    if (nframes < 0 || cap < 0) return set_err(ORBG_EINVAL, "negative size");
    if (nframes == 0 || cap == 0) return ORBG_OK;
    if (!d_cams || !d_mps || !d_counts || !d_proj || !d_nvisible)
        return set_err(ORBG_EINVAL, "NULL device array");
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = c->stream;
    int rc = 0;
    PROF_LAUNCH(c, "frustum",
                rc = launch_frustum(st, d_cams, d_mps, d_counts, cap, nframes, viewing_cos_limit,
                                    d_proj, d_nvisible));
    if (rc) return set_err(ORBG_EIO, "k_frustum launch failed");
    return ORBG_OK;
}

extern "C" int orbg_is_in_frustum(orbg_ctx *c, const orbg_frustum_camera *cam,
                                  const orbg_map_point *mps, int n, float viewing_cos_limit,
                                  orbg_map_projection *proj, int *nvisible)
{
    if (!c || !cam || !nvisible) return set_err(ORBG_EINVAL, "NULL argument");
    if (n < 0) return set_err(ORBG_EINVAL, "negative size");
    *nvisible = 0;
    if (n == 0) return ORBG_OK;
    if (!mps || !proj) return set_err(ORBG_EINVAL, "NULL array");
    HIPCHK(hipSetDevice(c->device));
    size_t o = 0;
    auto take = [&](size_t bytes) {
        const size_t r = o;
        o += al256(bytes);
        return r;
    };
    const size_t o_cam = take(sizeof(orbg_frustum_camera)), o_cnt = take(4),
                 o_mp = take((size_t)n * sizeof(orbg_map_point)),
                 o_pr = take((size_t)n * sizeof(orbg_map_projection)), o_nv = take(4);
    uint8_t *hs;
    int rc = stage(c, o, &hs);
    if (rc) return rc;
    void *d;
    if ((rc = scratch(c, o, &d))) return rc;
    uint8_t *db = (uint8_t *)d;
    HIPCHK(hipStreamSynchronize(c->stream));
    memcpy(hs + o_cam, cam, sizeof(orbg_frustum_camera));
    const int32_t cnt = n;
    memcpy(hs + o_cnt, &cnt, 4);
    memcpy(hs + o_mp, mps, (size_t)n * sizeof(orbg_map_point));
    // the projections a point not in view keeps (only its flags are written)
    memcpy(hs + o_pr, proj, (size_t)n * sizeof(orbg_map_projection));
    HIPCHK(hipMemcpyAsync(db, hs, o_nv, hipMemcpyHostToDevice, c->stream));
    rc = launch_frustum(c->stream, (const orbg_frustum_camera *)(db + o_cam),
                        (const orbg_map_point *)(db + o_mp), (const int32_t *)(db + o_cnt), n, 1,
                        viewing_cos_limit, (orbg_map_projection *)(db + o_pr),
                        (int32_t *)(db + o_nv));
    if (rc) return set_err(ORBG_EIO, "k_frustum launch failed");
    HIPCHK(hipMemcpyAsync(hs + o_pr, db + o_pr, o - o_pr, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    memcpy(proj, hs + o_pr, (size_t)n * sizeof(orbg_map_projection));
    memcpy(nvisible, hs + o_nv, 4);
    return ORBG_OK;
}

extern "C" int orbg_distinctive_descriptors_batch_device(orbg_ctx *c, const uint8_t *d_pool,
                                                         const int32_t *d_rows,
                                                         const int32_t *d_off, int npoints,
                                                         int32_t *d_best, uint8_t *d_desc)
{
    if (!c) return set_err(ORBG_EINVAL, "NULL context");
    if (npoints < 0) return set_err(ORBG_EINVAL, "negative size");
    if (npoints == 0) return ORBG_OK;
    if (!d_pool || !d_rows || !d_off || !d_best) return set_err(ORBG_EINVAL, "NULL device array");
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = c->stream;
    int rc = 0;
    PROF_LAUNCH(c, "distinctive",
                rc = launch_distinctive(st, d_pool, d_rows, d_off, npoints, d_best, d_desc));
    if (rc) return set_err(ORBG_EIO, "k_distinctive launch failed");
    return ORBG_OK;
}

extern "C" int orbg_distinctive_descriptor(orbg_ctx *c, const uint8_t *desc, int n, int32_t *best)
{
    if (!c || !best) return set_err(ORBG_EINVAL, "NULL argument");
    if (n < 0) return set_err(ORBG_EINVAL, "negative size");
    *best = -1;
    if (n == 0) return ORBG_OK;  // observations empty: the reference returns (MapPoint.cc:356)
    if (!desc) return set_err(ORBG_EINVAL, "NULL array");
    HIPCHK(hipSetDevice(c->device));
    size_t o = 0;
    auto take = [&](size_t bytes) {
        const size_t r = o;
        o += al256(bytes);
        return r;
    };
    const size_t o_d = take((size_t)n * 32), o_r = take((size_t)n * 4), o_off = take(8),
                 o_b = take(4);
    uint8_t *hs;
    int rc = stage(c, o, &hs);
    if (rc) return rc;
    void *d;
    if ((rc = scratch(c, o, &d))) return rc;
    uint8_t *db = (uint8_t *)d;
    HIPCHK(hipStreamSynchronize(c->stream));
    memcpy(hs + o_d, desc, (size_t)n * 32);
    int32_t *hr = (int32_t *)(hs + o_r);
    for (int i = 0; i < n; i++) hr[i] = i;
    int32_t *ho = (int32_t *)(hs + o_off);
    ho[0] = 0;
    ho[1] = n;
    HIPCHK(hipMemcpyAsync(db, hs, o_b, hipMemcpyHostToDevice, c->stream));
    rc = launch_distinctive(c->stream, db + o_d, (const int32_t *)(db + o_r),
                            (const int32_t *)(db + o_off), 1, (int32_t *)(db + o_b), nullptr);
    if (rc) return set_err(ORBG_EIO, "k_distinctive launch failed");
    HIPCHK(hipMemcpyAsync(hs + o_b, db + o_b, 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    memcpy(best, hs + o_b, 4);
    return ORBG_OK;
}

// ---------------------------------------------------------------------------
// LocalMapping matchers (mapping_kernels.hip)
// ---------------------------------------------------------------------------
extern "C" int orbg_search_for_triangulation_batch_device(
    orbg_ctx *c, const orbg_keyframes *kfs, int cap, const int32_t *d_kf1, const int32_t *d_kf2,
    const orbg_triangulation_pair *d_geo, int npairs, int only_stereo, int check_ori,
    int32_t *d_matches12, int32_t *d_nmatches)
{
    if (!c || !kfs) return set_err(ORBG_EINVAL, "NULL argument");
    if (npairs < 0 || cap <= 0) return set_err(ORBG_EINVAL, "bad npairs / cap");
    if (npairs == 0) return ORBG_OK;
    if (!d_kf1 || !d_kf2 || !d_geo || !d_matches12 || !d_nmatches || !kfs->desc || !kfs->kps ||
        !kfs->counts || !kfs->fv_nodes || !kfs->fv_off || !kfs->fv_feats || !kfs->nfv)
        return set_err(ORBG_EINVAL, "NULL device array");
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = c->stream;
    int rc = 0;
    PROF_LAUNCH(c, "tri_match",
                rc = launch_tri_match(st, *kfs, cap, d_kf1, d_kf2, d_geo, npairs, c->scale,
                                      c->sigma2, c->p.nlevels, only_stereo, check_ori,
                                      d_matches12, d_nmatches));
    if (rc == -95) return set_err(ORBG_ENOTSUP, "SearchForTriangulation: more than 65535 features");
    if (rc) return set_err(ORBG_EIO, "k_tri_match launch failed");
    return ORBG_OK;
}

static int kf_check(const orbg_keyframe *k)
{
    if (!k || k->n < 0 || k->nfv < 0 || k->nfv > std::max(k->n, 0)) return 0;
    if (k->n && (!k->kps || !k->desc)) return 0;
    if (k->nfv && (!k->fv_nodes || !k->fv_off || !k->fv_feats)) return 0;
    for (int j = 0; j < k->nfv; j++)
        for (int i = k->fv_off[j]; i < k->fv_off[j + 1]; i++)
            if (k->fv_feats[i] < 0 || k->fv_feats[i] >= k->n) return 0;
    for (int i = 0; i < k->n; i++)
        if (k->kps[i].octave < 0 || k->kps[i].octave >= ORBG_MAX_LEVELS) return 0;
    return 1;
}

extern "C" int orbg_search_for_triangulation(orbg_ctx *c, const orbg_keyframe *kf1,
                                             const orbg_keyframe *kf2,
                                             const orbg_triangulation_pair *geo, int only_stereo,
                                             int check_ori, int32_t *matches12, int *nmatches)
{
    if (!c || !geo || !nmatches) return set_err(ORBG_EINVAL, "NULL argument");
    if (!kf_check(kf1) || !kf_check(kf2)) return set_err(ORBG_EINVAL, "bad KeyFrame arrays");
    if (kf1->n && !matches12) return set_err(ORBG_EINVAL, "NULL matches12");
    *nmatches = 0;
    for (int i = 0; i < kf1->n; i++) matches12[i] = -1;
    if (!kf1->n || !kf2->n || !kf1->nfv || !kf2->nfv) return ORBG_OK;
    HIPCHK(hipSetDevice(c->device));
    const int cap = std::max(kf1->n, kf2->n);
    if (cap > 65535) return set_err(ORBG_ENOTSUP, "more than 65535 features");
    const size_t cp = (size_t)cap;
    size_t o = 0;
    auto take = [&](size_t bytes) {
        const size_t r = o;
        o += al256(bytes);
        return r;
    };
    const size_t o_desc = take(2 * cp * 32), o_kps = take(2 * cp * sizeof(orbg_keypoint)),
                 o_ur = take(2 * cp * 4), o_mp = take(2 * cp), o_cnt = take(8),
                 o_nodes = take(2 * cp * 4), o_off = take(2 * (cp + 1) * 4),
                 o_feats = take(2 * cp * 4), o_nfv = take(8), o_idx = take(8),
                 o_geo = take(sizeof(orbg_triangulation_pair)), o_m = take(cp * 4), o_nm = take(4);
    uint8_t *hs;
    int rc = stage(c, o, &hs);
    if (rc) return rc;
    void *d;
    if ((rc = scratch(c, o, &d))) return rc;
    uint8_t *db = (uint8_t *)d;
    HIPCHK(hipStreamSynchronize(c->stream));
    memset(hs, 0, o_m);
    const orbg_keyframe *ks[2] = {kf1, kf2};
    for (int s = 0; s < 2; s++) {
        const orbg_keyframe *k = ks[s];
        memcpy(hs + o_desc + s * cp * 32, k->desc, (size_t)k->n * 32);
        memcpy(hs + o_kps + s * cp * sizeof(orbg_keypoint), k->kps, (size_t)k->n * sizeof(orbg_keypoint));
        float *ur = (float *)(hs + o_ur) + s * cp;
        for (int i = 0; i < k->n; i++) ur[i] = k->uright ? k->uright[i] : -1.0f;
        if (k->has_mp) memcpy(hs + o_mp + s * cp, k->has_mp, (size_t)k->n);
        ((int32_t *)(hs + o_cnt))[s] = k->n;
        memcpy(hs + o_nodes + s * cp * 4, k->fv_nodes, (size_t)k->nfv * 4);
        memcpy(hs + o_off + s * (cp + 1) * 4, k->fv_off, (size_t)(k->nfv + 1) * 4);
        memcpy(hs + o_feats + s * cp * 4, k->fv_feats, (size_t)k->fv_off[k->nfv] * 4);
        ((int32_t *)(hs + o_nfv))[s] = k->nfv;
        ((int32_t *)(hs + o_idx))[s] = s;
    }
    memcpy(hs + o_geo, geo, sizeof(orbg_triangulation_pair));
    HIPCHK(hipMemcpyAsync(db, hs, o_m, hipMemcpyHostToDevice, c->stream));
    orbg_keyframes K{};
    K.desc = db + o_desc;
    K.kps = (const orbg_keypoint *)(db + o_kps);
    K.uright = (const float *)(db + o_ur);
    K.has_mp = db + o_mp;
    K.counts = (const int32_t *)(db + o_cnt);
    K.fv_nodes = (const int32_t *)(db + o_nodes);
    K.fv_off = (const int32_t *)(db + o_off);
    K.fv_feats = (const int32_t *)(db + o_feats);
    K.nfv = (const int32_t *)(db + o_nfv);
    const int32_t *di = (const int32_t *)(db + o_idx);
    rc = launch_tri_match(c->stream, K, cap, di, di + 1, (const orbg_triangulation_pair *)(db + o_geo),
                          1, c->scale, c->sigma2, c->p.nlevels, only_stereo, check_ori,
                          (int32_t *)(db + o_m), (int32_t *)(db + o_nm));
    if (rc) return set_err(ORBG_EIO, "k_tri_match launch failed");
    HIPCHK(hipMemcpyAsync(hs + o_m, db + o_m, o - o_m, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    memcpy(matches12, hs + o_m, (size_t)kf1->n * 4);
    memcpy(nmatches, hs + o_nm, 4);
    return ORBG_OK;
}

extern "C" int orbg_triangulation_geometry_batch_device(orbg_ctx *c, const orbg_kf_camera *d_cams,
                                                        const int32_t *d_kf1, const int32_t *d_kf2,
                                                        int npairs, orbg_triangulation_pair *d_geo)
{
    if (!c) return set_err(ORBG_EINVAL, "NULL context");
    if (npairs < 0) return set_err(ORBG_EINVAL, "bad npairs");
    if (npairs == 0) return ORBG_OK;
    if (!d_cams || !d_kf1 || !d_kf2 || !d_geo) return set_err(ORBG_EINVAL, "NULL device array");
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = c->stream;
    int rc = 0;
    PROF_LAUNCH(c, "tri_geometry",
                rc = launch_tri_geometry(st, d_cams, d_kf1, d_kf2, npairs, d_geo));
    if (rc) return set_err(ORBG_EIO, "k_tri_geometry launch failed");
    return ORBG_OK;
}

extern "C" int orbg_triangulation_geometry(orbg_ctx *c, const orbg_kf_camera *cam1,
                                           const orbg_kf_camera *cam2, orbg_triangulation_pair *geo)
{
    if (!c || !cam1 || !cam2 || !geo) return set_err(ORBG_EINVAL, "NULL argument");
    HIPCHK(hipSetDevice(c->device));
    const size_t o_cam = 0, o_idx = al256(2 * sizeof(orbg_kf_camera)), o_geo = o_idx + 256,
                 o = o_geo + al256(sizeof(orbg_triangulation_pair));
    uint8_t *hs;
    int rc = stage(c, o, &hs);
    if (rc) return rc;
    void *d;
    if ((rc = scratch(c, o, &d))) return rc;
    uint8_t *db = (uint8_t *)d;
    HIPCHK(hipStreamSynchronize(c->stream));
    memcpy(hs + o_cam, cam1, sizeof(orbg_kf_camera));
    memcpy(hs + o_cam + sizeof(orbg_kf_camera), cam2, sizeof(orbg_kf_camera));
    ((int32_t *)(hs + o_idx))[0] = 0;
    ((int32_t *)(hs + o_idx))[1] = 1;
    HIPCHK(hipMemcpyAsync(db, hs, o_geo, hipMemcpyHostToDevice, c->stream));
    const int32_t *di = (const int32_t *)(db + o_idx);
    rc = launch_tri_geometry(c->stream, (const orbg_kf_camera *)(db + o_cam), di, di + 1, 1,
                             (orbg_triangulation_pair *)(db + o_geo));
    if (rc) return set_err(ORBG_EIO, "k_tri_geometry launch failed");
    HIPCHK(hipMemcpyAsync(hs + o_geo, db + o_geo, sizeof(orbg_triangulation_pair),
                          hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    memcpy(geo, hs + o_geo, sizeof(orbg_triangulation_pair));
    return ORBG_OK;
}

extern "C" int orbg_triangulate_batch_device(orbg_ctx *c, const orbg_keyframes *kfs,
                                             const orbg_keypoint *d_kps_raw, const float *d_depth,
                                             int cap, const orbg_kf_camera *d_cams,
                                             const int32_t *d_kf1, const int32_t *d_kf2,
                                             const int32_t *d_matches12, int npairs, float *d_x3d,
                                             int8_t *d_status, int32_t *d_nnew)
{
    if (!c || !kfs) return set_err(ORBG_EINVAL, "NULL argument");
    if (npairs < 0 || cap <= 0) return set_err(ORBG_EINVAL, "bad npairs / cap");
    if (npairs == 0) return ORBG_OK;
    if (npairs > 65535) return set_err(ORBG_ENOTSUP, "more than 65535 pairs per call");
    if (!kfs->kps || !kfs->counts || !d_cams || !d_kf1 || !d_kf2 || !d_matches12 || !d_x3d ||
        !d_status || !d_nnew)
        return set_err(ORBG_EINVAL, "NULL device array");
    if (kfs->uright && !d_depth) return set_err(ORBG_EINVAL, "mvuRight without mvDepth");
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = c->stream;
    int rc = 0;
    PROF_LAUNCH(c, "triangulate",
                rc = launch_triangulate(st, *kfs, d_kps_raw, d_depth, cap, d_cams, d_kf1,
                                        d_kf2, d_matches12, npairs, c->scale, c->sigma2,
                                        c->p.nlevels, c->p.scale_factor, d_x3d, d_status, d_nnew));
    if (rc) return set_err(ORBG_EIO, "k_triangulate launch failed");
    return ORBG_OK;
}

extern "C" int orbg_triangulate(orbg_ctx *c, const orbg_keyframe_geo *kf1,
                                const orbg_keyframe_geo *kf2, const orbg_kf_camera *cam1,
                                const orbg_kf_camera *cam2, const int32_t *matches12, float *x3d,
                                int8_t *status, int *nnew)
{
    if (!c || !kf1 || !kf2 || !cam1 || !cam2 || !nnew) return set_err(ORBG_EINVAL, "NULL argument");
    const orbg_keyframe_geo *ks[2] = {kf1, kf2};
    for (const orbg_keyframe_geo *k : ks) {
        if (k->n < 0 || (k->n && !k->kps)) return set_err(ORBG_EINVAL, "bad KeyFrame arrays");
        if (k->n && k->uright && !k->depth) return set_err(ORBG_EINVAL, "mvuRight without mvDepth");
    }
    if (kf1->n && (!matches12 || !x3d || !status)) return set_err(ORBG_EINVAL, "NULL output");
    *nnew = 0;
    if (!kf1->n) return ORBG_OK;
    HIPCHK(hipSetDevice(c->device));
    const int cap = std::max(kf1->n, kf2->n);
    const size_t cp = (size_t)cap;
    size_t o = 0;
    auto take = [&](size_t bytes) {
        const size_t r = o;
        o += al256(bytes);
        return r;
    };
    const size_t o_kps = take(2 * cp * sizeof(orbg_keypoint)),
                 o_raw = take(2 * cp * sizeof(orbg_keypoint)), o_ur = take(2 * cp * 4),
                 o_dp = take(2 * cp * 4), o_cnt = take(8), o_idx = take(8),
                 o_cam = take(2 * sizeof(orbg_kf_camera)), o_m = take(cp * 4),
                 o_x = take(cp * 12), o_st = take(cp), o_nn = take(4);
    uint8_t *hs;
    int rc = stage(c, o, &hs);
    if (rc) return rc;
    void *d;
    if ((rc = scratch(c, o, &d))) return rc;
    uint8_t *db = (uint8_t *)d;
    HIPCHK(hipStreamSynchronize(c->stream));
    memset(hs, 0, o_x);
    for (int s = 0; s < 2; s++) {
        const orbg_keyframe_geo *k = ks[s];
        const size_t n = (size_t)k->n;
        memcpy(hs + o_kps + s * cp * sizeof(orbg_keypoint), k->kps, n * sizeof(orbg_keypoint));
        memcpy(hs + o_raw + s * cp * sizeof(orbg_keypoint), k->kps_raw ? k->kps_raw : k->kps,
               n * sizeof(orbg_keypoint));
        float *ur = (float *)(hs + o_ur) + s * cp, *dp = (float *)(hs + o_dp) + s * cp;
        for (size_t i = 0; i < n; i++) {
            ur[i] = k->uright ? k->uright[i] : -1.0f;
            dp[i] = k->uright ? k->depth[i] : 0.0f;
        }
        ((int32_t *)(hs + o_cnt))[s] = k->n;
        ((int32_t *)(hs + o_idx))[s] = s;
    }
    memcpy(hs + o_cam, cam1, sizeof(orbg_kf_camera));
    memcpy(hs + o_cam + sizeof(orbg_kf_camera), cam2, sizeof(orbg_kf_camera));
    memcpy(hs + o_m, matches12, (size_t)kf1->n * 4);
    for (int i = kf1->n; i < cap; i++) ((int32_t *)(hs + o_m))[i] = -1;
    HIPCHK(hipMemcpyAsync(db, hs, o_x, hipMemcpyHostToDevice, c->stream));
    orbg_keyframes K{};
    K.kps = (const orbg_keypoint *)(db + o_kps);
    K.uright = (const float *)(db + o_ur);
    K.counts = (const int32_t *)(db + o_cnt);
    const int32_t *di = (const int32_t *)(db + o_idx);
    rc = launch_triangulate(c->stream, K, (const orbg_keypoint *)(db + o_raw),
                            (const float *)(db + o_dp), cap, (const orbg_kf_camera *)(db + o_cam),
                            di, di + 1, (const int32_t *)(db + o_m), 1, c->scale, c->sigma2,
                            c->p.nlevels, c->p.scale_factor, (float *)(db + o_x),
                            (int8_t *)(db + o_st), (int32_t *)(db + o_nn));
    if (rc) return set_err(ORBG_EIO, "k_triangulate launch failed");
    HIPCHK(hipMemcpyAsync(hs + o_x, db + o_x, o - o_x, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    memcpy(x3d, hs + o_x, (size_t)kf1->n * 12);
    memcpy(status, hs + o_st, (size_t)kf1->n);
    memcpy(nnew, hs + o_nn, 4);
    return ORBG_OK;
}

static int fuse_batch(orbg_ctx *c, const orbg_keyframes *kfs, int cap, const int32_t *d_kf,
                      const orbg_frustum_camera *d_cams, const orbg_map_point *d_mps,
                      const uint8_t *d_mdesc, const int32_t *d_mcounts, int mcap, int npairs,
                      float th, int sim3, int32_t *d_best_idx, int32_t *d_best_dist,
                      int32_t *d_nfused)
{
    if (!c || !kfs) return set_err(ORBG_EINVAL, "NULL argument");
    if (npairs < 0 || cap <= 0 || mcap < 0) return set_err(ORBG_EINVAL, "bad sizes");
    if (npairs == 0) return ORBG_OK;
    if (!d_nfused) return set_err(ORBG_EINVAL, "NULL device array");
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = c->stream;
    if (mcap == 0) {  // no MapPoints: every pair fuses nothing (orbg.h: d_nfused is written)
        HIPCHK(hipMemsetAsync(d_nfused, 0, (size_t)npairs * sizeof(int32_t), st));
        return ORBG_OK;
    }
    if (!d_kf || !d_cams || !d_mps || !d_mdesc || !d_mcounts || !d_best_idx || !d_best_dist ||
        !kfs->desc || !kfs->kps || !kfs->counts)
        return set_err(ORBG_EINVAL, "NULL device array");
    int rc = 0;
    PROF_LAUNCH(c, sim3 ? "fuse_sim3" : "fuse",
                rc = launch_fuse(st, *kfs, cap, d_kf, d_cams, d_mps, d_mdesc, d_mcounts, mcap,
                                 npairs, th, c->scale, c->inv_sigma2, c->p.nlevels, sim3,
                                 d_best_idx, d_best_dist, d_nfused, c->d_err));
    if (rc == -95) return set_err(ORBG_ENOTSUP, "Fuse: more than 8192 keypoints per KeyFrame");
    if (rc) return set_err(ORBG_EIO, "k_fuse launch failed");
    return ORBG_OK;
}

extern "C" int orbg_fuse_batch_device(orbg_ctx *c, const orbg_keyframes *kfs, int cap,
                                      const int32_t *d_kf, const orbg_frustum_camera *d_cams,
                                      const orbg_map_point *d_mps, const uint8_t *d_mdesc,
                                      const int32_t *d_mcounts, int mcap, int npairs, float th,
                                      int32_t *d_best_idx, int32_t *d_best_dist,
                                      int32_t *d_nfused)
{
    return fuse_batch(c, kfs, cap, d_kf, d_cams, d_mps, d_mdesc, d_mcounts, mcap, npairs, th, 0,
                      d_best_idx, d_best_dist, d_nfused);
}

extern "C" int orbg_fuse_sim3_batch_device(orbg_ctx *c, const orbg_keyframes *kfs, int cap,
                                           const int32_t *d_kf, const orbg_frustum_camera *d_cams,
                                           const orbg_map_point *d_mps, const uint8_t *d_mdesc,
                                           const int32_t *d_mcounts, int mcap, int npairs,
                                           float th, int32_t *d_best_idx, int32_t *d_best_dist,
                                           int32_t *d_nfused)
{
    return fuse_batch(c, kfs, cap, d_kf, d_cams, d_mps, d_mdesc, d_mcounts, mcap, npairs, th, 1,
                      d_best_idx, d_best_dist, d_nfused);
}

static int fuse_host(orbg_ctx *c, const orbg_keyframe *kf, const orbg_frustum_camera *cam,
                     const orbg_map_point *mps, const uint8_t *mdesc, int nmp, float th, int sim3,
                     int32_t *best_idx, int32_t *best_dist, int *nfused)
{
    if (!c || !kf || !cam || !nfused) return set_err(ORBG_EINVAL, "NULL argument");
    if (nmp < 0 || kf->n < 0) return set_err(ORBG_EINVAL, "negative size");
    if (kf->n && (!kf->kps || !kf->desc)) return set_err(ORBG_EINVAL, "NULL KeyFrame array");
    if (nmp && (!mps || !mdesc || !best_idx || !best_dist)) return set_err(ORBG_EINVAL, "NULL array");
    for (int i = 0; i < kf->n; i++)
        if (kf->kps[i].octave < 0 || kf->kps[i].octave >= ORBG_MAX_LEVELS)
            return set_err(ORBG_EINVAL, "keypoint octave out of range");
    *nfused = 0;
    if (nmp == 0) return ORBG_OK;
    HIPCHK(hipSetDevice(c->device));
    const int cap = std::max(kf->n, 1);
    if (cap > 8192) return set_err(ORBG_ENOTSUP, "more than 8192 keypoints");
    const size_t cp = (size_t)cap, nm = (size_t)nmp;
    size_t o = 0;
    auto take = [&](size_t bytes) {
        const size_t r = o;
        o += al256(bytes);
        return r;
    };
    const size_t o_desc = take(cp * 32), o_kps = take(cp * sizeof(orbg_keypoint)),
                 o_ur = take(cp * 4), o_cnt = take(4), o_idx = take(4),
                 o_cam = take(sizeof(orbg_frustum_camera)), o_mp = take(nm * sizeof(orbg_map_point)),
                 o_md = take(nm * 32), o_mc = take(4), o_bi = take(nm * 4), o_bd = take(nm * 4),
                 o_nf = take(4);
    uint8_t *hs;
    int rc = stage(c, o, &hs);
    if (rc) return rc;
    void *d;
    if ((rc = scratch(c, o, &d))) return rc;
    uint8_t *db = (uint8_t *)d;
    HIPCHK(hipStreamSynchronize(c->stream));
    memcpy(hs + o_desc, kf->desc, (size_t)kf->n * 32);
    memcpy(hs + o_kps, kf->kps, (size_t)kf->n * sizeof(orbg_keypoint));
    float *ur = (float *)(hs + o_ur);
    for (int i = 0; i < kf->n; i++) ur[i] = kf->uright ? kf->uright[i] : -1.0f;
    ((int32_t *)(hs + o_cnt))[0] = kf->n;
    ((int32_t *)(hs + o_idx))[0] = 0;
    memcpy(hs + o_cam, cam, sizeof(orbg_frustum_camera));
    memcpy(hs + o_mp, mps, nm * sizeof(orbg_map_point));
    memcpy(hs + o_md, mdesc, nm * 32);
    ((int32_t *)(hs + o_mc))[0] = nmp;
    HIPCHK(hipMemcpyAsync(db, hs, o_bi, hipMemcpyHostToDevice, c->stream));
    orbg_keyframes K{};
    K.desc = db + o_desc;
    K.kps = (const orbg_keypoint *)(db + o_kps);
    K.uright = (const float *)(db + o_ur);
    K.counts = (const int32_t *)(db + o_cnt);
    rc = launch_fuse(c->stream, K, cap, (const int32_t *)(db + o_idx),
                     (const orbg_frustum_camera *)(db + o_cam), (const orbg_map_point *)(db + o_mp),
                     db + o_md, (const int32_t *)(db + o_mc), nmp, 1, th, c->scale, c->inv_sigma2,
                     c->p.nlevels, sim3, (int32_t *)(db + o_bi), (int32_t *)(db + o_bd),
                     (int32_t *)(db + o_nf), c->d_err);
    if (rc) return set_err(ORBG_EIO, "k_fuse launch failed");
    HIPCHK(hipMemcpyAsync(hs + o_bi, db + o_bi, o - o_bi, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    memcpy(best_idx, hs + o_bi, nm * 4);
    memcpy(best_dist, hs + o_bd, nm * 4);
    memcpy(nfused, hs + o_nf, 4);
    return ORBG_OK;
}

// scratch for k_sim3_match's vnMatch1 / vnMatch2 (npairs * 2 * cap int32): a buffer of its
// own (not the tracking matchers' d_trk), so neither path depends on the other's stream.
// Growing it synchronises c->stream, the only stream its kernels are enqueued on.
static int sim3_scratch(orbg_ctx *c, size_t need, void **out)
{
    if (c->sim3_bytes < need) {
        HIPCHK(hipStreamSynchronize(c->stream));
        if (c->d_sim3) hipFree(c->d_sim3);
        c->d_sim3 = nullptr;
        c->sim3_bytes = 0;
        if (hipMalloc(&c->d_sim3, need) != hipSuccess)
            return set_err(ORBG_ENOMEM, "SearchBySim3 scratch %zu bytes", need);
        c->sim3_bytes = need;
    }
    *out = c->d_sim3;
    return ORBG_OK;
}

extern "C" int orbg_search_by_sim3_batch_device(orbg_ctx *c, const orbg_keyframes *kfs, int cap,
                                                const int32_t *d_kf1, const int32_t *d_kf2,
                                                const orbg_sim3_pair *d_pairs,
                                                const orbg_map_point *d_mps,
                                                const uint8_t *d_mdesc,
                                                const uint8_t *d_matched1,
                                                const uint8_t *d_matched2, int npairs, float th,
                                                int32_t *d_matches12, int32_t *d_nfound)
{
    if (!c || !kfs) return set_err(ORBG_EINVAL, "NULL argument");
    if (npairs < 0 || cap <= 0) return set_err(ORBG_EINVAL, "bad sizes");
    if (npairs == 0) return ORBG_OK;
    if (!d_kf1 || !d_kf2 || !d_pairs || !d_mps || !d_mdesc || !d_matches12 || !d_nfound ||
        !kfs->desc || !kfs->kps || !kfs->counts)
        return set_err(ORBG_EINVAL, "NULL device array");
    if (cap > 8192) return set_err(ORBG_ENOTSUP, "SearchBySim3: more than 8192 keypoints");
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = c->stream;
    void *vn;
    int rc = sim3_scratch(c, (size_t)npairs * 2 * cap * 4, &vn);
    if (rc) return rc;
    PROF_LAUNCH(c, "sim3_match",
                rc = launch_search_by_sim3(st, *kfs, cap, d_kf1, d_kf2, d_pairs, d_mps,
                                           d_mdesc, d_matched1, d_matched2, npairs, th, c->scale,
                                           c->p.nlevels, (int32_t *)vn, d_matches12, d_nfound,
                                           c->d_err));
    if (rc) return set_err(ORBG_EIO, "k_sim3_match launch failed");
    return ORBG_OK;
}

extern "C" int orbg_search_by_sim3(orbg_ctx *c, const orbg_keyframe *kf1, const orbg_map_point *mp1,
                                   const uint8_t *md1, const uint8_t *matched1,
                                   const orbg_keyframe *kf2, const orbg_map_point *mp2,
                                   const uint8_t *md2, const uint8_t *matched2,
                                   const orbg_sim3_pair *g, float th, int32_t *matches12,
                                   int *nfound)
{
    if (!c || !kf1 || !kf2 || !g || !nfound) return set_err(ORBG_EINVAL, "NULL argument");
    if (kf1->n < 0 || kf2->n < 0) return set_err(ORBG_EINVAL, "negative size");
    const orbg_keyframe *kk[2] = {kf1, kf2};
    for (int s = 0; s < 2; s++) {
        if (kk[s]->n && (!kk[s]->kps || !kk[s]->desc)) return set_err(ORBG_EINVAL, "NULL KeyFrame array");
        for (int i = 0; i < kk[s]->n; i++)
            if (kk[s]->kps[i].octave < 0 || kk[s]->kps[i].octave >= ORBG_MAX_LEVELS)
                return set_err(ORBG_EINVAL, "keypoint octave out of range");
    }
    if ((kf1->n && (!mp1 || !md1 || !matches12)) || (kf2->n && (!mp2 || !md2)))
        return set_err(ORBG_EINVAL, "NULL map point array");
    *nfound = 0;
    for (int i = 0; i < kf1->n; i++) matches12[i] = -1;
    if (kf1->n == 0 || kf2->n == 0) return ORBG_OK;
    HIPCHK(hipSetDevice(c->device));
    const int cap = std::max(kf1->n, kf2->n);
    if (cap > 8192) return set_err(ORBG_ENOTSUP, "more than 8192 keypoints");
    const size_t cp = (size_t)cap;
    size_t o = 0;
    auto take = [&](size_t bytes) {
        const size_t r = o;
        o += al256(bytes);
        return r;
    };
    const size_t o_desc = take(2 * cp * 32), o_kps = take(2 * cp * sizeof(orbg_keypoint)),
                 o_cnt = take(8), o_idx = take(8), o_pair = take(sizeof(orbg_sim3_pair)),
                 o_mp = take(2 * cp * sizeof(orbg_map_point)), o_md = take(2 * cp * 32),
                 o_am1 = take(cp), o_am2 = take(cp), o_m = take(cp * 4), o_nf = take(4);
    uint8_t *hs;
    int rc = stage(c, o, &hs);
    if (rc) return rc;
    void *d;
    if ((rc = scratch(c, o, &d))) return rc;
    uint8_t *db = (uint8_t *)d;
    HIPCHK(hipStreamSynchronize(c->stream));
    memset(hs, 0, o_m);
    const orbg_map_point *mpp[2] = {mp1, mp2};
    const uint8_t *mdp[2] = {md1, md2}, *amp[2] = {matched1, matched2};
    for (int s = 0; s < 2; s++) {
        const size_t n = (size_t)kk[s]->n;
        memcpy(hs + o_desc + s * cp * 32, kk[s]->desc, n * 32);
        memcpy(hs + o_kps + s * cp * sizeof(orbg_keypoint), kk[s]->kps, n * sizeof(orbg_keypoint));
        ((int32_t *)(hs + o_cnt))[s] = kk[s]->n;
        ((int32_t *)(hs + o_idx))[s] = s;
        memcpy(hs + o_mp + s * cp * sizeof(orbg_map_point), mpp[s], n * sizeof(orbg_map_point));
        memcpy(hs + o_md + s * cp * 32, mdp[s], n * 32);
        if (amp[s]) memcpy(hs + (s ? o_am2 : o_am1), amp[s], n);
    }
    memcpy(hs + o_pair, g, sizeof(orbg_sim3_pair));
    HIPCHK(hipMemcpyAsync(db, hs, o_m, hipMemcpyHostToDevice, c->stream));
    orbg_keyframes K{};
    K.desc = db + o_desc;
    K.kps = (const orbg_keypoint *)(db + o_kps);
    K.counts = (const int32_t *)(db + o_cnt);
    void *vn;
    if ((rc = sim3_scratch(c, cp * 2 * 4, &vn))) return rc;
    rc = launch_search_by_sim3(c->stream, K, cap, (const int32_t *)(db + o_idx),
                               (const int32_t *)(db + o_idx) + 1,
                               (const orbg_sim3_pair *)(db + o_pair),
                               (const orbg_map_point *)(db + o_mp), db + o_md, db + o_am1,
                               db + o_am2, 1, th, c->scale, c->p.nlevels, (int32_t *)vn,
                               (int32_t *)(db + o_m), (int32_t *)(db + o_nf), c->d_err);
    if (rc) return set_err(ORBG_EIO, "k_sim3_match launch failed");
    HIPCHK(hipMemcpyAsync(hs + o_m, db + o_m, o - o_m, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    memcpy(matches12, hs + o_m, (size_t)kf1->n * 4);
    memcpy(nfound, hs + o_nf, 4);
    return ORBG_OK;
}

extern "C" int orbg_fuse(orbg_ctx *c, const orbg_keyframe *kf, const orbg_frustum_camera *cam,
                         const orbg_map_point *mps, const uint8_t *mdesc, int nmp, float th,
                         int32_t *best_idx, int32_t *best_dist, int *nfused)
{
    return fuse_host(c, kf, cam, mps, mdesc, nmp, th, 0, best_idx, best_dist, nfused);
}

extern "C" int orbg_fuse_sim3(orbg_ctx *c, const orbg_keyframe *kf, const orbg_frustum_camera *cam,
                              const orbg_map_point *mps, const uint8_t *mdesc, int nmp, float th,
                              int32_t *best_idx, int32_t *best_dist, int *nfused)
{
    return fuse_host(c, kf, cam, mps, mdesc, nmp, th, 1, best_idx, best_dist, nfused);
}
