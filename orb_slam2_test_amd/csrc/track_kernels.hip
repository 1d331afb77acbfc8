// track_kernels.hip -- the per-frame tracking matchers for gfx950.
//
//   ORBmatcher::SearchByProjection(CurrentFrame, LastFrame, th, bMono)
//       (ORBmatcher.cc:1503-1667; Tracking::TrackWithMotionModel)
//   ORBmatcher::SearchByProjection(F, vpMapPoints, th)
//       (ORBmatcher.cc:59-146, RadiusByViewingCos :148-154; Tracking::SearchLocalPoints)
//   ORBmatcher::SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist)
//       (ORBmatcher.cc:1670-1798; Tracking::Relocalization)                  [TRK_RELOC]
//   ORBmatcher::SearchByProjection(pKF, Scw, vpPoints, vpMatched, th)
//       (ORBmatcher.cc:353-470; LoopClosing::ComputeSim3)                     [TRK_LOOP]
// The last two write every pick (mvpMapPoints[i2] / vpMatched[idx] != NULL is the skip), so
// their queries always take; RELOC keeps the rotation histogram, LOOP is TH_LOW on a
// KeyFrame (int bounds for IsInImage and the cell range, the level window after the area).
//
// Both are "project, window search, best Hamming distance" loops whose only order
// dependence is the skip of a keypoint that an earlier query already took
// (mvpMapPoints[i2] && Observations() > 0) plus, for the last-frame search, the rotation
// histogram.  Split like SearchForInitialization (match_kernels.hip):
//   k_track_cands    data parallel: per query, the window candidates of
//                    Frame::GetFeaturesInArea with the level and stereo filters, kept as
//                    the K smallest (distance, grid order, index) keys.  The frame's
//                    keypoints are counting-sorted by grid column in LDS once per
//                    workgroup; 16-lane groups, 4 queries per wave at a time.
//   k_track_resolve  one workgroup per frame: wave 0 walks the queries in index order over
//                    the K-lists in LDS while wave 1 prefetches the next chunk
//                    (the first two keys whose keypoint is not taken are best / second),
//                    with an exact wave-parallel rescan when a K-list runs out; then the
//                    rotation-consistency pass (ComputeThreeMaxima) for the last-frame
//                    search.
// Distances of 256 never change either loop's state (bestDist starts at 256), so keys
// with d = 256 are dropped.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>

#include "../../include/orbg.h"
#include "orbg_internal.h"
#include "orbg_device.h"
#include "frame_device.h"
#include "match_device.h"
#include "track_args.h"

#pragma clang fp contract(off)

namespace orbg {

void prof_begin(void *prof, hipStream_t s, const char *n, hipEvent_t *a);
void prof_end(void *prof, hipStream_t s, const char *n, hipEvent_t a);

#define TH_HIGH 100
#define TH_LOW 50
#define HISTO_LENGTH 30
#define TRK_ROT(m) ((m) == TRK_LASTFRAME || (m) == TRK_RELOC)  // rotation histogram
#ifndef TRK_QPW
#define TRK_QPW 32  // queries per wave in k_track_cands (8 x 4 in 16-lane groups)
#endif
#define TRK_NB (ORBG_MAX_LEVELS * ORBG_GRID_COLS)  // (octave, column) buckets

// cv::gemm small-matrix pin (see oracle/track_oracle.c orc_gemm3): double work type, one
// rounding per element.  R = 3x3 block of a 3x4 row-major matrix.
__device__ __forceinline__ void gemm3(const float *R, bool trans, const float x[3], double alpha,
                                      const float *c, float out[3])
{
#pragma unroll
    for (int r = 0; r < 3; r++) {
        double t = 0.0;
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const float a = trans ? R[4 * k + r] : R[4 * r + k];
            t += (double)a * (double)x[k];
        }
        t *= alpha;
        if (c) t += (double)c[r];
        out[r] = (float)t;
    }
}

// the search a query runs: window centre / radius, level range, stereo test
struct TrackQuery {
    bool valid;
    float x, y, r;          // GetFeaturesInArea(x, y, r, minL, maxL)
    int minL, maxL;
    float ur, ur_thr;       // skip i2 with uRight > 0 and |ur - uRight| > ur_thr
    bool has_obs;           // pMP->Observations() > 0
};

// ORBmatcher.cc:1511-1522 (bForward / bBackward), per frame
__device__ __forceinline__ void track_direction(const orbg_track_camera &cam, bool *fwd, bool *bwd)
{
    const float tcw[3] = {cam.Tcw[3], cam.Tcw[7], cam.Tcw[11]};
    const float tlw[3] = {cam.Tlw[3], cam.Tlw[7], cam.Tlw[11]};
    float twc[3], tlc[3];
    gemm3(cam.Tcw, true, tcw, -1.0, nullptr, twc);
    gemm3(cam.Tlw, false, twc, 1.0, tlw, tlc);
    *fwd = tlc[2] > cam.b && !cam.mono;
    *bwd = -tlc[2] > cam.b && !cam.mono;
}

template <int MODE>
__device__ TrackQuery track_query(const TrackArgs &A, int f, int i, bool fwd, bool bwd,
                                  const orbg_bounds &b)
{
    TrackQuery Q;
    Q.valid = false;
    if (MODE == TRK_LASTFRAME) {
        // ORBmatcher.cc:1528-1580
        const orbg_lastframe_point P = ((const orbg_lastframe_point *)A.q)[(size_t)f * A.qc + i];
        if (!(P.flags & ORBG_MP_VALID)) return Q;
        const orbg_track_camera &cam = A.cams[f];
        const float tcw[3] = {cam.Tcw[3], cam.Tcw[7], cam.Tcw[11]};
        const float X[3] = {P.x, P.y, P.z};
        float xc[3];
        gemm3(cam.Tcw, false, X, 1.0, tcw, xc);
        const float invzc = (float)(1.0 / (double)xc[2]);
        if (invzc < 0) return Q;
        const float u = cam.fx * xc[0] * invzc + cam.cx;
        const float v = cam.fy * xc[1] * invzc + cam.cy;
        if (u < b.min_x || u > b.max_x) return Q;
        if (v < b.min_y || v > b.max_y) return Q;
        const int o = P.octave;
        Q.r = A.th * A.scale[o];
        if (fwd) {
            Q.minL = o;
            Q.maxL = -1;
        } else if (bwd) {
            Q.minL = 0;
            Q.maxL = o;
        } else {
            Q.minL = o - 1;
            Q.maxL = o + 1;
        }
        Q.x = u;
        Q.y = v;
        Q.ur = u - cam.bf * invzc;
        Q.ur_thr = Q.r;
        Q.has_obs = (P.flags & ORBG_MP_HAS_OBS) != 0;
    } else if (MODE == TRK_RELOC) {
        // ORBmatcher.cc:1689-1727 (no depth test: the reference has none)
        const orbg_reloc_point P = ((const orbg_reloc_point *)A.q)[(size_t)f * A.qc + i];
        if (!(P.flags & ORBG_MP_VALID)) return Q;
        const orbg_frustum_camera &cam = A.fcams[f];
        const float tcw[3] = {cam.Tcw[3], cam.Tcw[7], cam.Tcw[11]};
        const float X[3] = {P.x, P.y, P.z};
        float xc[3], Ow[3];
        gemm3(cam.Tcw, false, X, 1.0, tcw, xc);
        const float invzc = (float)(1.0 / (double)xc[2]);
        const float u = cam.fx * xc[0] * invzc + cam.cx;
        const float v = cam.fy * xc[1] * invzc + cam.cy;
        if (u < b.min_x || u > b.max_x) return Q;
        if (v < b.min_y || v > b.max_y) return Q;
        gemm3(cam.Tcw, true, tcw, -1.0, nullptr, Ow);
        const float PO0 = X[0] - Ow[0], PO1 = X[1] - Ow[1], PO2 = X[2] - Ow[2];
        double s = 0.0;
        s += (double)PO0 * (double)PO0;
        s += (double)PO1 * (double)PO1;
        s += (double)PO2 * (double)PO2;
        const float dist3D = (float)sqrt(s);
        const float maxDistance = 1.2f * P.max_dist, minDistance = 0.8f * P.min_dist;
        if (dist3D < minDistance || dist3D > maxDistance) return Q;
        const int lvl = predict_scale(P.max_dist, dist3D, cam.log_scale_factor, cam.nlevels);
        Q.r = A.th * A.scale[lvl];
        Q.minL = lvl - 1;
        Q.maxL = lvl + 1;
        Q.x = u;
        Q.y = v;
        Q.ur = 0.f;
        Q.ur_thr = INFINITY;  // no stereo test
        Q.has_obs = true;     // every pick is written: a later point skips it
    } else if (MODE == TRK_LOOP) {
        // ORBmatcher.cc:379-425 on pKF with the decomposed Scw
        const orbg_map_point M = ((const orbg_map_point *)A.q)[(size_t)f * A.qc + i];
        if (!(M.flags & ORBG_MP_VALID)) return Q;
        const orbg_frustum_camera &cam = A.fcams[f];
        float T[12];
        sim3_decompose(cam.Tcw, T);
        const float tcw[3] = {T[3], T[7], T[11]};
        const float X[3] = {M.x, M.y, M.z};
        float Pc[3], Ow[3];
        gemm3(T, false, X, 1.0, tcw, Pc);
        if (Pc[2] < 0.0f) return Q;
        const float invz = 1 / Pc[2];
        const float x = Pc[0] * invz, y = Pc[1] * invz;
        const float u = cam.fx * x + cam.cx, v = cam.fy * y + cam.cy;
        // KeyFrame::IsInImage on the KeyFrame's int bounds (KeyFrame.h:288-291)
        const float kminx = (float)(int)b.min_x, kmaxx = (float)(int)b.max_x;
        const float kminy = (float)(int)b.min_y, kmaxy = (float)(int)b.max_y;
        if (!(u >= kminx && u < kmaxx && v >= kminy && v < kmaxy)) return Q;
        gemm3(T, true, tcw, -1.0, nullptr, Ow);
        const float PO0 = X[0] - Ow[0], PO1 = X[1] - Ow[1], PO2 = X[2] - Ow[2];
        double s = 0.0;
        s += (double)PO0 * (double)PO0;
        s += (double)PO1 * (double)PO1;
        s += (double)PO2 * (double)PO2;
        const float dist = (float)sqrt(s);
        const float maxDistance = 1.2f * M.max_dist, minDistance = 0.8f * M.min_dist;
        if (dist < minDistance || dist > maxDistance) return Q;
        double dot = 0.0;
        dot += (double)PO0 * (double)M.nx;
        dot += (double)PO1 * (double)M.ny;
        dot += (double)PO2 * (double)M.nz;
        if (dot < 0.5 * (double)dist) return Q;
        const int lvl = predict_scale(M.max_dist, dist, cam.log_scale_factor, cam.nlevels);
        Q.r = A.th * A.scale[lvl];
        Q.minL = lvl - 1;  // the loop's kpLevel window, applied after GetFeaturesInArea
        Q.maxL = lvl;
        Q.x = u;
        Q.y = v;
        Q.ur = 0.f;
        Q.ur_thr = INFINITY;
        Q.has_obs = true;
    } else {
        // ORBmatcher.cc:63-86
        const orbg_map_projection M = ((const orbg_map_projection *)A.q)[(size_t)f * A.qc + i];
        if (!(M.flags & ORBG_MP_VALID)) return Q;
        float r = (double)M.view_cos > 0.998 ? 2.5f : 4.0f;
        if ((double)A.th != 1.0) r *= A.th;
        Q.r = r * A.scale[M.level];
        Q.minL = M.level - 1;
        Q.maxL = M.level;
        Q.x = M.u;
        Q.y = M.v;
        Q.ur = M.ur;
        Q.ur_thr = r * A.scale[M.level];
        Q.has_obs = (M.flags & ORBG_MP_HAS_OBS) != 0;
    }
    Q.valid = true;
    return Q;
}

// KeyFrame::GetFeaturesInArea's cell range uses the KeyFrame's int mnMinX / mnMinY (the
// Frame's truncated) with the Frame's cell sizes; PosInGrid stays the Frame's
__device__ __forceinline__ GridPrm kf_window_prm(GridPrm g)
{
    g.min_x = (float)(int)g.min_x;
    g.min_y = (float)(int)g.min_y;
    return g;
}

// level / stereo filters of one keypoint (GetFeaturesInArea's bCheckLevels, :475-482, and
// the uRight test)
__device__ __forceinline__ bool track_static_ok(const TrackQuery &Q, int octave, float ur)
{
    if (Q.minL > 0 || Q.maxL >= 0) {
        if (octave < Q.minL) return false;
        if (Q.maxL >= 0 && octave > Q.maxL) return false;
    }
    if (ur > 0) {
        const float er = fabsf(Q.ur - ur);
        if (er > Q.ur_thr) return false;
    }
    return true;
}

// LDS image of one frame's keypoints, sorted by grid column
struct TKey {
    float x, y;
    uint32_t idx_oct;  // index | octave << 24
    float ur;
};

template <int MODE>
__global__ __launch_bounds__(256) void k_track_cands(TrackArgs A)
{
    extern __shared__ __attribute__((aligned(16))) TKey fk[];
    // bucket = octave * 64 + grid column: a query scans only its level range's columns
    __shared__ int colstart[TRK_NB + 1];
    __shared__ int cursor[TRK_NB];
    __shared__ int wsum[4];
    const int nbx = (A.qc + 4 * TRK_QPW - 1) / (4 * TRK_QPW);
    const int id = xcd_remap(blockIdx.x, gridDim.x);
    const int f = id / nbx, bx = id - f * nbx;
    const int nq = A.qcounts[f], n = A.counts[f];
    const int qbase = bx * 4 * TRK_QPW;
    if (qbase >= nq) return;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const orbg_bounds b = A.bounds[f];
    const GridPrm g = grid_prm(b);
    const orbg_keypoint *kps = A.kps + (size_t)f * A.fc;
    const float *urf = A.uright ? A.uright + (size_t)f * A.fc : nullptr;
    // counting sort by (octave, PosInGrid column) (Frame.cc:510-520); keypoints outside
    // the grid are in no cell and never candidates
    for (int i = tid; i <= TRK_NB; i += 256) colstart[i] = 0;
    __syncthreads();
    auto bucket = [&](const orbg_keypoint &kp) -> int {
        const int px = (int)roundf((kp.x - g.min_x) * g.inv_w);
        const int py = (int)roundf((kp.y - g.min_y) * g.inv_h);
        if (px < 0 || px >= ORBG_GRID_COLS || py < 0 || py >= ORBG_GRID_ROWS) return -1;
        return min(max(kp.octave, 0), ORBG_MAX_LEVELS - 1) * ORBG_GRID_COLS + px;
    };
    for (int i = tid; i < n; i += 256) {
        const int bk = bucket(kps[i]);
        if (bk >= 0) atomicAdd(&colstart[bk + 1], 1);
    }
    __syncthreads();
    {
        // inclusive scan of colstart[1..TRK_NB]: 4 consecutive buckets per thread
        int v[4], run = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            run += colstart[1 + 4 * tid + k];
            v[k] = run;
        }
        const int incl = wave_incl_scan(run);
        if (lane == 63) wsum[wv] = incl;
        __syncthreads();
        int base = incl - run;
        for (int w2 = 0; w2 < wv; w2++) base += wsum[w2];
#pragma unroll
        for (int k = 0; k < 4; k++) colstart[1 + 4 * tid + k] = base + v[k];
    }
    __syncthreads();
    for (int i = tid; i < TRK_NB; i += 256) cursor[i] = colstart[i];
    __syncthreads();
    for (int i = tid; i < n; i += 256) {
        const orbg_keypoint kp = kps[i];
        const int bk = bucket(kp);
        if (bk >= 0)
            fk[atomicAdd(&cursor[bk], 1)] =
                TKey{kp.x, kp.y, (uint32_t)i | (uint32_t)kp.octave << 24, urf ? urf[i] : 0.f};
    }
    __syncthreads();

    bool fwd = false, bwd = false;
    if (MODE == TRK_LASTFRAME) track_direction(A.cams[f], &fwd, &bwd);
    const uint8_t *fdesc = A.desc + (size_t)f * A.fc * 32;
    const int grp = lane >> 4, sub = lane & 15;
    for (int qq = 0; qq < TRK_QPW; qq += 4) {
        const int i = qbase + wv * TRK_QPW + qq + grp;
        bool act = i < nq;
        TrackQuery Q;
        Q.valid = false;
        if (act) {
            Q = track_query<MODE>(A, f, i, fwd, bwd, b);
            if (!Q.valid) {
                if (sub == 0) A.topn[(size_t)f * A.qc + i] = -1;
                act = false;
            }
        }
        if (!__any(act)) continue;
        unsigned long long loc[ORBG_MATCH_TOPK];
#pragma unroll
        for (int k = 0; k < ORBG_MATCH_TOPK; k++) loc[k] = ~0ull;
        int cnt = 0;
        if (act) {
            const Window w = make_window(MODE == TRK_LOOP ? kf_window_prm(g) : g, Q.x, Q.y, Q.r);
            uint32_t qd[8];
            {
                const uint4 *p = (const uint4 *)(A.qdesc + ((size_t)f * A.qc + i) * 32);
                const uint4 a = p[0], c = p[1];
                qd[0] = a.x; qd[1] = a.y; qd[2] = a.z; qd[3] = a.w;
                qd[4] = c.x; qd[5] = c.y; qd[6] = c.z; qd[7] = c.w;
            }
            // levels GetFeaturesInArea can return (bCheckLevels, :475-482)
            const bool chk = Q.minL > 0 || Q.maxL >= 0;
            const int lv0 = chk ? max(Q.minL, 0) : 0;
            const int lv1 = (chk && Q.maxL >= 0) ? min(Q.maxL, ORBG_MAX_LEVELS - 1) : ORBG_MAX_LEVELS - 1;
            for (int lv = lv0; !w.empty && lv <= lv1; lv++) {
                const int j0 = colstart[lv * ORBG_GRID_COLS + w.cx0];
                const int j1 = colstart[lv * ORBG_GRID_COLS + w.cx1 + 1];
                for (int j = j0 + sub; j < j1; j += 16) {
                    const TKey k = fk[j];
                    const int ord = cand_order(g, w, k.x, k.y);
                    if (ord < 0) continue;
                    if (!track_static_ok(Q, (int)(k.idx_oct >> 24), k.ur)) continue;
                    const int idx = (int)(k.idx_oct & 0xFFFFFF);
                    const int d = hamming8(qd, (const uint32_t *)(fdesc + (size_t)idx * 32));
                    if (d >= 256) continue;
                    unsigned long long key = ((unsigned long long)d << 32) |
                                             ((unsigned long long)ord << 20) | (unsigned)idx;
                    cnt++;
#pragma unroll
                    for (int k2 = 0; k2 < ORBG_MATCH_TOPK; k2++) {
                        const unsigned long long lo = key < loc[k2] ? key : loc[k2];
                        const unsigned long long hi = key < loc[k2] ? loc[k2] : key;
                        loc[k2] = lo;
                        key = hi;
                    }
                }
            }
        }
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 16);
        int head = 0;
        unsigned long long *out = A.topk + ((size_t)f * A.qc + i) * ORBG_MATCH_TOPK;
        for (int k = 0; k < ORBG_MATCH_TOPK; k++) {
            unsigned long long mine = ~0ull;
#pragma unroll
            for (int hh = 0; hh < ORBG_MATCH_TOPK; hh++)
                if (hh == head) mine = loc[hh];
            unsigned long long mn = mine;
#pragma unroll
            for (int o = 8; o > 0; o >>= 1) {
                const unsigned long long u = __shfl_xor(mn, o, 16);
                mn = u < mn ? u : mn;
            }
            if (mn != ~0ull && mine == mn) head++;
            if (act && sub == 0) out[k] = mn;
        }
        if (act && sub == 0) A.topn[(size_t)f * A.qc + i] = cnt;
    }
}

// exact rescan of one query against the current taken state: best and second keys over
// all keypoints of the frame, wave-parallel (the rare query whose K-list ran out)
template <int MODE>
__device__ __forceinline__ void track_rescan(const TrackArgs &A, int f, int i, const TrackQuery &Q,
                             const uint8_t *taken, unsigned long long *k1o,
                             unsigned long long *k2o)
{
    const int lane = threadIdx.x & 63, n = A.counts[f];
    const orbg_bounds b = A.bounds[f];
    const GridPrm g = grid_prm(b);
    const Window w = make_window(MODE == TRK_LOOP ? kf_window_prm(g) : g, Q.x, Q.y, Q.r);
    unsigned long long m1 = ~0ull, m2 = ~0ull;
    if (!w.empty) {
        uint32_t qd[8];
        const uint32_t *qp = (const uint32_t *)(A.qdesc + ((size_t)f * A.qc + i) * 32);
#pragma unroll
        for (int k = 0; k < 8; k++) qd[k] = qp[k];
        const orbg_keypoint *kps = A.kps + (size_t)f * A.fc;
        const float *urf = A.uright ? A.uright + (size_t)f * A.fc : nullptr;
        const uint8_t *fdesc = A.desc + (size_t)f * A.fc * 32;
        for (int j = lane; j < n; j += 64) {
            if (taken[j]) continue;
            const orbg_keypoint kp = kps[j];
            const int ord = cand_order(g, w, kp.x, kp.y);
            if (ord < 0) continue;
            if (!track_static_ok(Q, kp.octave, urf ? urf[j] : 0.f)) continue;
            const int d = hamming8(qd, (const uint32_t *)(fdesc + (size_t)j * 32));
            if (d >= 256) continue;
            const unsigned long long key =
                ((unsigned long long)d << 32) | ((unsigned long long)ord << 20) | (unsigned)j;
            if (key < m1) {
                m2 = m1;
                m1 = key;
            } else if (key < m2) {
                m2 = key;
            }
        }
    }
    const unsigned long long a = wave_min_u64(m1);
    const unsigned long long rest = (m1 == a) ? m2 : m1;
    *k1o = a;
    *k2o = wave_min_u64(rest);
}

#define TRK_CHUNK 64
#define TRK_RT 128  // resolver threads: wave 0 resolves, wave 1 prefetches the next chunk

// Resolver LDS (all of the sequential walk's reads are LDS reads):
//   lists[2][64 * K] u64, cnts[2][64], qinfo[2][64] (angle bits | flags), misc[64],
//   match[fc] i32, push[qc] i32 (index << 8 | bin), kang[fc] f32 (keypoint angles),
//   taken[fc] u8, koct[fc] i8, owner[fc] i32 (lowest taking lane of a speculative round)
__host__ __device__ constexpr size_t track_resolve_lds(int fc, int qc)
{
    return (size_t)2 * TRK_CHUNK * ORBG_MATCH_TOPK * 8 + 2 * TRK_CHUNK * 4 +
           2 * TRK_CHUNK * 8 + 64 * 4 + (size_t)fc * 4 + (size_t)qc * 4 + (size_t)fc * 4 +
           (size_t)fc + (size_t)fc + 4 + (size_t)fc * 4;
}

// one workgroup (two waves) per frame
template <int MODE>
__global__ __launch_bounds__(TRK_RT) void k_track_resolve(TrackArgs A)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t trs[];
    const int f = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int n = A.counts[f], nq = A.qcounts[f];
    unsigned long long *lists = (unsigned long long *)trs;          // [2][64 K]
    int2 *qinfo = (int2 *)(lists + 2 * TRK_CHUNK * ORBG_MATCH_TOPK);  // [2][64]
    int32_t *cnts = (int32_t *)(qinfo + 2 * TRK_CHUNK);             // [2][64]
    int32_t *misc = cnts + 2 * TRK_CHUNK;  // [0] npush, [1] nmatches, [2..31] histogram
    int32_t *match = misc + 64;
    int32_t *push = match + A.fc;
    float *kang = (float *)(push + A.qc);
    uint8_t *taken = (uint8_t *)(kang + A.fc);
    int8_t *koct = (int8_t *)(taken + A.fc);
    // offset arithmetic on the LDS base (an integer round trip of the pointer would lose the
    // address space and make every owner[] access a flat one)
    int32_t *owner = (int32_t *)(trs + (((int)((uint8_t *)(koct + A.fc) - trs) + 3) & ~3));
    const uint8_t *t0 = A.taken0 ? A.taken0 + (size_t)f * A.fc : nullptr;
    const orbg_keypoint *kps = A.kps + (size_t)f * A.fc;
    for (int i = tid; i < n; i += TRK_RT) {
        const orbg_keypoint kp = kps[i];
        taken[i] = t0 ? t0[i] : 0;
        match[i] = -1;
        kang[i] = kp.angle;
        koct[i] = (int8_t)kp.octave;
        owner[i] = 64;
    }
    if (tid < 64) misc[tid] = 0;
    bool fwd = false, bwd = false;
    if (MODE == TRK_LASTFRAME) track_direction(A.cams[f], &fwd, &bwd);
    const orbg_bounds b = A.bounds[f];
    const float factor = 1.0f / HISTO_LENGTH;

    // wave 1: chunk c's counts, K-lists and query info into buffer c & 1
    auto prefetch = [&](int c) {
        const int c0 = c * TRK_CHUNK;
        if (c0 >= nq) return;
        const int cn = min(TRK_CHUNK, nq - c0);
        const int bf = c & 1;
        const int t = lane < cn ? A.topn[(size_t)f * A.qc + c0 + lane] : -1;
        cnts[bf * TRK_CHUNK + lane] = t;
        if (__ballot(t > 0) == 0ull) return;
        int2 qi = make_int2(0, 0);
        if (lane < cn) {
            if (MODE == TRK_LASTFRAME) {
                const orbg_lastframe_point P =
                    ((const orbg_lastframe_point *)A.q)[(size_t)f * A.qc + c0 + lane];
                qi = make_int2(__float_as_int(P.angle), P.flags);
            } else if (MODE == TRK_RELOC) {
                const orbg_reloc_point P =
                    ((const orbg_reloc_point *)A.q)[(size_t)f * A.qc + c0 + lane];
                qi = make_int2(__float_as_int(P.angle), P.flags | ORBG_MP_HAS_OBS);
            } else if (MODE == TRK_LOOP) {
                qi.y = ((const orbg_map_point *)A.q)[(size_t)f * A.qc + c0 + lane].flags |
                       ORBG_MP_HAS_OBS;
            } else {
                qi.y = ((const orbg_map_projection *)A.q)[(size_t)f * A.qc + c0 + lane].flags;
            }
        }
        qinfo[bf * TRK_CHUNK + lane] = qi;
        unsigned long long e[ORBG_MATCH_TOPK];
#pragma unroll
        for (int u = 0; u < ORBG_MATCH_TOPK; u++) {
            const int k = u * 64 + lane;
            e[u] = k < cn * ORBG_MATCH_TOPK
                       ? A.topk[((size_t)f * A.qc + c0) * ORBG_MATCH_TOPK + k]
                       : ~0ull;
        }
#pragma unroll
        for (int u = 0; u < ORBG_MATCH_TOPK; u++)
            lists[bf * TRK_CHUNK * ORBG_MATCH_TOPK + u * 64 + lane] = e[u];
    };

    // wave 0's running counts (the rotation histogram is built from the push list)
    int npush = 0, nmatch = 0;

    if (wv == 1) prefetch(0);
    __syncthreads();
    const int nchunks = (nq + TRK_CHUNK - 1) / TRK_CHUNK;
    for (int c = 0; c < nchunks; c++) {
        if (wv == 1) {
            prefetch(c + 1);
        } else {
            const int c0 = c * TRK_CHUNK, cn = min(TRK_CHUNK, nq - c0), bf = c & 1;
            const int *cnt = cnts + bf * TRK_CHUNK;
            const unsigned long long *lst0 = lists + bf * TRK_CHUNK * ORBG_MATCH_TOPK;
            const int2 *qin = qinfo + bf * TRK_CHUNK;
            // Speculative parallel walk, one query per lane.  Every pending lane picks
            // best / second from its K-list against the current taken state; a lane's
            // picks are exact unless an earlier pending lane takes (has_obs) a keypoint at
            // or before its last consulted list position.  owner[idx] = lowest taking lane
            // finds the first such lane l*; lanes below l* (and below the first lane whose
            // K-list ran out) commit in lane order, the rest go again.  Same result as the
            // in-order loop, typically in one or two rounds per chunk.
            const int need = MODE == TRK_LOCAL ? 2 : 1;
            // the loop's acceptance (:1623 TH_HIGH, :131 TH_HIGH, :1760 ORBdist, :458 TH_LOW)
            const int thr = MODE == TRK_RELOC ? A.orb_dist : MODE == TRK_LOOP ? TH_LOW : TH_HIGH;
            const int qidx = c0 + lane;
            const int total = lane < cn ? cnt[lane] : 0;
            const int2 qv = qin[lane];
            unsigned long long e[ORBG_MATCH_TOPK];
#pragma unroll
            for (int k = 0; k < ORBG_MATCH_TOPK; k++) e[k] = lst0[lane * ORBG_MATCH_TOPK + k];
            const int kk = min(total, ORBG_MATCH_TOPK);
            unsigned long long pending = __ballot(total > 0);
            while (pending) {
                const bool pend = (pending >> lane) & 1ull;
                unsigned long long k1 = ~0ull, k2 = ~0ull;
                int found = 0, lastpos = kk - 1;
                // every entry's taken flag read at once (indices clamped, entries past the list
                // ignored), then the in-order pick on registers
                int tk[ORBG_MATCH_TOPK];
#pragma unroll
                for (int k = 0; k < ORBG_MATCH_TOPK; k++)
                    tk[k] = taken[min((int)(e[k] & 0xFFFFF), A.fc - 1)];
#pragma unroll
                for (int k = 0; k < ORBG_MATCH_TOPK; k++) {
                    if (!pend || k >= kk || found >= need) continue;
                    if (tk[k]) continue;
                    if (found == 0) k1 = e[k]; else k2 = e[k];
                    if (++found == need) lastpos = k;
                }
                const bool resc = pend && found < need && total > ORBG_MATCH_TOPK;
                // the loop body's decision (ORBmatcher.cc:1623-1625 / 129-139)
                bool app = false;
                int bestIdx = 0, bin = 0;
                if (pend && !resc && k1 != ~0ull && (int)(k1 >> 32) <= thr) {
                    bestIdx = (int)(k1 & 0xFFFFF);
                    app = true;
                    if (MODE == TRK_LOCAL) {
                        const int bestDist2 = k2 == ~0ull ? 256 : (int)(k2 >> 32);
                        const int o2 = k2 == ~0ull ? -1 : koct[(int)(k2 & 0xFFFFF)];
                        if (koct[bestIdx] == o2 && (int)(k1 >> 32) > A.nnratio * bestDist2)
                            app = false;
                    } else if (TRK_ROT(MODE) && A.check_ori) {
                        float rot = __int_as_float(qv.x) - kang[bestIdx];
                        if (rot < 0.0) rot += 360.0f;
                        bin = (int)roundf(rot * factor);
                        if (bin == HISTO_LENGTH) bin = 0;
                    }
                }
                const bool takes = app && (qv.y & ORBG_MP_HAS_OBS);
                if (takes) atomicMin(&owner[bestIdx], lane);
                wave_sync_lds();
                bool conf = false;
                int ow[ORBG_MATCH_TOPK];
#pragma unroll
                for (int k = 0; k < ORBG_MATCH_TOPK; k++)
                    ow[k] = owner[min((int)(e[k] & 0xFFFFF), A.fc - 1)];
#pragma unroll
                for (int k = 0; k < ORBG_MATCH_TOPK; k++)
                    if (pend && k < kk && k <= lastpos && ow[k] < lane) conf = true;
                const unsigned long long cm = __ballot(conf), rm = __ballot(resc);
                const int lc = cm ? __builtin_ctzll(cm) : 64, lr = rm ? __builtin_ctzll(rm) : 64;
                const int lstar = min(lc, lr);
                const unsigned long long below = lstar >= 64 ? ~0ull : ((1ull << lstar) - 1ull);
                const bool commit = pend && lane < lstar;
                if (takes) owner[bestIdx] = 64;
                if (commit && app) {
                    atomicMax(&match[bestIdx], qidx);  // later query overwrites: larger index
                    if (takes) taken[bestIdx] = 1;
                }
                const unsigned long long am = __ballot(commit && app);
                if (TRK_ROT(MODE) && A.check_ori && commit && app) {
                    const int pos = __builtin_amdgcn_mbcnt_hi(
                        (uint32_t)(am >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)am, 0));
                    push[npush + pos] = bestIdx << 8 | bin;
                }
                npush += (TRK_ROT(MODE) && A.check_ori) ? __popcll(am) : 0;
                nmatch += __popcll(am);
                pending &= ~below;
                wave_sync_lds();
                if (lr < 64 && lr == lstar) {
                    // K-list exhausted: exact rescan of query lr against the committed state
                    const TrackQuery Q = track_query<MODE>(A, f, c0 + lr, fwd, bwd, b);
                    unsigned long long r1, r2;
                    track_rescan<MODE>(A, f, c0 + lr, Q, taken, &r1, &r2);
                    const int qy = __shfl(qv.y, lr, 64), qx = __shfl(qv.x, lr, 64);
                    if (lane == 0 && r1 != ~0ull && (int)(r1 >> 32) <= thr) {
                        const int bi = (int)(r1 & 0xFFFFF);
                        bool ok = true;
                        int bn = 0;
                        if (MODE == TRK_LOCAL) {
                            const int bestDist2 = r2 == ~0ull ? 256 : (int)(r2 >> 32);
                            const int o2 = r2 == ~0ull ? -1 : koct[(int)(r2 & 0xFFFFF)];
                            if (koct[bi] == o2 && (int)(r1 >> 32) > A.nnratio * bestDist2) ok = false;
                        } else if (TRK_ROT(MODE) && A.check_ori) {
                            float rot = __int_as_float(qx) - kang[bi];
                            if (rot < 0.0) rot += 360.0f;
                            bn = (int)roundf(rot * factor);
                            if (bn == HISTO_LENGTH) bn = 0;
                        }
                        if (ok) {
                            match[bi] = max(match[bi], c0 + lr);
                            if (qy & ORBG_MP_HAS_OBS) taken[bi] = 1;
                            if (TRK_ROT(MODE) && A.check_ori) push[npush] = bi << 8 | bn;
                            misc[63] = 1;
                        } else {
                            misc[63] = 0;
                        }
                    } else if (lane == 0) {
                        misc[63] = 0;
                    }
                    wave_sync_lds();
                    const int ap = misc[63];
                    npush += (TRK_ROT(MODE) && A.check_ori) ? ap : 0;
                    nmatch += ap;
                    pending &= ~(1ull << lr);
                    wave_sync_lds();
                }
            }
        }
        __syncthreads();
    }
    if (tid == 0) {
        misc[0] = npush;
        misc[1] = nmatch;
    }
    __syncthreads();
    int nm = misc[1];
    if (TRK_ROT(MODE) && A.check_ori) {
        // rotation histogram of the pushes, ComputeThreeMaxima (:1800-1841), then every
        // push in a dropped bin NULLs its slot and decrements nmatches (:1651-1663)
        const int np = misc[0];
        for (int k = tid; k < np; k += TRK_RT) atomicAdd(&misc[2 + (push[k] & 0xFF)], 1);
        __syncthreads();
        int ind1 = -1, ind2 = -1, ind3 = -1;
        {
            int max1 = 0, max2 = 0, max3 = 0;
            for (int i = 0; i < HISTO_LENGTH; i++) {
                const int s = misc[2 + i];
                if (s > max1) {
                    max3 = max2; max2 = max1; max1 = s;
                    ind3 = ind2; ind2 = ind1; ind1 = i;
                } else if (s > max2) {
                    max3 = max2; max2 = s;
                    ind3 = ind2; ind2 = i;
                } else if (s > max3) {
                    max3 = s;
                    ind3 = i;
                }
            }
            if (max2 < 0.1f * (float)max1) {
                ind2 = -1;
                ind3 = -1;
            } else if (max3 < 0.1f * (float)max1) {
                ind3 = -1;
            }
        }
        int removed = 0;
        for (int k = tid; k < np; k += TRK_RT) {
            const int e = push[k], bn = e & 0xFF;
            if (bn != ind1 && bn != ind2 && bn != ind3) {
                match[e >> 8] = -2;  // NULLed by the rotation filter (same value from every writer)
                removed++;
            }
        }
        removed = wave_isum(removed);
        __shared__ int rem[2];
        if (lane == 0) rem[wv] = removed;
        __syncthreads();
        nm -= rem[0] + rem[1];
    }
    int32_t *mo = A.match + (size_t)f * A.fc;
    for (int i = tid; i < n; i += TRK_RT) mo[i] = match[i];
    if (tid == 0) A.nmatches[f] = nm;
}

#define PL(prof, st, name, launch)                                    \
    do {                                                              \
        hipEvent_t ev_ = nullptr;                                     \
        prof_begin(prof, st, name, &ev_);                             \
        launch;                                                       \
        prof_end(prof, st, name, ev_);                                \
    } while (0)

size_t track_cands_lds(int fc) { return (size_t)std::max(fc, 1) * sizeof(TKey); }
size_t track_resolve_lds_bytes(int fc, int qc) { return track_resolve_lds(fc, qc); }

template <int MODE>
static void launch_mode(hipStream_t st, const TrackArgs &A, int nframes, int nbx, size_t l1,
                        size_t l2, void *prof)
{
    hipFuncSetAttribute((const void *)k_track_cands<MODE>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)l1);
    hipFuncSetAttribute((const void *)k_track_resolve<MODE>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)l2);
    PL(prof, st, "track_cands",
       hipLaunchKernelGGL(k_track_cands<MODE>, dim3(nbx * nframes), dim3(256), l1, st, A));
    PL(prof, st, "track_resolve",
       hipLaunchKernelGGL(k_track_resolve<MODE>, dim3(nframes), dim3(TRK_RT), l2, st, A));
}

// mode: TRK_LASTFRAME / TRK_LOCAL / TRK_RELOC / TRK_LOOP.  A's pointers are device pointers;
// nframes frames.
int launch_track(hipStream_t st, int mode, const TrackArgs &A, int nframes, void *prof)
{
    if (A.fc > (1 << 20) || nframes <= 0) return ORBG_EINVAL;
    const size_t l1 = track_cands_lds(A.fc), l2 = track_resolve_lds(A.fc, A.qc);
    if (l1 > 160 * 1024 || l2 > 160 * 1024) return ORBG_ENOTSUP;
    const int nbx = (A.qc + 4 * TRK_QPW - 1) / (4 * TRK_QPW);
    switch (mode) {
    case TRK_LASTFRAME: launch_mode<TRK_LASTFRAME>(st, A, nframes, nbx, l1, l2, prof); break;
    case TRK_LOCAL: launch_mode<TRK_LOCAL>(st, A, nframes, nbx, l1, l2, prof); break;
    case TRK_RELOC: launch_mode<TRK_RELOC>(st, A, nframes, nbx, l1, l2, prof); break;
    case TRK_LOOP: launch_mode<TRK_LOOP>(st, A, nframes, nbx, l1, l2, prof); break;
    default: return ORBG_EINVAL;
    }
    return hipGetLastError() == hipSuccess ? ORBG_OK : ORBG_EIO;
}

}  // namespace orbg
