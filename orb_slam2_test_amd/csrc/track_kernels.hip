// track_kernels.hip -- the per-frame tracking matchers for gfx950.
//
//   ORBmatcher::SearchByProjection(CurrentFrame, LastFrame, th, bMono)
//       (ORBmatcher.cc:1503-1667; Tracking::TrackWithMotionModel)
//   ORBmatcher::SearchByProjection(F, vpMapPoints, th)
//       (ORBmatcher.cc:59-146, RadiusByViewingCos :148-154; Tracking::SearchLocalPoints)
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
//   k_track_resolve  one wave per frame walks the queries in index order over the K-lists
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
#include "match_device.h"
#include "track_args.h"

#pragma clang fp contract(off)

namespace orbg {

void prof_begin(void *prof, hipStream_t s, const char *n, hipEvent_t *a);
void prof_end(void *prof, hipStream_t s, const char *n, hipEvent_t a);

#define TH_HIGH 100
#define HISTO_LENGTH 30
#define TRK_QPW 16  // queries per wave in k_track_cands (4 x 4 in 16-lane groups)

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
    __shared__ int colstart[ORBG_GRID_COLS + 1];
    __shared__ int cursor[ORBG_GRID_COLS];
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
    // counting sort by PosInGrid column (Frame.cc:510-520); keypoints outside the grid are
    // in no cell and never candidates
    if (tid <= ORBG_GRID_COLS) colstart[tid] = 0;
    __syncthreads();
    for (int i = tid; i < n; i += 256) {
        const orbg_keypoint kp = kps[i];
        const int px = (int)roundf((kp.x - g.min_x) * g.inv_w);
        const int py = (int)roundf((kp.y - g.min_y) * g.inv_h);
        if (px >= 0 && px < ORBG_GRID_COLS && py >= 0 && py < ORBG_GRID_ROWS)
            atomicAdd(&colstart[px + 1], 1);
    }
    __syncthreads();
    if (wv == 0) {
        const int c = colstart[lane + 1];
        colstart[lane + 1] = wave_incl_scan(c);
    }
    __syncthreads();
    if (tid < ORBG_GRID_COLS) cursor[tid] = colstart[tid];
    __syncthreads();
    for (int i = tid; i < n; i += 256) {
        const orbg_keypoint kp = kps[i];
        const int px = (int)roundf((kp.x - g.min_x) * g.inv_w);
        const int py = (int)roundf((kp.y - g.min_y) * g.inv_h);
        if (px >= 0 && px < ORBG_GRID_COLS && py >= 0 && py < ORBG_GRID_ROWS)
            fk[atomicAdd(&cursor[px], 1)] =
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
            const Window w = make_window(g, Q.x, Q.y, Q.r);
            uint32_t qd[8];
            {
                const uint4 *p = (const uint4 *)(A.qdesc + ((size_t)f * A.qc + i) * 32);
                const uint4 a = p[0], c = p[1];
                qd[0] = a.x; qd[1] = a.y; qd[2] = a.z; qd[3] = a.w;
                qd[4] = c.x; qd[5] = c.y; qd[6] = c.z; qd[7] = c.w;
            }
            if (!w.empty) {
                const int j0 = colstart[w.cx0], j1 = colstart[w.cx1 + 1];
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
__device__ void track_rescan(const TrackArgs &A, int f, int i, const TrackQuery &Q,
                             const uint8_t *taken, unsigned long long *k1o,
                             unsigned long long *k2o)
{
    const int lane = threadIdx.x & 63, n = A.counts[f];
    const orbg_bounds b = A.bounds[f];
    const GridPrm g = grid_prm(b);
    const Window w = make_window(g, Q.x, Q.y, Q.r);
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

// LDS: chunk lists (u64), chunk counts, misc, match[fc] i32, pushes[qc] i32
// (index << 8 | bin), taken[fc] u8
__host__ __device__ constexpr size_t track_resolve_lds(int fc, int qc)
{
    return (size_t)TRK_CHUNK * ORBG_MATCH_TOPK * 8 + TRK_CHUNK * 4 + 64 * 4 + (size_t)fc * 4 +
           (size_t)qc * 4 + (size_t)fc;
}

// one wave per frame
template <int MODE>
__global__ __launch_bounds__(64) void k_track_resolve(TrackArgs A)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t trs[];
    const int f = blockIdx.x, lane = threadIdx.x;
    const int n = A.counts[f], nq = A.qcounts[f];
    unsigned long long *lists = (unsigned long long *)trs;
    int32_t *cnts = (int32_t *)(lists + TRK_CHUNK * ORBG_MATCH_TOPK);
    int32_t *misc = cnts + TRK_CHUNK;  // [0] npush, [1] nmatches, [2..31] histogram sizes
    int32_t *match = misc + 64;
    int32_t *push = match + A.fc;
    uint8_t *taken = (uint8_t *)(push + A.qc);
    const uint8_t *t0 = A.taken0 ? A.taken0 + (size_t)f * A.fc : nullptr;
    for (int i = lane; i < n; i += 64) {
        taken[i] = t0 ? t0[i] : 0;
        match[i] = -1;
    }
    misc[lane] = 0;
    wave_sync_lds();
    bool fwd = false, bwd = false;
    if (MODE == TRK_LASTFRAME) track_direction(A.cams[f], &fwd, &bwd);
    const orbg_keypoint *kps = A.kps + (size_t)f * A.fc;
    const orbg_bounds b = A.bounds[f];
    const float factor = 1.0f / HISTO_LENGTH;

    // lane 0: the loop body's state update once best / second are known
    auto apply = [&](int i, unsigned long long k1, unsigned long long k2) {
        if (k1 == ~0ull) return;
        const int bestDist = (int)(k1 >> 32), bestIdx = (int)(k1 & 0xFFFFF);
        if (bestDist > TH_HIGH) return;
        bool has_obs;
        if (MODE == TRK_LOCAL) {
            // ORBmatcher.cc:131-139: ratio only between matches of the same level
            const int bestLevel = kps[bestIdx].octave;
            const int bestDist2 = k2 == ~0ull ? 256 : (int)(k2 >> 32);
            const int bestLevel2 = k2 == ~0ull ? -1 : kps[(int)(k2 & 0xFFFFF)].octave;
            if (bestLevel == bestLevel2 && bestDist > A.nnratio * bestDist2) return;
            has_obs = (((const orbg_map_projection *)A.q)[(size_t)f * A.qc + i].flags &
                       ORBG_MP_HAS_OBS) != 0;
        } else {
            const orbg_lastframe_point P =
                ((const orbg_lastframe_point *)A.q)[(size_t)f * A.qc + i];
            has_obs = (P.flags & ORBG_MP_HAS_OBS) != 0;
            if (A.check_ori) {
                // ORBmatcher.cc:1633-1642
                float rot = P.angle - kps[bestIdx].angle;
                if (rot < 0.0) rot += 360.0f;
                int bin = (int)roundf(rot * factor);
                if (bin == HISTO_LENGTH) bin = 0;
                push[misc[0]++] = bestIdx << 8 | bin;
                misc[2 + bin]++;
            }
        }
        match[bestIdx] = i;
        taken[bestIdx] = has_obs ? 1 : 0;
        misc[1]++;
    };

    for (int c0 = 0; c0 < nq; c0 += TRK_CHUNK) {
        const int cn = min(TRK_CHUNK, nq - c0);
        const int t = lane < cn ? A.topn[(size_t)f * A.qc + c0 + lane] : -1;
        cnts[lane] = t;
        if (__ballot(t > 0) == 0ull) continue;
#pragma unroll
        for (int u = 0; u < ORBG_MATCH_TOPK; u++) {
            const int e = u * 64 + lane;
            lists[e] = e < cn * ORBG_MATCH_TOPK
                           ? A.topk[((size_t)f * A.qc + c0) * ORBG_MATCH_TOPK + e]
                           : ~0ull;
        }
        wave_sync_lds();
        int qi = 0;
        while (qi < cn) {
            int q = qi, fb = 0;
            if (lane == 0) {
                for (; q < cn; q++) {
                    const int total = cnts[q];
                    if (total <= 0) continue;
                    const int kk = min(total, ORBG_MATCH_TOPK);
                    const unsigned long long *lst = &lists[q * ORBG_MATCH_TOPK];
                    unsigned long long k1 = ~0ull, k2 = ~0ull;
                    int found = 0;
                    for (int k = 0; k < kk && found < 2; k++) {
                        const unsigned long long e = lst[k];
                        if (taken[(int)(e & 0xFFFFF)]) continue;
                        if (found == 0) k1 = e; else k2 = e;
                        found++;
                    }
                    // the last-frame search needs only the best
                    const int need = MODE == TRK_LOCAL ? 2 : 1;
                    if (found < need && total > ORBG_MATCH_TOPK) {
                        fb = 1;
                        break;
                    }
                    apply(c0 + q, k1, k2);
                }
            }
            q = __shfl(q, 0, 64);
            fb = __shfl(fb, 0, 64);
            wave_sync_lds();
            qi = q;
            if (fb) {
                const int i = c0 + qi;
                const TrackQuery Q = track_query<MODE>(A, f, i, fwd, bwd, b);
                unsigned long long k1, k2;
                track_rescan<MODE>(A, f, i, Q, taken, &k1, &k2);
                if (lane == 0) apply(i, k1, k2);
                wave_sync_lds();
                qi++;
            }
        }
    }
    int nm = misc[1];
    if (MODE == TRK_LASTFRAME && A.check_ori) {
        // ComputeThreeMaxima (:1800-1841), then every push in a dropped bin NULLs its slot
        // and decrements nmatches (:1651-1663)
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
        const int np = misc[0];
        int removed = 0;
        for (int k = lane; k < np; k += 64) {
            const int e = push[k], bn = e & 0xFF;
            if (bn != ind1 && bn != ind2 && bn != ind3) {
                match[e >> 8] = -1;  // same value from every writer: no ordering needed
                removed++;
            }
        }
        nm -= wave_isum(removed);
        wave_sync_lds();
    }
    int32_t *mo = A.match + (size_t)f * A.fc;
    for (int i = lane; i < n; i += 64) mo[i] = match[i];
    if (lane == 0) A.nmatches[f] = nm;
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

// mode: 0 last frame, 1 local map.  A's pointers are device pointers; nframes frames.
int launch_track(hipStream_t st, int mode, const TrackArgs &A, int nframes, void *prof)
{
    if (A.fc > (1 << 20) || nframes <= 0) return ORBG_EINVAL;
    const size_t l1 = track_cands_lds(A.fc), l2 = track_resolve_lds(A.fc, A.qc);
    if (l1 > 160 * 1024 || l2 > 160 * 1024) return ORBG_ENOTSUP;
    const int nbx = (A.qc + 4 * TRK_QPW - 1) / (4 * TRK_QPW);
    if (mode == TRK_LASTFRAME) {
        hipFuncSetAttribute((const void *)k_track_cands<TRK_LASTFRAME>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)l1);
        hipFuncSetAttribute((const void *)k_track_resolve<TRK_LASTFRAME>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)l2);
        PL(prof, st, "track_cands",
           hipLaunchKernelGGL(k_track_cands<TRK_LASTFRAME>, dim3(nbx * nframes), dim3(256), l1,
                              st, A));
        PL(prof, st, "track_resolve",
           hipLaunchKernelGGL(k_track_resolve<TRK_LASTFRAME>, dim3(nframes), dim3(64), l2, st,
                              A));
    } else {
        hipFuncSetAttribute((const void *)k_track_cands<TRK_LOCAL>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)l1);
        hipFuncSetAttribute((const void *)k_track_resolve<TRK_LOCAL>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)l2);
        PL(prof, st, "track_cands",
           hipLaunchKernelGGL(k_track_cands<TRK_LOCAL>, dim3(nbx * nframes), dim3(256), l1, st,
                              A));
        PL(prof, st, "track_resolve",
           hipLaunchKernelGGL(k_track_resolve<TRK_LOCAL>, dim3(nframes), dim3(64), l2, st, A));
    }
    return hipGetLastError() == hipSuccess ? ORBG_OK : ORBG_EIO;
}

}  // namespace orbg
