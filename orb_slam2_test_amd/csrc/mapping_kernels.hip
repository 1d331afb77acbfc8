// mapping_kernels.hip -- LocalMapping's per-keyframe Hamming matchers for gfx950.
//
//   k_fuse        ORBmatcher::Fuse(pKF, vpMapPoints, th)'s per-MapPoint search (src/ORBmatcher.cc:
//                 968-1069; LocalMapping::SearchInNeighbors, LocalMapping.cc:622-690), one
//                 workgroup per (KeyFrame, MapPoint list) pair: the KeyFrame's grid
//                 (Frame::AssignFeaturesToGrid, PosInGrid) counting-sorted into LDS, then a thread
//                 per MapPoint: projection, IsInImage, the scale-invariance and viewing-angle
//                 gates, PredictScale, GetFeaturesInArea's cells, the level window and the
//                 chi-square reprojection gates, best distance by the 64-bit key (distance,
//                 grid cell, index): the first candidate of the least distance in the
//                 reference's enumeration (cell major, ascending index inside a cell), its
//                 strict <.  Returns bestIdx per point (-1 unless bestDist <= TH_LOW): the
//                 caller's sequential map update (Replace / AddObservation) applies it.
//   k_sim3_match  ORBmatcher::SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th)
//   k_sim3_resolve  (src/ORBmatcher.cc:1262-1470; LoopClosing::ComputeSim3): both projection
//                 directions on the same LDS grid machinery, then the mutual check.
//   k_tri_match   ORBmatcher::SearchForTriangulation(pKF1, pKF2, F12, vMatchedPairs,
//                 bOnlyStereo) (src/ORBmatcher.cc:779-957; LocalMapping::CreateNewMapPoints,
//                 LocalMapping.cc:305-378), one 256-thread workgroup per (KF1, KF2) pair.
//
// The reference walks both FeatureVectors in node order and, for every KF1 feature without a
// MapPoint, scans the shared node's KF2 features: a candidate passes when it has no MapPoint
// (vbMatched2 is never set, :810, so KF1 features do not compete), its distance is <= TH_LOW,
// it is away from the epipole (both monocular) and CheckDistEpipolarLine holds; it replaces
// the best on dist <= bestDist, so the result is the LAST passing candidate of the least
// distance.  Every KF1 feature is therefore independent:
//   join      KF1 node ids joined with KF2's by binary search into an LDS list (as k_bow_match);
//   node      a wave per common node: lane l holds KF2 candidate l (and l + 64) with its
//             descriptor, position, octave thresholds and flags in registers; each KF1 feature
//             of the node is broadcast through scalar registers, its epipolar line (a, b, c)
//             computed once (wave-uniform), every lane tests its candidate, and one wave-wide
//             max of (51 - dist) << 16 | position gives the least distance, last position;
//   rotation  ComputeThreeMaxima over an LDS histogram when checkOri (CreateNewMapPoints uses
//             ORBmatcher(0.6, false): off), then the matches outside the three bins dropped.
// Float pins as the oracle (oracle/mapping_oracle.c): C2 = R2w*Cw+t2w by cv::gemm's double
// work type, the epipolar test's float dsqr compared with 3.84 * sigma2 in double; no FMA.
#include <hip/hip_runtime.h>

#include "../../include/orbg.h"
#include "frame_device.h"
#include "orbg_device.h"
#include "orbg_internal.h"

#pragma clang fp contract(off)

namespace orbg {

#define TM_HISTO 30
#define TM_TH_LOW 50
#define TM_LIST 1024  // common nodes per pass held in LDS

struct TriTables {
    float scale[ORBG_MAX_LEVELS];   // pKF2->mvScaleFactors
    double epi_th[ORBG_MAX_LEVELS]; // 3.84 * mvLevelSigma2 (double, as the reference compares)
};

__device__ __forceinline__ unsigned wave_max_u32(unsigned v)
{
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0xb1, 0xf, 0xf, false));  // quad_perm 1,0,3,2
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x4e, 0xf, 0xf, false));  // quad_perm 2,3,0,1
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xf, 0xf, false)); // row_ror 4
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xf, 0xf, false)); // row_ror 8
    const unsigned r0 = (unsigned)__builtin_amdgcn_readlane((int)v, 0);
    const unsigned r1 = (unsigned)__builtin_amdgcn_readlane((int)v, 16);
    const unsigned r2 = (unsigned)__builtin_amdgcn_readlane((int)v, 32);
    const unsigned r3 = (unsigned)__builtin_amdgcn_readlane((int)v, 48);
    return max(max(r0, r1), max(r2, r3));
}

__device__ __forceinline__ int tm_rot_bin(float a1, float a2)
{
    const float factor = 1.0f / TM_HISTO;
    float rot = a1 - a2;
    if (rot < 0.0) rot += 360.0f;
    int bin = (int)roundf(rot * factor);
    if (bin == TM_HISTO) bin = 0;
    return bin;
}

// one KF2 candidate as a lane holds it
struct TriCand {
    uint32_t d[8];
    float x, y;
    double th;      // 3.84 * sigma2[octave]
    int idx;        // -1: no candidate (past the node) or unusable (MapPoint / not stereo)
    bool stereo;
    bool epi_far;   // away from the epipole (the monocular pair test)
};

__device__ __forceinline__ void tri_load(TriCand &c, const orbg_keyframes &K, int kf2, int cap,
                                         int f2, int pos, int nF, float ex, float ey,
                                         const TriTables &T, int only_stereo)
{
    c.idx = -1;
#pragma unroll
    for (int w = 0; w < 8; w++) c.d[w] = 0u;
    c.x = c.y = 0.f;
    c.th = 0.0;
    c.stereo = false;
    c.epi_far = false;
    if (pos >= nF) return;
    const int idx = K.fv_feats[(size_t)kf2 * cap + f2 + pos];
    const size_t g = (size_t)kf2 * cap + idx;
    if (K.has_mp && K.has_mp[g]) return;
    const bool st = K.uright ? K.uright[g] >= 0 : false;
    if (only_stereo && !st) return;
    const orbg_keypoint kp = K.kps[g];
    const uint4 *p = (const uint4 *)(K.desc + g * 32);
    const uint4 a = p[0], b = p[1];
    c.d[0] = a.x; c.d[1] = a.y; c.d[2] = a.z; c.d[3] = a.w;
    c.d[4] = b.x; c.d[5] = b.y; c.d[6] = b.z; c.d[7] = b.w;
    c.x = kp.x;
    c.y = kp.y;
    c.th = T.epi_th[kp.octave];
    const float distex = ex - kp.x, distey = ey - kp.y;
    c.epi_far = !(distex * distex + distey * distey < 100 * T.scale[kp.octave]);
    c.stereo = st;
    c.idx = idx;
}

// key of a passing candidate: (51 - dist) << 16 | position (wave max = least distance, last
// position); 0 = does not pass
__device__ __forceinline__ unsigned tri_key(const TriCand &c, const uint32_t q[8], bool stereo1,
                                            float a, float b, float cc, float den, int pos)
{
    if (c.idx < 0) return 0u;
    int dist = 0;
#pragma unroll
    for (int w = 0; w < 8; w++) dist += __popc(q[w] ^ c.d[w]);
    if (dist > TM_TH_LOW) return 0u;
    if (!stereo1 && !c.stereo && !c.epi_far) return 0u;
    // CheckDistEpipolarLine (ORBmatcher.cc:165-182)
    if (den == 0) return 0u;
    const float num = a * c.x + b * c.y + cc;
    const float dsqr = num * num / den;
    if (!((double)dsqr < c.th)) return 0u;
    return ((unsigned)(51 - dist) << 16) | (unsigned)pos;
}

__global__ __launch_bounds__(256) void k_tri_match(orbg_keyframes K, int cap,
                                                   const int32_t *__restrict__ kf1_index,
                                                   const int32_t *__restrict__ kf2_index,
                                                   const orbg_triangulation_pair *__restrict__ geo,
                                                   TriTables T, int only_stereo, int check_ori,
                                                   int32_t *__restrict__ match,
                                                   int32_t *__restrict__ nmatch)
{
    __shared__ int2 common[TM_LIST];
    __shared__ int ncommon, nm, removed, hist[TM_HISTO], ind[3];
    const int p = blockIdx.x;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int k1 = kf1_index[p], k2 = kf2_index[p];
    const int n1 = K.counts[k1];
    const int nn1 = K.nfv[k1], nn2 = K.nfv[k2];
    const int32_t *n1ids = K.fv_nodes + (size_t)k1 * cap, *o1 = K.fv_off + (size_t)k1 * (cap + 1),
                  *fe1 = K.fv_feats + (size_t)k1 * cap;
    const int32_t *n2ids = K.fv_nodes + (size_t)k2 * cap, *o2 = K.fv_off + (size_t)k2 * (cap + 1);
    const orbg_keypoint *kp1 = K.kps + (size_t)k1 * cap, *kp2 = K.kps + (size_t)k2 * cap;
    const uint8_t *desc1 = K.desc + (size_t)k1 * cap * 32;
    int32_t *out = match + (size_t)p * cap;
    // the epipole (ORBmatcher.cc:800-806): C2 = R2w*Cw+t2w, cv::gemm small-matrix pin
    const orbg_triangulation_pair &G = geo[p];
    float C2[3];
#pragma unroll
    for (int r = 0; r < 3; r++) {
        double t = 0.0;
#pragma unroll
        for (int k = 0; k < 3; k++) t += (double)G.Tcw2[4 * r + k] * (double)G.Cw1[k];
        t *= 1.0;
        t += (double)G.Tcw2[4 * r + 3];
        C2[r] = (float)t;
    }
    const float invz = 1.0f / C2[2];
    const float ex = G.fx2 * C2[0] * invz + G.cx2;
    const float ey = G.fy2 * C2[1] * invz + G.cy2;
    float F[9];
#pragma unroll
    for (int i = 0; i < 9; i++) F[i] = G.F12[i];

    if (threadIdx.x == 0) {
        nm = 0;
        removed = 0;
    }
    if (threadIdx.x < TM_HISTO) hist[threadIdx.x] = 0;
    for (int i = threadIdx.x; i < n1; i += blockDim.x) out[i] = -1;
    int wave_nm = 0;
    for (int j0 = 0; j0 < nn1; j0 += TM_LIST) {
        if (threadIdx.x == 0) ncommon = 0;
        __syncthreads();
        for (int j = j0 + (int)threadIdx.x; j < min(nn1, j0 + TM_LIST); j += blockDim.x) {
            const int id = n1ids[j];
            int lo = 0, hi = nn2;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (n2ids[mid] < id)
                    lo = mid + 1;
                else
                    hi = mid;
            }
            if (lo < nn2 && n2ids[lo] == id) common[atomicAdd(&ncommon, 1)] = make_int2(j, lo);
        }
        __syncthreads();
        const int nc = ncommon;
        for (int c = wv; c < nc; c += (int)(blockDim.x >> 6)) {
            const int2 jb = common[c];
            const int a0 = o1[jb.x], a1 = o1[jb.x + 1];
            const int f2 = o2[jb.y], nF = o2[jb.y + 1] - f2;
            TriCand c0, c1;
            tri_load(c0, K, k2, cap, f2, lane, nF, ex, ey, T, only_stereo);
            tri_load(c1, K, k2, cap, f2, lane + 64, nF, ex, ey, T, only_stereo);
            // the node's KF1 features, 64 at a time: lane l loads feature ib + l (index,
            // MapPoint / stereo flags, descriptor, position, angle) so the serial walk below
            // broadcasts them from registers instead of waiting on dependent global loads
            for (int ib = a0; ib < a1; ib += 64) {
                const int cn = min(64, a1 - ib);
                int my_idx = 0, my_ok = 0, my_st = 0;
                uint32_t my_q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
                float my_x = 0.f, my_y = 0.f, my_ang = 0.f;
                if (lane < cn) {
                    my_idx = fe1[ib + lane];
                    const size_t g1 = (size_t)k1 * cap + my_idx;
                    my_st = K.uright ? K.uright[g1] >= 0 : 0;
                    // pMP1 (ORBmatcher.cc:837-840) and the stereo-only filter
                    my_ok = !(K.has_mp && K.has_mp[g1]) && !(only_stereo && !my_st);
                    const uint4 *dp = (const uint4 *)(desc1 + (size_t)my_idx * 32);
                    const uint4 qa = dp[0], qb = dp[1];
                    my_q[0] = qa.x; my_q[1] = qa.y; my_q[2] = qa.z; my_q[3] = qa.w;
                    my_q[4] = qb.x; my_q[5] = qb.y; my_q[6] = qb.z; my_q[7] = qb.w;
                    const orbg_keypoint k = kp1[my_idx];
                    my_x = k.x;
                    my_y = k.y;
                    my_ang = k.angle;
                }
                const unsigned long long okm = __ballot(lane < cn && my_ok);
                for (int t = 0; t < cn; t++) {
                    if (!((okm >> t) & 1ull)) continue;  // wave-uniform skip
                    const int idx1 = __builtin_amdgcn_readlane(my_idx, t);
                    const bool st1 = __builtin_amdgcn_readlane(my_st, t) != 0;
                    uint32_t q[8];
#pragma unroll
                    for (int w = 0; w < 8; w++) q[w] = (uint32_t)__builtin_amdgcn_readlane((int)my_q[w], t);
                    const float kx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(my_x), t));
                    const float ky = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(my_y), t));
                    // epipolar line l = x1' F12 (ORBmatcher.cc:168-170), wave-uniform
                    const float a = kx * F[0] + ky * F[3] + F[6];
                    const float b = kx * F[1] + ky * F[4] + F[7];
                    const float cc = kx * F[2] + ky * F[5] + F[8];
                    const float den = a * a + b * b;
                    unsigned key = max(tri_key(c0, q, st1, a, b, cc, den, lane),
                                       tri_key(c1, q, st1, a, b, cc, den, lane + 64));
                    for (int ch = 2; ch * 64 < nF; ch++) {  // nodes past 128 candidates: re-read
                        TriCand cx;
                        tri_load(cx, K, k2, cap, f2, ch * 64 + lane, nF, ex, ey, T, only_stereo);
                        key = max(key, tri_key(cx, q, st1, a, b, cc, den, ch * 64 + lane));
                    }
                    const unsigned best = wave_max_u32(key);
                    const float ang = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(my_ang), t));
                    if (best) {
                        wave_nm++;
                        if (lane == 0) {
                            const int idx2 = K.fv_feats[(size_t)k2 * cap + f2 + (int)(best & 0xFFFFu)];
                            out[idx1] = idx2;
                            if (check_ori) atomicAdd(&hist[tm_rot_bin(ang, kp2[idx2].angle)], 1);
                        }
                    }
                }
            }
        }
        __syncthreads();
    }
    if (lane == 0 && wave_nm) atomicAdd(&nm, wave_nm);
    __syncthreads();
    if (check_ori) {
        if (threadIdx.x == 0) {
            // ComputeThreeMaxima (ORBmatcher.cc:1800-1841)
            int max1 = 0, max2 = 0, max3 = 0, i1 = -1, i2 = -1, i3 = -1;
            for (int i = 0; i < TM_HISTO; i++) {
                const int s = hist[i];
                if (s > max1) {
                    max3 = max2;
                    max2 = max1;
                    max1 = s;
                    i3 = i2;
                    i2 = i1;
                    i1 = i;
                } else if (s > max2) {
                    max3 = max2;
                    max2 = s;
                    i3 = i2;
                    i2 = i;
                } else if (s > max3) {
                    max3 = s;
                    i3 = i;
                }
            }
            if (max2 < 0.1f * (float)max1) {
                i2 = -1;
                i3 = -1;
            } else if (max3 < 0.1f * (float)max1) {
                i3 = -1;
            }
            ind[0] = i1;
            ind[1] = i2;
            ind[2] = i3;
        }
        __syncthreads();
        int rm = 0;
        for (int i = threadIdx.x; i < n1; i += blockDim.x) {
            const int m = out[i];
            if (m < 0) continue;
            const int bin = tm_rot_bin(kp1[i].angle, kp2[m].angle);
            if (bin != ind[0] && bin != ind[1] && bin != ind[2]) {
                out[i] = -1;
                rm++;
            }
        }
        if (rm) atomicAdd(&removed, rm);
        __syncthreads();
    }
    if (threadIdx.x == 0) nmatch[p] = nm - removed;
}

// ---------------------------------------------------------------------------
// Fuse
// ---------------------------------------------------------------------------
struct FuseTables {
    float scale[ORBG_MAX_LEVELS];      // pKF->mvScaleFactors
    float inv_sigma2[ORBG_MAX_LEVELS]; // pKF->mvInvLevelSigma2
};

struct FuseKey {  // a grid entry in LDS
    float x, y;
    int io;  // index << 4 | octave
};

#ifndef FUSE_SPLIT
#define FUSE_SPLIT 4
#endif
#define FU_CELLS (ORBG_GRID_COLS * ORBG_GRID_ROWS)
static_assert(FU_CELLS == 256 * 12, "kf_grid_build's scan gives 12 grid cells to each of 256 threads");

// A KeyFrame's grid (Frame::AssignFeaturesToGrid / PosInGrid, Frame.cc:273-274, 292-307,
// 510-520, copied into the KeyFrame) counting-sorted into LDS by all 256 threads:
// afterwards cstart[c] is the END of cell c (its start cstart[c - 1]); the order inside a cell
// is irrelevant (the selection keys carry the index).
__device__ void kf_grid_build(const orbg_keypoint *__restrict__ kps, int n, const orbg_bounds &B,
                              float inv_w, float inv_h, int *cstart, FuseKey *keys)
{
    const int tid = threadIdx.x;
    for (int c = tid; c <= FU_CELLS; c += 256) cstart[c] = 0;
    __syncthreads();
    for (int i = tid; i < n; i += 256) {
        const orbg_keypoint kp = kps[i];
        const int px = (int)roundf((kp.x - B.min_x) * inv_w);
        const int py = (int)roundf((kp.y - B.min_y) * inv_h);
        if (px < 0 || px >= ORBG_GRID_COLS || py < 0 || py >= ORBG_GRID_ROWS) continue;
        atomicAdd(&cstart[px * ORBG_GRID_ROWS + py + 1], 1);
    }
    __syncthreads();
    // exclusive starts: 12 cells per thread, then a block scan of the thread totals
    {
        __shared__ int part[256];
        const int c0 = tid * 12;
        int loc = 0;
        for (int c = c0; c < c0 + 12; c++) loc += cstart[c + 1];
        part[tid] = loc;
        __syncthreads();
        for (int o = 1; o < 256; o <<= 1) {
            const int v = tid >= o ? part[tid - o] : 0;
            __syncthreads();
            part[tid] += v;
            __syncthreads();
        }
        int run = tid ? part[tid - 1] : 0;
        for (int c = c0; c < c0 + 12; c++) {
            const int v = cstart[c + 1];
            cstart[c + 1] = run + v;
            run += v;
        }
    }
    __syncthreads();
    // scatter: cstart[c] (the start of cell c) is the cell's cursor
    for (int i = tid; i < n; i += 256) {
        const orbg_keypoint kp = kps[i];
        const int px = (int)roundf((kp.x - B.min_x) * inv_w);
        const int py = (int)roundf((kp.y - B.min_y) * inv_h);
        if (px < 0 || px >= ORBG_GRID_COLS || py < 0 || py >= ORBG_GRID_ROWS) continue;
        const int slot = atomicAdd(&cstart[px * ORBG_GRID_ROWS + py], 1);
        keys[slot] = FuseKey{kp.x, kp.y, i << 4 | (kp.octave & 15)};
    }
    __syncthreads();
}

// KeyFrame::GetFeaturesInArea(u, v, r) (KeyFrame.cc:750-790: the cell range on the int
// bounds kminx / kminy with the Frame's cell sizes, |dx| < r && |dy| < r), the level window
// [lvl - 1, lvl], gate(idx, octave, kx, ky) and the least 64-bit key (distance, cell, index):
// the first candidate of the least distance in the reference's enumeration (strict <).
// Returns ~0 when no candidate passes.
template <class Gate>
__device__ __forceinline__ unsigned long long kf_grid_best(const int *cstart, const FuseKey *keys,
                                                           const uint8_t *__restrict__ kdesc,
                                                           const uint32_t q[8], float u, float v,
                                                           float r, int lvl, float kminx,
                                                           float kminy, float inv_w, float inv_h,
                                                           Gate gate)
{
    const int cx0 = max(0, (int)floorf((u - kminx - r) * inv_w));
    if (cx0 >= ORBG_GRID_COLS) return ~0ull;
    const int cx1 = min(ORBG_GRID_COLS - 1, (int)ceilf((u - kminx + r) * inv_w));
    if (cx1 < 0) return ~0ull;
    const int cy0 = max(0, (int)floorf((v - kminy - r) * inv_h));
    if (cy0 >= ORBG_GRID_ROWS) return ~0ull;
    const int cy1 = min(ORBG_GRID_ROWS - 1, (int)ceilf((v - kminy + r) * inv_h));
    if (cy1 < 0) return ~0ull;
    unsigned long long best = ~0ull;
    for (int ix = cx0; ix <= cx1; ix++)
        for (int iy = cy0; iy <= cy1; iy++) {
            const int c = ix * ORBG_GRID_ROWS + iy;
            const int j0 = c ? cstart[c - 1] : 0, j1 = cstart[c];
            for (int j = j0; j < j1; j++) {
                const FuseKey e = keys[j];
                if (!(fabsf(e.x - u) < r && fabsf(e.y - v) < r)) continue;
                const int kl = e.io & 15, idx = e.io >> 4;
                if (kl < lvl - 1 || kl > lvl) continue;
                if (!gate(idx, kl, e.x, e.y)) continue;
                const uint4 *kd = (const uint4 *)(kdesc + (size_t)idx * 32);
                const uint4 a = kd[0], b = kd[1];
                const int d = __popc(q[0] ^ a.x) + __popc(q[1] ^ a.y) + __popc(q[2] ^ a.z) +
                              __popc(q[3] ^ a.w) + __popc(q[4] ^ b.x) + __popc(q[5] ^ b.y) +
                              __popc(q[6] ^ b.z) + __popc(q[7] ^ b.w);
                const unsigned long long key = ((unsigned long long)d << 40) |
                                               ((unsigned long long)c << 20) | (unsigned)idx;
                best = key < best ? key : best;
            }
        }
    return best;
}

__device__ __forceinline__ void load_desc8(const uint8_t *__restrict__ p, uint32_t q[8])
{
    const uint4 *dp = (const uint4 *)p;
    const uint4 a = dp[0], b = dp[1];
    q[0] = a.x; q[1] = a.y; q[2] = a.z; q[3] = a.w;
    q[4] = b.x; q[5] = b.y; q[6] = b.z; q[7] = b.w;
}

// cv::gemm small-matrix pin: out = alpha * A x (+ c), A the 3x3 block of a 3x4 (stride 4) or
// 3x3 (stride 3) row-major matrix, double work type, one rounding per element
__device__ __forceinline__ void mk_gemm3(const float *A, int stride, bool trans, const float x[3],
                                         double alpha, const float *c, float out[3])
{
#pragma unroll
    for (int r = 0; r < 3; r++) {
        double t = 0.0;
#pragma unroll
        for (int k = 0; k < 3; k++)
            t += (double)(trans ? A[stride * k + r] : A[stride * r + k]) * (double)x[k];
        t *= alpha;
        if (c) t += (double)c[r];
        out[r] = (float)t;
    }
}

// SIM3 = false: Fuse(pKF, vpMapPoints, th) (:968-1069).  SIM3 = true: Fuse(pKF, Scw, vpPoints,
// th, vpReplacePoint) (:1133-1238): cams[p].Tcw holds Scw's rows 0..2, and the candidates
// are ranked by descriptor distance alone (no reprojection gate, no mvuRight)
template <bool SIM3>
__global__ __launch_bounds__(256) void k_fuse(orbg_keyframes K, int cap,
                                              const int32_t *__restrict__ kf_index,
                                              const orbg_frustum_camera *__restrict__ cams,
                                              const orbg_map_point *__restrict__ mps,
                                              const uint8_t *__restrict__ mdesc,
                                              const int32_t *__restrict__ mcounts, int mcap,
                                              float th, FuseTables T,
                                              int32_t *__restrict__ best_idx,
                                              int32_t *__restrict__ best_dist,
                                              int32_t *__restrict__ nfused,
                                              int32_t *__restrict__ err_flag)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t fu_lds[];
    int *cstart = (int *)fu_lds;                         // FU_CELLS + 1
    FuseKey *keys = (FuseKey *)(fu_lds + (FU_CELLS + 4) * 4);
    __shared__ int nf_total;
    // FUSE_SPLIT workgroups per pair share its MapPoints (each builds the KeyFrame grid);
    // their counts meet in nfused[p] (zeroed by the launcher)
    const int p = blockIdx.x / FUSE_SPLIT, split = blockIdx.x - p * FUSE_SPLIT, tid = threadIdx.x;
    const int kf = kf_index[p];
    // counts are device data the host never sees: one past its capacity would overrun the
    // LDS grid (cap entries) or the pair's output rows, so it is clamped and flagged
    // (ORBG_DEVFLAG_COUNT, sticky until orbg_check_errors)
    const int n_in = K.counts[kf], nm_in = mcounts[p];
    const int n = min(max(n_in, 0), cap), nm = min(max(nm_in, 0), mcap);
    if (tid == 0 && split == 0 && (n != n_in || nm != nm_in)) {
        atomicOr(err_flag, ORBG_DEVFLAG_COUNT);
        atomicMin(err_flag + 1, p);
    }
    const orbg_frustum_camera C = cams[p];
    const orbg_keypoint *kps = K.kps + (size_t)kf * cap;
    const float inv_w = (float)ORBG_GRID_COLS / (float)(C.bounds.max_x - C.bounds.min_x);
    const float inv_h = (float)ORBG_GRID_ROWS / (float)(C.bounds.max_y - C.bounds.min_y);
    if (tid == 0) nf_total = 0;
    kf_grid_build(kps, n, C.bounds, inv_w, inv_h, cstart, keys);
    // KeyFrame::mnMinX .. mnMaxY are ints, the Frame's truncated (KeyFrame.h:288-291,
    // KeyFrame.cc:51): IsInImage and GetFeaturesInArea's cell range use them, the grid (and
    // its inverse cell sizes) is the Frame's
    const float kminx = (float)(int)C.bounds.min_x, kmaxx = (float)(int)C.bounds.max_x;
    const float kminy = (float)(int)C.bounds.min_y, kmaxy = (float)(int)C.bounds.max_y;
    int fused = 0;
    float Tw[12];
    if (SIM3) {
        sim3_decompose(C.Tcw, Tw);
    } else {
#pragma unroll
        for (int k = 0; k < 12; k++) Tw[k] = C.Tcw[k];
    }
    const float tc[3] = {Tw[3], Tw[7], Tw[11]};
    // KeyFrame::GetCameraCenter: Ow = -Rwc*tcw (cv::gemm pin); the Sim3 variant's
    // Ow = -Rcw.t()*tcw is the same sums
    float Ow[3];
    mk_gemm3(Tw, 4, true, tc, -1.0, nullptr, Ow);
    const uint8_t *kdesc = K.desc + (size_t)kf * cap * 32;
    const float *kur = (!SIM3 && K.uright) ? K.uright + (size_t)kf * cap : nullptr;
    for (int i = split * 256 + tid; i < nm; i += 256 * FUSE_SPLIT) {
        const size_t o = (size_t)p * mcap + i;
        int bidx = -1, bdist = 256;
        const orbg_map_point mp = mps[o];
        do {
            if (!(mp.flags & ORBG_MP_VALID)) break;
            const float P[3] = {mp.x, mp.y, mp.z};
            float Pc[3];
            mk_gemm3(Tw, 4, false, P, 1.0, tc, Pc);
            if (Pc[2] < 0.0f) break;
            const float invz = 1 / Pc[2];
            const float x = Pc[0] * invz, y = Pc[1] * invz;
            const float u = C.fx * x + C.cx, v = C.fy * y + C.cy;
            if (!(u >= kminx && u < kmaxx && v >= kminy && v < kmaxy)) break;
            const float ur = u - C.bf * invz;
            const float maxDistance = 1.2f * mp.max_dist, minDistance = 0.8f * mp.min_dist;
            const float PO0 = P[0] - Ow[0], PO1 = P[1] - Ow[1], PO2 = P[2] - Ow[2];
            double s = 0.0;
            s += (double)PO0 * (double)PO0;
            s += (double)PO1 * (double)PO1;
            s += (double)PO2 * (double)PO2;
            const float dist3D = (float)sqrt(s);
            if (dist3D < minDistance || dist3D > maxDistance) break;
            double dot = 0.0;
            dot += (double)PO0 * (double)mp.nx;
            dot += (double)PO1 * (double)mp.ny;
            dot += (double)PO2 * (double)mp.nz;
            if (dot < 0.5 * (double)dist3D) break;
            const int lvl = predict_scale(mp.max_dist, dist3D, C.log_scale_factor, C.nlevels);
            const float r = th * T.scale[lvl];
            uint32_t q[8];
            load_desc8(mdesc + o * 32, q);
            // the chi-square reprojection gates (:1041-1063); the Sim3 variant has none
            auto gate = [&](int idx, int kl, float kx, float ky) -> bool {
                if (SIM3) return true;
                const float kr = kur ? kur[idx] : -1.0f;
                if (kr >= 0) {
                    const float ex = u - kx, ey = v - ky, er = ur - kr;
                    const float e2 = ex * ex + ey * ey + er * er;
                    return !((double)(e2 * T.inv_sigma2[kl]) > 7.8);
                }
                const float ex = u - kx, ey = v - ky;
                const float e2 = ex * ex + ey * ey;
                return !((double)(e2 * T.inv_sigma2[kl]) > 5.99);
            };
            const unsigned long long best =
                kf_grid_best(cstart, keys, kdesc, q, u, v, r, lvl, kminx, kminy, inv_w, inv_h, gate);
            if (best == ~0ull) break;
            bdist = (int)(best >> 40);
            if (bdist <= TM_TH_LOW) {
                bidx = (int)(best & 0xFFFFFu);
                fused++;
            }
        } while (0);
        best_idx[o] = bidx;
        best_dist[o] = bdist;
    }
    if (fused) atomicAdd(&nf_total, fused);
    __syncthreads();
    if (tid == 0 && nf_total) atomicAdd(&nfused[p], nf_total);
}

// ---------------------------------------------------------------------------
// SearchBySim3
// ---------------------------------------------------------------------------
// ORBmatcher::SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th) (ORBmatcher.cc:
// 1262-1470; LoopClosing::ComputeSim3): both directions are per-point searches with no
// shared state (each point's best over the other KeyFrame's grid, TH_HIGH), then the matches
// that agree both ways are kept.  k_sim3_match: workgroup 2p + d = direction d of pair p
// (d = 0: pKF1's points into pKF2 with sR21 / t21; d = 1: pKF2's into pKF1 with sR12 / t12),
// writing vnMatch1 / vnMatch2; k_sim3_resolve: one workgroup per pair, the mutual check.
#define SIM3_TH_HIGH 100
#ifndef SIM3_SPLIT
#define SIM3_SPLIT 4
#endif

__global__ __launch_bounds__(256) void k_sim3_match(orbg_keyframes K, int cap,
                                                    const int32_t *__restrict__ kf1,
                                                    const int32_t *__restrict__ kf2,
                                                    const orbg_sim3_pair *__restrict__ pairs,
                                                    const orbg_map_point *__restrict__ mps,
                                                    const uint8_t *__restrict__ mdesc,
                                                    const uint8_t *__restrict__ matched1,
                                                    const uint8_t *__restrict__ matched2,
                                                    float th, FuseTables T,
                                                    int32_t *__restrict__ vn,
                                                    int32_t *__restrict__ err_flag)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t fu_lds[];
    int *cstart = (int *)fu_lds;
    FuseKey *keys = (FuseKey *)(fu_lds + (FU_CELLS + 4) * 4);
    // workgroup = (pair, direction, split): SIM3_SPLIT workgroups share a direction's points
    // (each builds the target grid), so a launch of 256 pairs fills the chip
    const int p = blockIdx.x / (2 * SIM3_SPLIT), rem = blockIdx.x - p * 2 * SIM3_SPLIT;
    const int d = rem & 1, split = rem >> 1, tid = threadIdx.x;
    const int ks = d ? kf2[p] : kf1[p], kt = d ? kf1[p] : kf2[p];  // source / target KeyFrame
    // clamped to the capacity and flagged as in k_fuse
    const int ns_in = K.counts[ks], nt_in = K.counts[kt];
    const int ns = min(max(ns_in, 0), cap), nt = min(max(nt_in, 0), cap);
    if (tid == 0 && split == 0 && (ns != ns_in || nt != nt_in)) {
        atomicOr(err_flag, ORBG_DEVFLAG_COUNT);
        atomicMin(err_flag + 1, p);
    }
    const orbg_sim3_pair G = pairs[p];
    const float inv_w = (float)ORBG_GRID_COLS / (float)(G.bounds.max_x - G.bounds.min_x);
    const float inv_h = (float)ORBG_GRID_ROWS / (float)(G.bounds.max_y - G.bounds.min_y);
    kf_grid_build(K.kps + (size_t)kt * cap, nt, G.bounds, inv_w, inv_h, cstart, keys);
    const float kminx = (float)(int)G.bounds.min_x, kmaxx = (float)(int)G.bounds.max_x;
    const float kminy = (float)(int)G.bounds.min_y, kmaxy = (float)(int)G.bounds.max_y;
    // sR12 = s12*R12, sR21 = (1.0/s12)*R12.t() (Mat * scalar: convertTo with the float alpha,
    // one rounding), t21 = -sR21*t12 (gemm, alpha -1), :1275-1279
    float M[9], tm[3];
    if (d == 0) {
        const float a = (float)(1.0 / (double)G.s12);
#pragma unroll
        for (int r = 0; r < 3; r++)
#pragma unroll
            for (int c = 0; c < 3; c++) M[3 * r + c] = G.R12[3 * c + r] * a + 0.0f;
        mk_gemm3(M, 3, false, G.t12, -1.0, nullptr, tm);
    } else {
#pragma unroll
        for (int k = 0; k < 9; k++) M[k] = G.R12[k] * G.s12 + 0.0f;
#pragma unroll
        for (int k = 0; k < 3; k++) tm[k] = G.t12[k];
    }
    const float *Tsw = d ? G.T2w : G.T1w;  // the source KeyFrame's pose
    const float ts[3] = {Tsw[3], Tsw[7], Tsw[11]};
    const uint8_t *am = d ? matched2 : matched1;
    const uint8_t *kdesc = K.desc + (size_t)kt * cap * 32;
    auto nogate = [](int, int, float, float) { return true; };
    for (int i = split * 256 + tid; i < ns; i += 256 * SIM3_SPLIT) {
        const size_t o = (size_t)ks * cap + i;
        int best_i = -1;
        const orbg_map_point mp = mps[o];
        do {
            // !pMP || vbAlreadyMatched || isBad (:1298-1304 / :1366-1372)
            if (!(mp.flags & ORBG_MP_VALID)) break;
            if (am && am[(size_t)p * cap + i]) break;
            const float P[3] = {mp.x, mp.y, mp.z};
            float Pcs[3], Pc[3];
            mk_gemm3(Tsw, 4, false, P, 1.0, ts, Pcs);  // R1w*p3Dw + t1w
            mk_gemm3(M, 3, false, Pcs, 1.0, tm, Pc);   // sR21*p3Dc1 + t21
            if (Pc[2] < 0.0f) break;
            const float invz = (float)(1.0 / (double)Pc[2]);
            const float x = Pc[0] * invz, y = Pc[1] * invz;
            const float u = G.fx * x + G.cx, v = G.fy * y + G.cy;
            if (!(u >= kminx && u < kmaxx && v >= kminy && v < kmaxy)) break;
            const float maxDistance = 1.2f * mp.max_dist, minDistance = 0.8f * mp.min_dist;
            double s = 0.0;
            s += (double)Pc[0] * (double)Pc[0];
            s += (double)Pc[1] * (double)Pc[1];
            s += (double)Pc[2] * (double)Pc[2];
            const float dist3D = (float)sqrt(s);  // cv::norm(p3Dc2)
            if (dist3D < minDistance || dist3D > maxDistance) break;
            const int lvl = predict_scale(mp.max_dist, dist3D, G.log_scale_factor, G.nlevels);
            const float r = th * T.scale[lvl];
            uint32_t q[8];
            load_desc8(mdesc + o * 32, q);
            const unsigned long long best = kf_grid_best(cstart, keys, kdesc, q, u, v, r, lvl,
                                                         kminx, kminy, inv_w, inv_h, nogate);
            if (best != ~0ull && (int)(best >> 40) <= SIM3_TH_HIGH)
                best_i = (int)(best & 0xFFFFFu);
        } while (0);
        vn[((size_t)p * 2 + d) * cap + i] = best_i;
    }
}

// the mutual check (:1458-1470): vpMatches12[i1] = vpMapPoints2[idx2] when vnMatch1[i1] =
// idx2 and vnMatch2[idx2] = i1
__global__ __launch_bounds__(256) void k_sim3_resolve(const int32_t *__restrict__ kf1,
                                                      const int32_t *__restrict__ counts, int cap,
                                                      const int32_t *__restrict__ vn,
                                                      int32_t *__restrict__ match12,
                                                      int32_t *__restrict__ nfound)
{
    __shared__ int tot;
    const int p = blockIdx.x, tid = threadIdx.x;
    const int n1 = min(max(counts[kf1[p]], 0), cap);  // flagged by k_sim3_match
    if (tid == 0) tot = 0;
    __syncthreads();
    const int32_t *v1 = vn + (size_t)p * 2 * cap, *v2 = v1 + cap;
    int cnt = 0;
    for (int i = tid; i < n1; i += 256) {
        const int i2 = v1[i];
        const bool ok = i2 >= 0 && v2[i2] == i;
        match12[(size_t)p * cap + i] = ok ? i2 : -1;
        cnt += ok;
    }
    if (cnt) atomicAdd(&tot, cnt);
    __syncthreads();
    if (tid == 0) nfound[p] = tot;
}

int launch_fuse(hipStream_t st, const orbg_keyframes &K, int cap, const int32_t *kf,
                const orbg_frustum_camera *cams, const orbg_map_point *mps, const uint8_t *mdesc,
                const int32_t *mcounts, int mcap, int npairs, float th, const float *scale,
                const float *inv_sigma2, int nlevels, int sim3, int32_t *best_idx,
                int32_t *best_dist, int32_t *nfused, int32_t *err_flag)
{
    if (npairs <= 0) return 0;
    if (cap > 8192) return -95;  // the grid's entries in LDS
    FuseTables T{};
    for (int l = 0; l < ORBG_MAX_LEVELS; l++) {
        const int s = l < nlevels ? l : nlevels - 1;
        T.scale[l] = scale[s];
        T.inv_sigma2[l] = inv_sigma2[s];
    }
    const size_t lds = (FU_CELLS + 4) * 4 + (size_t)cap * sizeof(FuseKey);
    const void *fn = sim3 ? (const void *)k_fuse<true> : (const void *)k_fuse<false>;
    if (lds > 64 * 1024 &&
        hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
            hipSuccess)
        return -5;
    if (hipMemsetAsync(nfused, 0, (size_t)npairs * sizeof(int32_t), st) != hipSuccess) return -5;
    if (sim3)
        hipLaunchKernelGGL(k_fuse<true>, dim3(npairs * FUSE_SPLIT), dim3(256), lds, st, K, cap,
                           kf, cams, mps, mdesc, mcounts, mcap, th, T, best_idx, best_dist, nfused,
                           err_flag);
    else
        hipLaunchKernelGGL(k_fuse<false>, dim3(npairs * FUSE_SPLIT), dim3(256), lds, st, K, cap,
                           kf, cams, mps, mdesc, mcounts, mcap, th, T, best_idx, best_dist, nfused,
                           err_flag);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

// vn: scratch of npairs * 2 * cap int32 (vnMatch1 / vnMatch2 per pair)
int launch_search_by_sim3(hipStream_t st, const orbg_keyframes &K, int cap, const int32_t *kf1,
                          const int32_t *kf2, const orbg_sim3_pair *pairs,
                          const orbg_map_point *mps, const uint8_t *mdesc,
                          const uint8_t *matched1, const uint8_t *matched2, int npairs, float th,
                          const float *scale, int nlevels, int32_t *vn, int32_t *match12,
                          int32_t *nfound, int32_t *err_flag)
{
    if (npairs <= 0) return 0;
    if (cap > 8192) return -95;  // the grid's entries in LDS
    FuseTables T{};
    for (int l = 0; l < ORBG_MAX_LEVELS; l++) T.scale[l] = scale[l < nlevels ? l : nlevels - 1];
    const size_t lds = (FU_CELLS + 4) * 4 + (size_t)cap * sizeof(FuseKey);
    if (lds > 64 * 1024 &&
        hipFuncSetAttribute((const void *)k_sim3_match, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds) != hipSuccess)
        return -5;
    hipLaunchKernelGGL(k_sim3_match, dim3(2 * SIM3_SPLIT * npairs), dim3(256), lds, st, K, cap, kf1, kf2,
                       pairs, mps, mdesc, matched1, matched2, th, T, vn, err_flag);
    hipLaunchKernelGGL(k_sim3_resolve, dim3(npairs), dim3(256), 0, st, kf1, K.counts, cap, vn,
                       match12, nfound);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

int launch_tri_match(hipStream_t st, const orbg_keyframes &K, int cap, const int32_t *kf1,
                     const int32_t *kf2, const orbg_triangulation_pair *geo, int npairs,
                     const float *scale, const float *sigma2, int nlevels, int only_stereo,
                     int check_ori, int32_t *match, int32_t *nmatch)
{
    if (npairs <= 0) return 0;
    if (cap > 65535) return -95;  // positions in the key's low 16 bits
    TriTables T{};
    for (int l = 0; l < ORBG_MAX_LEVELS; l++) {
        const int s = l < nlevels ? l : nlevels - 1;
        T.scale[l] = scale[s];
        T.epi_th[l] = 3.84 * (double)sigma2[s];
    }
    hipLaunchKernelGGL(k_tri_match, dim3(npairs), dim3(256), 0, st, K, cap, kf1, kf2, geo, T,
                       only_stereo, check_ori, match, nmatch);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

}  // namespace orbg
