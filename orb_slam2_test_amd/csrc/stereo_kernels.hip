// stereo_kernels.hip -- Frame::ComputeStereoMatches (src/Frame.cc:619-834) on gfx950.
//
// Per stereo pair (left frame, right frame of the last batch), four launches:
//   k_stereo_rows    :637-662  row table (vRowIndices): right keypoint iR is listed in rows
//                              floor(y - r) .. ceil(y + r), r = 2 * scale[octave]; one
//                              workgroup per pair, counts / scan / fill in LDS, the lists go
//                              to global scratch (order inside a row is free: see below)
//   k_stereo_match   :676-738  wave per left keypoint: candidates of row (int)vL, octave
//                              within +-1, uL - maxD <= uR <= uL; best = minimum of
//                              (Hamming distance, iR) below TH_HIGH -- the reference walks
//                              each row in increasing iR with a strict <, so its winner is
//                              exactly the lexicographic minimum
//   k_stereo_sad     :740-832  wave per accepted keypoint: 11 shifts x 11 rows of 11-pixel
//                              SADs (both patches minus their centre, integer-exact like the
//                              float cv::norm of integer values), first minimum, parabola in
//                              float, sub-pixel uR, disparity range, depth = bf / disparity
//   k_stereo_median  :836-851  workgroup per pair: median = (n/2)-th smallest SAD by a
//                              two-pass 8-bit radix select (SAD <= 121 * 510 < 2^16), then
//                              clear every match with SAD >= 1.5f * 1.4f * median
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdlib>
#include <mutex>

#include "../../include/orbg.h"
#include "orbg_device.h"
#include "orbg_internal.h"

#define ORBG_ST_MAX_DEV 64  // devices whose k_stereo_rows_match LDS attribute is cached

#pragma clang fp contract(off)

namespace orbg {

void prof_begin(void *prof, hipStream_t s, const char *n, hipEvent_t *a);
void prof_end(void *prof, hipStream_t s, const char *n, hipEvent_t a);

#ifndef ORBG_ST_XCD
#define ORBG_ST_XCD 1  // XCD-aware pair mapping of k_stereo_match / k_stereo_sad (0: A/B)
#endif
#ifndef ORBG_ST_SADW
#define ORBG_ST_SADW 1  // k_stereo_sad rows read as dwords, v_sad_u16 (0: byte reads, A/B)
#endif
#ifndef ORBG_ST_STG16
#define ORBG_ST_STG16 1  // k_stereo_sad staging: 16-byte loads on 33 lanes (0: dword per lane, +17% stereo_sad)
#endif
#define ST_TH_HIGH 100
#define ST_TH_ORB ((100 + 50) / 2)
#define ST_W 5
#define ST_L 5
#define ST_ROWS_T 1024
#define ST_MAX_ROWS 4096

// geometry of the stereo pass (host-filled)
struct StereoGeom {
    int32_t h;            // level-0 rows (nRows)
    int32_t fc;           // keypoints per frame slot
    int32_t list_cap;     // row-list entries per pair
    float bf, max_d;      // mbf, maxD = mbf / minZ (+inf for minZ <= 0)
    float scale[16], inv_scale[16];
    int32_t lw[16], lpitch[16];
    int64_t pyr_off[16];  // level l >= 1 in a frame's pyramid
};

// ---- row table --------------------------------------------------------------------
__global__ __launch_bounds__(ST_ROWS_T) void k_stereo_rows(StereoGeom G,
                                                          const orbg_keypoint *__restrict__ kps,
                                                          const int32_t *__restrict__ counts,
                                                          const int32_t *__restrict__ right,
                                                          int32_t *__restrict__ row_off,
                                                          int16_t *__restrict__ row_list)
{
    __shared__ int cnt[ST_MAX_ROWS + 1];
    const int p = blockIdx.x, tid = threadIdx.x;
    const int fr = right[p];
    const orbg_keypoint *kr = kps + (size_t)fr * G.fc;
    const int nr = counts[fr];
    const int H = G.h;
    for (int y = tid; y <= H; y += ST_ROWS_T) cnt[y] = 0;
    __syncthreads();
    for (int iR = tid; iR < nr; iR += ST_ROWS_T) {
        const orbg_keypoint k = kr[iR];
        const float r = 2.0f * G.scale[k.octave];
        const int maxr = (int)ceilf(k.y + r), minr = (int)floorf(k.y - r);
        for (int yi = max(minr, 0); yi <= min(maxr, H - 1); yi++) atomicAdd(&cnt[yi], 1);
    }
    __syncthreads();
    // exclusive scan over H rows (<= 4 per thread)
    __shared__ int wsum[ST_ROWS_T / 64];
    const int per = (H + ST_ROWS_T - 1) / ST_ROWS_T;
    int loc = 0;
    for (int k = 0; k < per; k++) {
        const int y = tid * per + k;
        loc += y < H ? cnt[y] : 0;
    }
    const int lane = tid & 63, wv = tid >> 6;
    const int incl = wave_incl_scan(loc);
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    int before = 0;
    for (int i = 0; i < wv; i++) before += wsum[i];
    int run = before + incl - loc;
    int32_t *off = row_off + (size_t)p * (ST_MAX_ROWS + 1);
    for (int k = 0; k < per; k++) {
        const int y = tid * per + k;
        if (y < H) {
            const int c = cnt[y];
            cnt[y] = run;  // becomes the fill cursor
            off[y] = run;
            run += c;
        }
    }
    if (tid == ST_ROWS_T - 1) off[H] = run;
    __syncthreads();
    int16_t *list = row_list + (size_t)p * G.list_cap;
    for (int iR = tid; iR < nr; iR += ST_ROWS_T) {
        const orbg_keypoint k = kr[iR];
        const float r = 2.0f * G.scale[k.octave];
        const int maxr = (int)ceilf(k.y + r), minr = (int)floorf(k.y - r);
        for (int yi = max(minr, 0); yi <= min(maxr, H - 1); yi++) {
            const int slot = atomicAdd(&cnt[yi], 1);
            if (slot < G.list_cap) list[slot] = (int16_t)iR;
        }
    }
}

// ---- descriptor match ---------------------------------------------------------------
// 16 lanes per left keypoint over the row's candidates, then a 16-lane minimum of
// (dist << 16 | iR) -- the lexicographic (distance, index) minimum.  ST_WAVES waves per pair
// walk the left keypoints.
#define ST_WAVES 512
#ifndef ST_MATCH_WAVES
#define ST_MATCH_WAVES ST_WAVES  // waves per pair of k_stereo_match (256: +4%, 1024: +50%)
#endif
#ifndef ST_SAD_WAVES
#define ST_SAD_WAVES 256  // waves per pair of k_stereo_sad (512: +3%, 128: tie, 64: +1.5%)
#endif

// A wave matches ST_MG left keypoints at once (iL = base + j * ST_WAVES), 16 lanes each: the
// dependent chain (left keypoint -> row offsets -> row list -> right keypoint -> descriptor)
// is paid once per batch instead of once per keypoint.
#ifndef ST_MG
#define ST_MG 4  // keypoints per wave batch (measured: 2 -> 0.371 ms, 8 -> 0.444 against 0.327)
#endif
#define ST_LPK (64 / ST_MG)  // lanes per keypoint

__global__ __launch_bounds__(256) void k_stereo_match(StereoGeom G,
                                                     const orbg_keypoint *__restrict__ kps,
                                                     const uint8_t *__restrict__ desc,
                                                     const int32_t *__restrict__ counts,
                                                     const int32_t *__restrict__ left,
                                                     const int32_t *__restrict__ right,
                                                     const int32_t *__restrict__ row_off,
                                                     const int16_t *__restrict__ row_list,
                                                     int32_t *__restrict__ best_r)
{
    static_assert(ST_MG == 2 || ST_MG == 4 || ST_MG == 8, "lanes per keypoint: 32, 16 or 8");
    // XCD-aware: the workgroups of one pair run on one XCD, so the right frame's keypoint and
    // descriptor rows they share are fetched into one L2 (not once per XCD)
    const int id = ORBG_ST_XCD ? xcd_remap(blockIdx.x + gridDim.x * blockIdx.y, gridDim.x * gridDim.y)
                               : (int)(blockIdx.x + gridDim.x * blockIdx.y);
    const int p = id / gridDim.x, bx = id - p * gridDim.x;
    const int lane = threadIdx.x & 63, j = lane / ST_LPK, q16 = lane % ST_LPK;
    const int fl = left[p], fr = right[p];
    const int nl = counts[fl];
    const int32_t *off = row_off + (size_t)p * (ST_MAX_ROWS + 1);
    const orbg_keypoint *kr = kps + (size_t)fr * G.fc;
    const uint8_t *dr = desc + (size_t)fr * G.fc * 32;
    const int16_t *list = row_list + (size_t)p * G.list_cap;
    int32_t *out = best_r + (size_t)p * G.fc;
    for (int base = bx * 4 + (threadIdx.x >> 6); base < nl; base += ST_MG * ST_MATCH_WAVES) {
        const int iL = base + j * ST_MATCH_WAVES;
        const bool have = iL < nl;
        const orbg_keypoint kl = kps[(size_t)fl * G.fc + (have ? iL : base)];
        const int row = (int)kl.y;
        const float minU = kl.x - G.max_d, maxU = kl.x - 0.0f;
        int c0 = 0, c1 = 0;
        if (have && row >= 0 && row < G.h && !(maxU < 0)) {
            c0 = off[row];
            c1 = min(off[row + 1], G.list_cap);
        }
        const uint4 *qd = (const uint4 *)(desc + ((size_t)fl * G.fc + (have ? iL : base)) * 32);
        const uint4 q0 = qd[0], q1 = qd[1];
        uint32_t best = 0xFFFFFFFFu;
        for (int c = c0 + q16; c < c1; c += ST_LPK) {
            const int iR = list[c];
            const orbg_keypoint k = kr[iR];
            if (k.octave < kl.octave - 1 || k.octave > kl.octave + 1) continue;
            if (!(k.x >= minU && k.x <= maxU)) continue;
            const uint4 *d = (const uint4 *)(dr + (size_t)iR * 32);
            const uint4 d0 = d[0], d1 = d[1];
            const uint32_t dist = __popc(q0.x ^ d0.x) + __popc(q0.y ^ d0.y) + __popc(q0.z ^ d0.z) +
                                  __popc(q0.w ^ d0.w) + __popc(q1.x ^ d1.x) + __popc(q1.y ^ d1.y) +
                                  __popc(q1.z ^ d1.z) + __popc(q1.w ^ d1.w);
            best = min(best, (dist << 16) | (uint32_t)iR);
        }
#pragma unroll
        for (int o = ST_LPK / 2; o > 0; o >>= 1) best = min(best, (uint32_t)__shfl_xor((int)best, o, 64));
        if (q16 == 0 && have) {
            const int bestDist = best == 0xFFFFFFFFu ? ST_TH_HIGH : (int)(best >> 16);
            // the reference keeps a candidate only below TH_HIGH, then needs < (TH_HIGH+TH_LOW)/2
            out[iL] = (bestDist < ST_TH_HIGH && bestDist < ST_TH_ORB) ? (int)(best & 0xFFFF) : -1;
        }
    }
}

// ---- row table + descriptor match in one workgroup per pair (default) ----------------
// k_stereo_rows + k_stereo_match's semantics with the right frame staged in LDS: the row table
// is built in LDS (never written to HBM), the right keypoints' (x, octave) and descriptors are
// copied in once with coalesced 16-byte loads, and the match's dependent chain (row offsets ->
// row list -> right keypoint -> descriptor) is LDS reads only.  ST_FUSED_T threads; a pair
// whose row lists outgrow the LDS list capacity (host: what the layout leaves) builds them in
// its global scratch instead (same code, global reads).
#ifndef ORBG_ST_FUSED
#define ORBG_ST_FUSED 1  // 0: k_stereo_rows + k_stereo_match (A/B)
#endif
#define ST_FUSED_T 1024

struct StFusedLds {
    int lcap;  // int16 list entries in LDS
};

// LDS layout (bytes): cnt[(h + 1) ints] | rx[fc floats] | roct[fc bytes, padded to 16] |
// rdesc[fc * 32] | list[lcap int16]
__host__ __device__ inline size_t st_fused_head(int h, int fc)
{
    size_t o = ((size_t)(h + 1) * 4 + 15) & ~(size_t)15;
    o += ((size_t)fc * 4 + 15) & ~(size_t)15;
    o += ((size_t)fc + 15) & ~(size_t)15;
    o += (size_t)fc * 32;
    return o;
}

template <bool LDSLIST>
__device__ __forceinline__ void st_fused_body(const StereoGeom &G, int p, int nr, int nl,
                                              const orbg_keypoint *__restrict__ kr,
                                              const orbg_keypoint *__restrict__ klf,
                                              const uint8_t *__restrict__ dlf, int *cnt,
                                              const float *rx, const int8_t *roct,
                                              const uint4 *rdesc, int16_t *list, int total,
                                              int32_t *__restrict__ out)
{
    const int tid = threadIdx.x, H = G.h;
    // fill (order inside a row is free: the match takes the lexicographic minimum)
    for (int iR = tid; iR < nr; iR += ST_FUSED_T) {
        const float y = kr[iR].y;
        const float r = 2.0f * G.scale[roct[iR]];
        const int maxr = (int)ceilf(y + r), minr = (int)floorf(y - r);
        for (int yi = max(minr, 0); yi <= min(maxr, H - 1); yi++) {
            const int slot = atomicAdd(&cnt[yi], 1);
            if (LDSLIST || slot < G.list_cap) list[slot] = (int16_t)iR;  // LDS: total <= lcap
        }
    }
    if (!LDSLIST) __threadfence_block();
    __syncthreads();
    // cnt[y] is now the end of row y; row y starts at cnt[y - 1] (0 for y = 0)
    const int lane = tid & 63, j = lane / ST_LPK, q16 = lane % ST_LPK;
    const int wv = tid >> 6;
    constexpr int NW = ST_FUSED_T / 64;
    // the left keypoint and descriptor of the next batch are loaded one batch ahead (the only
    // global reads of the loop: their latency behind this batch's LDS work)
    float nx, ny;
    int noct;
    uint4 nq0, nq1;
    auto fetch = [&](int base) {
        const int iL = base + j * NW;
        const int idx = iL < nl ? iL : (base < nl ? base : 0);
        const orbg_keypoint *k = klf + idx;
        nx = k->x;
        ny = k->y;
        noct = k->octave;
        const uint4 *qd = (const uint4 *)(dlf + (size_t)idx * 32);
        nq0 = qd[0];
        nq1 = qd[1];
    };
    fetch(wv);
    for (int base = wv; base < nl; base += ST_MG * NW) {
        const int iL = base + j * NW;
        const bool have = iL < nl;
        const float klx = nx, kly = ny;
        const int kloct = noct;
        const uint4 q0 = nq0, q1 = nq1;
        fetch(base + ST_MG * NW);
        const int row = (int)kly;
        const float minU = klx - G.max_d, maxU = klx - 0.0f;
        int c0 = 0, c1 = 0;
        if (have && row >= 0 && row < G.h && !(maxU < 0)) {
            c0 = row > 0 ? cnt[row - 1] : 0;
            c1 = LDSLIST ? cnt[row] : min(cnt[row], G.list_cap);
        }
        uint32_t best = 0xFFFFFFFFu;
        for (int c = c0 + q16; c < c1; c += ST_LPK) {
            const int iR = list[c];
            const int oct = roct[iR];
            if (oct < kloct - 1 || oct > kloct + 1) continue;
            const float x = rx[iR];
            if (!(x >= minU && x <= maxU)) continue;
            const uint4 d0 = rdesc[2 * iR], d1 = rdesc[2 * iR + 1];
            const uint32_t dist = __popc(q0.x ^ d0.x) + __popc(q0.y ^ d0.y) + __popc(q0.z ^ d0.z) +
                                  __popc(q0.w ^ d0.w) + __popc(q1.x ^ d1.x) + __popc(q1.y ^ d1.y) +
                                  __popc(q1.z ^ d1.z) + __popc(q1.w ^ d1.w);
            best = min(best, (dist << 16) | (uint32_t)iR);
        }
#pragma unroll
        for (int o = ST_LPK / 2; o > 0; o >>= 1) best = min(best, (uint32_t)__shfl_xor((int)best, o, 64));
        if (q16 == 0 && have) {
            const int bestDist = best == 0xFFFFFFFFu ? ST_TH_HIGH : (int)(best >> 16);
            out[iL] = (bestDist < ST_TH_HIGH && bestDist < ST_TH_ORB) ? (int)(best & 0xFFFF) : -1;
        }
    }
}

__global__ __launch_bounds__(ST_FUSED_T) void k_stereo_rows_match(
    StereoGeom G, const orbg_keypoint *__restrict__ kps, const uint8_t *__restrict__ desc,
    const int32_t *__restrict__ counts, const int32_t *__restrict__ left,
    const int32_t *__restrict__ right, int16_t *__restrict__ row_list, int lcap,
    int32_t *__restrict__ best_r)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t st_lds[];
    const int p = blockIdx.x, tid = threadIdx.x, H = G.h, fc = G.fc;
    const int fl = left[p], fr = right[p];
    const int nl = counts[fl], nr = counts[fr];
    uint8_t *b = st_lds;
    int *cnt = (int *)b;
    b += ((size_t)(H + 1) * 4 + 15) & ~(size_t)15;
    float *rx = (float *)b;
    b += ((size_t)fc * 4 + 15) & ~(size_t)15;
    int8_t *roct = (int8_t *)b;
    b += ((size_t)fc + 15) & ~(size_t)15;
    uint4 *rdesc = (uint4 *)b;
    b += (size_t)fc * 32;
    int16_t *llist = (int16_t *)b;
    const orbg_keypoint *kr = kps + (size_t)fr * fc;
    for (int y = tid; y <= H; y += ST_FUSED_T) cnt[y] = 0;
    // the right frame's descriptors: 16-byte words, coalesced
    {
        // four 16-byte loads in flight per thread before the LDS stores
        const uint4 *src = (const uint4 *)(desc + (size_t)fr * fc * 32);
        for (int i0 = 0; i0 < 2 * nr; i0 += 4 * ST_FUSED_T) {
            uint4 v[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int i = i0 + u * ST_FUSED_T + tid;
                v[u] = src[i < 2 * nr ? i : 0];
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int i = i0 + u * ST_FUSED_T + tid;
                if (i < 2 * nr) rdesc[i] = v[u];
            }
        }
    }
    __syncthreads();
    for (int iR = tid; iR < nr; iR += ST_FUSED_T) {
        const orbg_keypoint k = kr[iR];
        rx[iR] = k.x;
        roct[iR] = (int8_t)k.octave;
        const float r = 2.0f * G.scale[k.octave];
        const int maxr = (int)ceilf(k.y + r), minr = (int)floorf(k.y - r);
        for (int yi = max(minr, 0); yi <= min(maxr, H - 1); yi++) atomicAdd(&cnt[yi], 1);
    }
    __syncthreads();
    // exclusive scan over H rows (<= 4 per thread); cnt[y] becomes row y's fill cursor
    __shared__ int wsum[ST_FUSED_T / 64];
    const int per = (H + ST_FUSED_T - 1) / ST_FUSED_T;
    int loc = 0;
    for (int k = 0; k < per; k++) {
        const int y = tid * per + k;
        loc += y < H ? cnt[y] : 0;
    }
    const int lane = tid & 63, wv = tid >> 6;
    const int incl = wave_incl_scan(loc);
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    int before = 0, total = 0;
    for (int i = 0; i < ST_FUSED_T / 64; i++) {
        before += i < wv ? wsum[i] : 0;
        total += wsum[i];
    }
    int run = before + incl - loc;
    for (int k = 0; k < per; k++) {
        const int y = tid * per + k;
        if (y < H) {
            const int c = cnt[y];
            cnt[y] = run;
            run += c;
        }
    }
    __syncthreads();
    const orbg_keypoint *klf = kps + (size_t)fl * fc;
    const uint8_t *dlf = desc + (size_t)fl * fc * 32;
    int32_t *out = best_r + (size_t)p * fc;
    if (total <= lcap)  // workgroup-uniform
        st_fused_body<true>(G, p, nr, nl, kr, klf, dlf, cnt, rx, roct, rdesc, llist, total, out);
    else
        st_fused_body<false>(G, p, nr, nl, kr, klf, dlf, cnt, rx, roct, rdesc,
                             row_list + (size_t)p * G.list_cap, total, out);
}

// ---- SAD refinement -----------------------------------------------------------------
__device__ __forceinline__ const uint8_t *st_level(const StereoGeom &G, const uint8_t *img0,
                                                   int64_t img_fs, int img_pitch,
                                                   const uint8_t *pyr, int64_t pyr_frame, int f,
                                                   int l, int *pitch)
{
    if (l == 0) {
        *pitch = img_pitch;
        return img0 + f * img_fs;
    }
    *pitch = G.lpitch[l];
    return pyr + f * pyr_frame + G.pyr_off[l];
}

__device__ __forceinline__ void stereo_sad_one(const StereoGeom &G,
                                               const orbg_keypoint *__restrict__ kps,
                                               const int32_t *__restrict__ best_r,
                                               const uint8_t *__restrict__ img0, int64_t img_fs,
                                               int img_pitch, const uint8_t *__restrict__ pyr,
                                               int64_t pyr_frame, float *__restrict__ uright,
                                               float *__restrict__ depth,
                                               int32_t *__restrict__ sad_out, int p, int fl,
                                               int fr, int iL, int lane, int *sadw,
                                               uint32_t *stagew, int *shlw, int *shrw)
{
    float *ur = uright + (size_t)p * G.fc, *dp = depth + (size_t)p * G.fc;
    int32_t *so = sad_out + (size_t)p * G.fc;
    const int iR = best_r[(size_t)p * G.fc + iL];
    if (lane == 0) {
        ur[iL] = -1.0f;
        dp[iL] = -1.0f;
        so[iL] = -1;
    }
    if (iR < 0) return;
    const orbg_keypoint kl = kps[(size_t)fl * G.fc + iL];
    const float uR0 = kps[(size_t)fr * G.fc + iR].x;
    const int lev = kl.octave;
    const float sf = G.inv_scale[lev];
    const float scaleduL = roundf(kl.x * sf);
    const float scaledvL = roundf(kl.y * sf);
    const float scaleduR0 = roundf(uR0 * sf);
    const float iniu = scaleduR0 + ST_L - ST_W;
    const float endu = scaleduR0 + ST_L + ST_W + 1;
    if (iniu < 0 || endu >= G.lw[lev]) return;
    int lp, rp;
    const uint8_t *IL = st_level(G, img0, img_fs, img_pitch, pyr, pyr_frame, fl, lev, &lp);
    const uint8_t *IR = st_level(G, img0, img_fs, img_pitch, pyr, pyr_frame, fr, lev, &rp);
    const int yl = (int)scaledvL, xl = (int)scaleduL, xr = (int)scaleduR0;
    // stage the 11x11 left patch (columns xl-5..xl+5) and the 11x21 right strip (xr-10..xr+10)
    // as 4 / 7 aligned dwords per row (per-row alignment: the level-0 pitch may be odd)
    uint32_t *stL = stagew, *stR = stagew + 11 * 4;
#if ORBG_ST_STG16
    // one 16-byte load per lane, 33 lanes: (row, part) = left dwords 0-3, right dwords 0-3,
    // right dwords 3-6 (dword 3 stored twice, the same value)
    if (lane < 33) {
        const int r = lane / 3, c = lane - 3 * r;
        const int y = yl - ST_W + r;
        const uint8_t *src = c == 0 ? IL + (int64_t)y * lp + xl - ST_W
                                    : IR + (int64_t)y * rp + xr - 2 * ST_W;
        const int sh = (int)((uintptr_t)src & 3);
        const int d0 = c == 2 ? 3 : 0;
        const uint4 v = *(const uint4 *)((const uint32_t *)(src - sh) + d0);
        uint32_t *dst = (c == 0 ? stL + r * 4 : stR + r * 7) + d0;
        dst[0] = v.x;
        dst[1] = v.y;
        dst[2] = v.z;
        dst[3] = v.w;
        if (c == 0) shlw[r] = sh;
        if (c == 1) shrw[r] = sh;
    }
#else
    for (int t = lane; t < 11 * 11; t += 64) {
        const int r = t / 11, c = t - r * 11;  // c < 4: left dword, else right dword c - 4
        const int y = yl - ST_W + r;
        const uint8_t *src = c < 4 ? IL + (int64_t)y * lp + xl - ST_W
                                   : IR + (int64_t)y * rp + xr - 2 * ST_W;
        // pointer arithmetic, not an integer round trip: a global_, not a flat_, load
        const uint8_t *a = src - ((uintptr_t)src & 3);
        const uint32_t v = ((const uint32_t *)a)[c < 4 ? c : c - 4];
        if (c < 4)
            stL[r * 4 + c] = v;
        else
            stR[r * 7 + c - 4] = v;
        if (c == 0) shlw[r] = (int)((uintptr_t)src & 3);
        if (c == 4) shrw[r] = (int)((uintptr_t)src & 3);
    }
#endif
    if (lane < 2 * ST_L + 1) sadw[lane] = 0;
    wave_sync_lds();
    const uint8_t *bL = (const uint8_t *)stL, *bR = (const uint8_t *)stR;
    const int cl = bL[ST_W * 16 + shlw[ST_W] + ST_W];
    // items t = (shift, row): 11 x 11, two per lane
    for (int t = lane; t < (2 * ST_L + 1) * (2 * ST_W + 1); t += 64) {
        const int inc = t / (2 * ST_W + 1) - ST_L, dy = t % (2 * ST_W + 1);
        const int cr = bR[ST_W * 28 + shrw[ST_W] + 2 * ST_W + inc];
#if ORBG_ST_SADW
        // |(a - cl) - (b - cr)| = |(a + cr) - (b + cl)|: the row's 11 bytes as dwords (4 LDS
        // reads per side instead of 11 byte reads: the byte reads made k_stereo_sad LDS-bound),
        // aligned by v_alignbyte, two pixels per v_sad_u16 on u16 lanes (a + cr <= 510: the
        // 32-bit add of (cr, cr) cannot carry between the lanes); byte 11 is not in the row
        const int ls = shlw[dy];
        const int s = shrw[dy] + ST_L + inc;  // right row byte offset, 0 .. 13
        const uint32_t *la = stL + dy * 4, *ra = stR + dy * 7 + (s >> 2);
        uint32_t Lw[4], Rw[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            Lw[k] = la[k];
            Rw[k] = ra[k];
        }
        const uint32_t cr2 = (uint32_t)cr * 0x10001u, cl2 = (uint32_t)cl * 0x10001u;
        uint32_t sacc = 0;
#pragma unroll
        for (int j = 0; j < 3; j++) {
            const uint32_t A = __builtin_amdgcn_alignbyte(Lw[j + 1], Lw[j], ls);
            const uint32_t B = __builtin_amdgcn_alignbyte(Rw[j + 1], Rw[j], s & 3);
            sacc = __builtin_amdgcn_sad_u16(__builtin_amdgcn_perm(A, A, 0x0c010c00u) + cr2,
                                            __builtin_amdgcn_perm(B, B, 0x0c010c00u) + cl2, sacc);
            if (j < 2)
                sacc = __builtin_amdgcn_sad_u16(__builtin_amdgcn_perm(A, A, 0x0c030c02u) + cr2,
                                                __builtin_amdgcn_perm(B, B, 0x0c030c02u) + cl2, sacc);
            else  // byte 10 only
                sacc = __builtin_amdgcn_sad_u16(__builtin_amdgcn_perm(A, A, 0x0c0c0c02u) + (uint32_t)cr,
                                                __builtin_amdgcn_perm(B, B, 0x0c0c0c02u) + (uint32_t)cl, sacc);
        }
        atomicAdd(&sadw[inc + ST_L], (int)sacc);
#else
        const uint8_t *a = bL + dy * 16 + shlw[dy];
        const uint8_t *b = bR + dy * 28 + shrw[dy] + ST_L + inc;
        int s = 0;
#pragma unroll
        for (int dx = 0; dx < 2 * ST_W + 1; dx++) s += abs((a[dx] - cl) - (b[dx] - cr));
        atomicAdd(&sadw[inc + ST_L], s);
#endif
    }
    wave_sync_lds();
    if (lane != 0) return;
    int best = INT_MAX, bestinc = 0;
    for (int inc = -ST_L; inc <= ST_L; inc++) {
        const int s = sadw[inc + ST_L];
        if (s < best) {
            best = s;
            bestinc = inc;
        }
    }
    if (bestinc == -ST_L || bestinc == ST_L) return;
    const float dist1 = (float)sadw[ST_L + bestinc - 1];
    const float dist2 = (float)sadw[ST_L + bestinc];
    const float dist3 = (float)sadw[ST_L + bestinc + 1];
    const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
    if (deltaR < -1 || deltaR > 1) return;
    float bestuR = G.scale[lev] * ((float)scaleduR0 + (float)bestinc + deltaR);
    float disparity = kl.x - bestuR;
    if (disparity >= 0.0f && disparity < G.max_d) {
        if (disparity <= 0) {
            disparity = 0.01f;
            bestuR = (float)((double)kl.x - 0.01);
        }
        dp[iL] = G.bf / disparity;
        ur[iL] = bestuR;
        so[iL] = best;
    }
}

__global__ __launch_bounds__(256) void k_stereo_sad(StereoGeom G,
                                                   const orbg_keypoint *__restrict__ kps,
                                                   const int32_t *__restrict__ counts,
                                                   const int32_t *__restrict__ left,
                                                   const int32_t *__restrict__ right,
                                                   const int32_t *__restrict__ best_r,
                                                   const uint8_t *__restrict__ img0,
                                                   int64_t img_fs, int img_pitch,
                                                   const uint8_t *__restrict__ pyr,
                                                   int64_t pyr_frame, float *__restrict__ uright,
                                                   float *__restrict__ depth,
                                                   int32_t *__restrict__ sad_out)
{
    __shared__ int sad[4][2 * ST_L + 1];
    __shared__ uint32_t stage[4][11 * 4 + 11 * 7];
    __shared__ int shl[4][11], shr[4][11];
    // XCD-aware: a pair's workgroups on one XCD, so the pyramid rows their patches and strips
    // share come into one L2
    const int id = ORBG_ST_XCD ? xcd_remap(blockIdx.x + gridDim.x * blockIdx.y, gridDim.x * gridDim.y)
                               : (int)(blockIdx.x + gridDim.x * blockIdx.y);
    const int p = id / gridDim.x, bx = id - p * gridDim.x;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int fl = left[p], fr = right[p];
    const int nl = counts[fl];
    for (int iL = bx * 4 + wv; iL < nl; iL += ST_SAD_WAVES) {
        stereo_sad_one(G, kps, best_r, img0, img_fs, img_pitch, pyr, pyr_frame, uright, depth,
                       sad_out, p, fl, fr, iL, lane, sad[wv], stage[wv], shl[wv], shr[wv]);
        wave_sync_lds();  // the next keypoint reuses this wave's LDS
    }
}

// Batched form of the same per-keypoint work (ORBG_ST_MG4, default): the kernel is bound by
// each keypoint's chain of dependent loads (vbest_r -> the two keypoints -> the patch and strip
// rows), so a wave runs four keypoints of its sequence at once, 16 lanes each, and pays the
// chain once per four.  Per keypoint: its 33 row words staged by 16 lanes (3 loads per lane),
// then lane i < 11 of the group owns shift inc = i - 5 and sums its 11 rows in registers (no
// LDS atomics), and the first minimum, its neighbours and the parabola are 16-lane shuffles.
// The level table (scales, widths, pitches, offsets) is read from LDS, not from the kernel
// arguments by a dynamic index (a dependent global load per keypoint).
#ifndef ORBG_ST_MG4
#define ORBG_ST_MG4 1
#endif
#define ST_SMG 4  // keypoints per wave

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_stereo_sad_mg(StereoGeom G,
                                                      const orbg_keypoint *__restrict__ kps,
                                                      const int32_t *__restrict__ counts,
                                                      const int32_t *__restrict__ left,
                                                      const int32_t *__restrict__ right,
                                                      const int32_t *__restrict__ best_r,
                                                      const uint8_t *__restrict__ img0,
                                                      int64_t img_fs, int img_pitch,
                                                      const uint8_t *__restrict__ pyr,
                                                      int64_t pyr_frame, float *__restrict__ uright,
                                                      float *__restrict__ depth,
                                                      int32_t *__restrict__ sad_out)
{
    __shared__ uint32_t stage[4][ST_SMG][11 * 4 + 11 * 7];
    __shared__ int shl[4][ST_SMG][11], shr[4][ST_SMG][11];
    __shared__ float t_inv[16], t_scale[16];
    __shared__ int t_lw[16], t_pitch[16];
    __shared__ int64_t t_off[16];
    if (threadIdx.x < 16) {
        const int l = threadIdx.x;
        t_inv[l] = G.inv_scale[l];
        t_scale[l] = G.scale[l];
        t_lw[l] = G.lw[l];
        t_pitch[l] = l == 0 ? img_pitch : G.lpitch[l];
        t_off[l] = l == 0 ? 0 : G.pyr_off[l];
    }
    __syncthreads();
    const int id = ORBG_ST_XCD ? xcd_remap(blockIdx.x + gridDim.x * blockIdx.y, gridDim.x * gridDim.y)
                               : (int)(blockIdx.x + gridDim.x * blockIdx.y);
    const int p = id / gridDim.x, bx = id - p * gridDim.x;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, g = lane >> 4, l16 = lane & 15;
    const int fl = left[p], fr = right[p];
    const int nl = counts[fl];
    const int i0 = bx * 4 + wv;
    float *ur = uright + (size_t)p * G.fc, *dp = depth + (size_t)p * G.fc;
    int32_t *so = sad_out + (size_t)p * G.fc;
    uint32_t *stL = stage[wv][g], *stR = stage[wv][g] + 11 * 4;
    int *shlw = shl[wv][g], *shrw = shr[wv][g];
    const int inc = l16 - ST_L;  // lanes l16 < 11: this shift
    for (int j0 = 0; i0 + j0 * ST_SAD_WAVES < nl; j0 += ST_SMG) {
        const int iL = i0 + (j0 + g) * ST_SAD_WAVES;
        const bool have = iL < nl;
        const int iR = have ? best_r[(size_t)p * G.fc + iL] : -1;
        if (have && l16 == 0) {
            ur[iL] = -1.0f;
            dp[iL] = -1.0f;
            so[iL] = -1;
        }
        bool ok = iR >= 0;
        orbg_keypoint kl{};
        float uR0 = 0.0f;
        if (ok) {
            kl = kps[(size_t)fl * G.fc + iL];
            uR0 = kps[(size_t)fr * G.fc + iR].x;
        }
        const int lev = ok ? kl.octave : 0;
        const float sf = t_inv[lev];
        const float scaleduL = roundf(kl.x * sf);
        const float scaledvL = roundf(kl.y * sf);
        const float scaleduR0 = roundf(uR0 * sf);
        const float iniu = scaleduR0 + ST_L - ST_W;
        const float endu = scaleduR0 + ST_L + ST_W + 1;
        ok = ok && !(iniu < 0 || endu >= t_lw[lev]);
        // rows: word w = l16 + 16 u (u = 0..2, w < 33) = (row w / 3, part w % 3)
        if (ok) {
            const int pitch = t_pitch[lev];
            const uint8_t *IL = (lev == 0 ? img0 + fl * img_fs : pyr + fl * pyr_frame + t_off[lev]);
            const uint8_t *IR = (lev == 0 ? img0 + fr * img_fs : pyr + fr * pyr_frame + t_off[lev]);
            const int yl = (int)scaledvL, xl = (int)scaleduL, xr = (int)scaleduR0;
            uint4 v[3];
            int sh[3];
#pragma unroll
            for (int u = 0; u < 3; u++) {
                const int w = min(l16 + 16 * u, 32);
                const int r = w / 3, c = w - 3 * r;
                const uint8_t *src = c == 0 ? IL + (int64_t)(yl - ST_W + r) * pitch + xl - ST_W
                                            : IR + (int64_t)(yl - ST_W + r) * pitch + xr - 2 * ST_W;
                sh[u] = (int)((uintptr_t)src & 3);
                v[u] = *(const uint4 *)((const uint32_t *)(src - sh[u]) + (c == 2 ? 3 : 0));
            }
#pragma unroll
            for (int u = 0; u < 3; u++) {
                const int w = l16 + 16 * u;
                if (w < 33) {
                    const int r = w / 3, c = w - 3 * r;
                    uint32_t *dst = (c == 0 ? stL + r * 4 : stR + r * 7) + (c == 2 ? 3 : 0);
                    dst[0] = v[u].x;
                    dst[1] = v[u].y;
                    dst[2] = v[u].z;
                    dst[3] = v[u].w;
                    if (c == 0) shlw[r] = sh[u];
                    if (c == 1) shrw[r] = sh[u];
                }
            }
        }
        wave_sync_lds();
        int sad = INT_MAX;
        if (ok && l16 < 2 * ST_L + 1) {
            const uint8_t *bL = (const uint8_t *)stL, *bR = (const uint8_t *)stR;
            const int cl = bL[ST_W * 16 + shlw[ST_W] + ST_W];
            const int cr = bR[ST_W * 28 + shrw[ST_W] + 2 * ST_W + inc];
            const uint32_t cr2 = (uint32_t)cr * 0x10001u, cl2 = (uint32_t)cl * 0x10001u;
            uint32_t sacc = 0;
#pragma unroll 1
            for (int dy = 0; dy < 2 * ST_W + 1; dy++) {
                const int ls = shlw[dy];
                const int s = shrw[dy] + ST_L + inc;
                const uint32_t *la = stL + dy * 4, *ra = stR + dy * 7 + (s >> 2);
                uint32_t Lw[4], Rw[4];
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    Lw[k] = la[k];
                    Rw[k] = ra[k];
                }
#pragma unroll
                for (int j = 0; j < 3; j++) {
                    const uint32_t A = __builtin_amdgcn_alignbyte(Lw[j + 1], Lw[j], ls);
                    const uint32_t B = __builtin_amdgcn_alignbyte(Rw[j + 1], Rw[j], s & 3);
                    sacc = __builtin_amdgcn_sad_u16(__builtin_amdgcn_perm(A, A, 0x0c010c00u) + cr2,
                                                    __builtin_amdgcn_perm(B, B, 0x0c010c00u) + cl2, sacc);
                    if (j < 2)
                        sacc = __builtin_amdgcn_sad_u16(__builtin_amdgcn_perm(A, A, 0x0c030c02u) + cr2,
                                                        __builtin_amdgcn_perm(B, B, 0x0c030c02u) + cl2, sacc);
                    else
                        sacc = __builtin_amdgcn_sad_u16(__builtin_amdgcn_perm(A, A, 0x0c0c0c02u) + (uint32_t)cr,
                                                        __builtin_amdgcn_perm(B, B, 0x0c0c0c02u) + (uint32_t)cl, sacc);
                }
            }
            sad = (int)sacc;
        }
        // first minimum over the group's 11 shifts: (sad, inc) lexicographic, 16-lane butterfly
        int key_s = sad, key_i = l16;
#pragma unroll
        for (int m = 8; m >= 1; m >>= 1) {
            const int os = __shfl_xor(key_s, m, 16), oi = __shfl_xor(key_i, m, 16);
            if (os < key_s || (os == key_s && oi < key_i)) {
                key_s = os;
                key_i = oi;
            }
        }
        const int bestinc = key_i - ST_L;
        const int base = lane & ~15;
        const int d1 = __shfl(sad, base + min(max(key_i - 1, 0), 15)),
                  d3 = __shfl(sad, base + min(key_i + 1, 15));
        if (ok && l16 == 0 && bestinc != -ST_L && bestinc != ST_L) {
            const float dist1 = (float)d1;
            const float dist2 = (float)key_s;
            const float dist3 = (float)d3;
            const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
            if (!(deltaR < -1 || deltaR > 1)) {
                float bestuR = t_scale[lev] * ((float)scaleduR0 + (float)bestinc + deltaR);
                float disparity = kl.x - bestuR;
                if (disparity >= 0.0f && disparity < G.max_d) {
                    if (disparity <= 0) {
                        disparity = 0.01f;
                        bestuR = (float)((double)kl.x - 0.01);
                    }
                    dp[iL] = G.bf / disparity;
                    ur[iL] = bestuR;
                    so[iL] = key_s;
                }
            }
        }
        wave_sync_lds();  // the next batch reuses this wave's LDS
    }
}

// ---- median cut ---------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_stereo_median(StereoGeom G,
                                                      const int32_t *__restrict__ counts,
                                                      const int32_t *__restrict__ left,
                                                      const int32_t *__restrict__ sad_in,
                                                      float *__restrict__ uright,
                                                      float *__restrict__ depth,
                                                      int32_t *__restrict__ nvalid)
{
    __shared__ int hist[256];
    __shared__ int s_n, s_hi, s_k, s_val;
    const int p = blockIdx.x, tid = threadIdx.x;
    const int nl = counts[left[p]];
    const int32_t *sd = sad_in + (size_t)p * G.fc;
    float *ur = uright + (size_t)p * G.fc, *dp = depth + (size_t)p * G.fc;
    // n accepted, then the (n/2)-th smallest SAD: high byte, then low byte
    hist[tid] = 0;
    if (tid == 0) s_n = 0;
    __syncthreads();
    for (int i = tid; i < nl; i += 256) {
        const int s = sd[i];
        if (s >= 0) {
            atomicAdd(&hist[(s >> 8) & 255], 1);
            atomicAdd(&s_n, 1);
        }
    }
    __syncthreads();
    const int n = s_n;
    if (n == 0) {
        if (tid == 0) nvalid[p] = 0;
        return;
    }
    if (tid == 0) {
        int k = n / 2, b = 0;
        while (k >= hist[b]) {
            k -= hist[b];
            b++;
        }
        s_hi = b;
        s_k = k;
    }
    __syncthreads();
    hist[tid] = 0;
    __syncthreads();
    for (int i = tid; i < nl; i += 256) {
        const int s = sd[i];
        if (s >= 0 && ((s >> 8) & 255) == s_hi) atomicAdd(&hist[s & 255], 1);
    }
    __syncthreads();
    if (tid == 0) {
        int k = s_k, b = 0;
        while (k >= hist[b]) {
            k -= hist[b];
            b++;
        }
        s_val = (s_hi << 8) | b;
    }
    __syncthreads();
    const float median = (float)s_val;
    const float thDist = 1.5f * 1.4f * median;
    int kept = 0;
    for (int i = tid; i < nl; i += 256) {
        const int s = sd[i];
        if (s < 0) continue;
        if ((float)s >= thDist) {
            ur[i] = -1.0f;
            dp[i] = -1.0f;
        } else {
            kept++;
        }
    }
    kept = wave_sum(kept);
    __shared__ int ks[4];
    if ((tid & 63) == 0) ks[tid >> 6] = kept;
    __syncthreads();
    if (tid == 0) nvalid[p] = ks[0] + ks[1] + ks[2] + ks[3];
}

// ---- host launcher --------------------------------------------------------------------
int stereo_list_cap(int frame_cap) { return frame_cap * 20; }

size_t stereo_scratch_bytes(int npairs, int frame_cap)
{
    const size_t P = (size_t)(npairs > 0 ? npairs : 1);
    return P * (ST_MAX_ROWS + 1) * 4 + P * (size_t)stereo_list_cap(frame_cap) * 2 + 256 +
           2 * P * (size_t)frame_cap * 4 + 256;
}

int launch_stereo(hipStream_t st, const OrbgGeom &g, const orbg_keypoint *kps,
                  const uint8_t *desc, const int32_t *counts, const int32_t *d_left,
                  const int32_t *d_right, int npairs, const uint8_t *img0, int64_t img_fs,
                  int img_pitch, const uint8_t *pyr, float bf, float min_z, void *scratch,
                  float *uright, float *depth, int32_t *nvalid, void *prof)
{
    if (g.h > ST_MAX_ROWS || g.frame_cap > 32767) return ORBG_ENOTSUP;
    StereoGeom G{};
    G.h = g.h;
    G.fc = g.frame_cap;
    G.list_cap = stereo_list_cap(g.frame_cap);
    G.bf = bf;
    G.max_d = min_z > 0 ? bf / min_z : __builtin_huge_valf();
    for (int l = 0; l < g.L; l++) {
        G.scale[l] = g.lv[l].scale;
        G.inv_scale[l] = 1.0f / g.lv[l].scale;
        G.lw[l] = g.lv[l].w;
        G.lpitch[l] = g.lv[l].pitch;
        G.pyr_off[l] = g.lv[l].pyr_off;
    }
    uint8_t *s = (uint8_t *)scratch;
    int32_t *row_off = (int32_t *)s;
    s += (size_t)npairs * (ST_MAX_ROWS + 1) * 4;
    int16_t *row_list = (int16_t *)s;
    s += ((size_t)npairs * G.list_cap * 2 + 255) & ~(size_t)255;
    int32_t *best_r = (int32_t *)s;
    s += (size_t)npairs * G.fc * 4;
    int32_t *sad = (int32_t *)s;
    hipEvent_t a = nullptr;
    // fused rows + match: the right frame (keypoints' x / octave, descriptors) and the row
    // lists in LDS, up to 160 KB per workgroup
    const size_t head = st_fused_head(G.h, G.fc);
    int lcap = (int)std::min<size_t>((size_t)G.list_cap,
                                     head < 160 * 1024 - 1024 ? (160 * 1024 - 1024 - head) / 2 : 0);
    // ORBG_ST_FUSED=0|1 (default ORBG_ST_FUSED); ORBG_ST_LCAP (tests): a smaller LDS list, so
    // pairs take the fused kernel's global-list path
    const char *ef = getenv("ORBG_ST_FUSED"), *el = getenv("ORBG_ST_LCAP");
    const bool fused = (ef ? atoi(ef) != 0 : ORBG_ST_FUSED != 0) && lcap >= 4 * G.fc;
    if (el) lcap = std::max(0, std::min(lcap, atoi(el)));
    if (fused) {
        const size_t lds = head + (size_t)lcap * 2;
        // the attribute is per device: cached per device under a lock (contexts on several
        // devices, or threads, share this function)
        static std::mutex attr_mu;
        static size_t attr[ORBG_ST_MAX_DEV] = {};
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || dev < 0) return ORBG_EIO;
        {
            std::lock_guard<std::mutex> lk(attr_mu);
            if (dev >= ORBG_ST_MAX_DEV || attr[dev] < lds) {
                if (hipFuncSetAttribute((const void *)k_stereo_rows_match,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
                    return ORBG_EIO;
                if (dev < ORBG_ST_MAX_DEV) attr[dev] = lds;
            }
        }
        prof_begin(prof, st, "stereo_match", &a);
        hipLaunchKernelGGL(k_stereo_rows_match, dim3(npairs), dim3(ST_FUSED_T), lds, st, G, kps,
                           desc, counts, d_left, d_right, row_list, lcap, best_r);
        prof_end(prof, st, "stereo_match", a);
    } else {
        prof_begin(prof, st, "stereo_rows", &a);
        hipLaunchKernelGGL(k_stereo_rows, dim3(npairs), dim3(ST_ROWS_T), 0, st, G, kps, counts,
                           d_right, row_off, row_list);
        prof_end(prof, st, "stereo_rows", a);
        prof_begin(prof, st, "stereo_match", &a);
        hipLaunchKernelGGL(k_stereo_match, dim3(ST_MATCH_WAVES / 4, npairs), dim3(256), 0, st, G,
                           kps, desc, counts, d_left, d_right, row_off, row_list, best_r);
        prof_end(prof, st, "stereo_match", a);
    }
    prof_begin(prof, st, "stereo_sad", &a);
    hipLaunchKernelGGL(ORBG_ST_MG4 ? k_stereo_sad_mg : k_stereo_sad,
                       dim3(ST_SAD_WAVES / 4, npairs), dim3(256), 0, st, G, kps, counts, d_left,
                       d_right, best_r, img0, img_fs, img_pitch, pyr, g.pyr_frame, uright, depth,
                       sad);
    prof_end(prof, st, "stereo_sad", a);
    prof_begin(prof, st, "stereo_median", &a);
    hipLaunchKernelGGL(k_stereo_median, dim3(npairs), dim3(256), 0, st, G, counts, d_left, sad,
                       uright, depth, nvalid);
    prof_end(prof, st, "stereo_median", a);
    return hipGetLastError() == hipSuccess ? ORBG_OK : ORBG_EIO;
}

}  // namespace orbg
