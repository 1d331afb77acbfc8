// stereo_kernels.hip -- Frame::ComputeStereoMatches (src/Frame.cc:619-834) on gfx950.
//
// Per stereo pair (left frame, right frame of the last batch), four launches:
//   k_stereo_rows    :637-662  row table (vRowIndices): right keypoint iR is listed in rows
//                              floor(y - r) .. ceil(y + r), r = 2 * scale[octave]; one
//                              workgroup per pair, counts / scan / fill in LDS, the lists go
//                              to global scratch (order inside a row is free: see below)
//   k_stereo_match   :676-738  thread per left keypoint: candidates of row (int)vL, octave
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

#include <climits>

#include "../../include/orbg.h"
#include "orbg_device.h"
#include "orbg_internal.h"

#pragma clang fp contract(off)

namespace orbg {

void prof_begin(void *prof, hipStream_t s, const char *n, hipEvent_t *a);
void prof_end(void *prof, hipStream_t s, const char *n, hipEvent_t a);

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
    const int p = blockIdx.y;
    const int iL = blockIdx.x * 256 + threadIdx.x;
    const int fl = left[p], fr = right[p];
    const int nl = counts[fl];
    if (iL >= nl) return;
    int32_t *out = best_r + (size_t)p * G.fc;
    const orbg_keypoint kl = kps[(size_t)fl * G.fc + iL];
    out[iL] = -1;
    const int row = (int)kl.y;
    if (row < 0 || row >= G.h) return;
    const int32_t *off = row_off + (size_t)p * (ST_MAX_ROWS + 1);
    const int c0 = off[row], c1 = min(off[row + 1], G.list_cap);
    if (c0 >= c1) return;
    const float minU = kl.x - G.max_d, maxU = kl.x - 0.0f;
    if (maxU < 0) return;
    const uint32_t *ql = (const uint32_t *)(desc + ((size_t)fl * G.fc + iL) * 32);
    uint32_t qd[8];
#pragma unroll
    for (int i = 0; i < 8; i++) qd[i] = ql[i];
    const orbg_keypoint *kr = kps + (size_t)fr * G.fc;
    const uint8_t *dr = desc + (size_t)fr * G.fc * 32;
    const int16_t *list = row_list + (size_t)p * G.list_cap;
    int bestDist = ST_TH_HIGH, bestIdx = INT_MAX;
    for (int c = c0; c < c1; c++) {
        const int iR = list[c];
        const orbg_keypoint k = kr[iR];
        if (k.octave < kl.octave - 1 || k.octave > kl.octave + 1) continue;
        if (!(k.x >= minU && k.x <= maxU)) continue;
        const uint32_t *d = (const uint32_t *)(dr + (size_t)iR * 32);
        int dist = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) dist += __popc(qd[i] ^ d[i]);
        if (dist < bestDist || (dist == bestDist && iR < bestIdx && dist < ST_TH_HIGH)) {
            bestDist = dist;
            bestIdx = iR;
        }
    }
    if (bestDist < ST_TH_ORB) out[iL] = bestIdx;
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
    const int p = blockIdx.y;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int iL = blockIdx.x * 4 + wv;
    const int fl = left[p], fr = right[p];
    const int nl = counts[fl];
    if (iL >= nl) return;  // wave-uniform
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
    const int cl = IL[(int64_t)yl * lp + xl];
    if (lane < 2 * ST_L + 1) sad[wv][lane] = 0;
    wave_sync_lds();
    // items t = (shift, row): 11 x 11, two per lane
    for (int t = lane; t < (2 * ST_L + 1) * (2 * ST_W + 1); t += 64) {
        const int inc = t / (2 * ST_W + 1) - ST_L, dy = t % (2 * ST_W + 1) - ST_W;
        const int cr = IR[(int64_t)yl * rp + xr + inc];
        const uint8_t *a = IL + (int64_t)(yl + dy) * lp + xl - ST_W;
        const uint8_t *b = IR + (int64_t)(yl + dy) * rp + xr + inc - ST_W;
        int s = 0;
#pragma unroll
        for (int dx = 0; dx < 2 * ST_W + 1; dx++) s += abs((a[dx] - cl) - (b[dx] - cr));
        atomicAdd(&sad[wv][inc + ST_L], s);
    }
    wave_sync_lds();
    if (lane != 0) return;
    int best = INT_MAX, bestinc = 0;
    for (int inc = -ST_L; inc <= ST_L; inc++) {
        const int s = sad[wv][inc + ST_L];
        if (s < best) {
            best = s;
            bestinc = inc;
        }
    }
    if (bestinc == -ST_L || bestinc == ST_L) return;
    const float dist1 = (float)sad[wv][ST_L + bestinc - 1];
    const float dist2 = (float)sad[wv][ST_L + bestinc];
    const float dist3 = (float)sad[wv][ST_L + bestinc + 1];
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
    prof_begin(prof, st, "stereo", &a);
    hipLaunchKernelGGL(k_stereo_rows, dim3(npairs), dim3(ST_ROWS_T), 0, st, G, kps, counts,
                       d_right, row_off, row_list);
    hipLaunchKernelGGL(k_stereo_match, dim3((G.fc + 255) / 256, npairs), dim3(256), 0, st, G, kps,
                       desc, counts, d_left, d_right, row_off, row_list, best_r);
    hipLaunchKernelGGL(k_stereo_sad, dim3((G.fc + 3) / 4, npairs), dim3(256), 0, st, G, kps,
                       counts, d_left, d_right, best_r, img0, img_fs, img_pitch, pyr,
                       g.pyr_frame, uright, depth, sad);
    hipLaunchKernelGGL(k_stereo_median, dim3(npairs), dim3(256), 0, st, G, counts, d_left, sad,
                       uright, depth, nvalid);
    prof_end(prof, st, "stereo", a);
    return hipGetLastError() == hipSuccess ? ORBG_OK : ORBG_EIO;
}

}  // namespace orbg
