// frame_kernels.hip -- the per-frame / per-MapPoint geometry around the matchers, gfx950:
//
//   k_undistort     Frame::UndistortKeyPoints (src/Frame.cc:542-572): cv::undistortPoints of
//                   every keypoint of a batch of frames, one thread per keypoint, double
//                   arithmetic (frame_device.h); the record is copied with x, y replaced.
//   k_frustum       Frame::isInFrustum (src/Frame.cc:342-409) for the local map points of a
//                   batch of frames (Tracking::SearchLocalPoints, Tracking.cc:1676-1691), one
//                   thread per (frame, map point); writes the mTrack* members as the
//                   orbg_map_projection records SearchByProjection(F, vpMapPoints) reads
//                   (k_track_cands<LOCAL>, track_kernels.hip).
//   k_distinctive   MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:342-420), one
//                   wave per map point: lane j holds observation j's descriptor; row i of the
//                   distance matrix is one Hamming distance per lane (row i's descriptor
//                   broadcast through scalar registers), its median the k-th smallest across
//                   the lanes by a 9-step binary search over [0, 256] with ballot counts (no
//                   LDS, no sort); the least median wins, the first row on ties.  Up to 32
//                   observations the wave splits into 16- or 32-lane groups that each hold
//                   every observation and take one row per iteration (four or two rows at
//                   once, the search on the group's ballot bits).
//
// Float / double pins as the oracle (oracle/frame_oracle.c): cv::gemm's small-matrix path
// with a double work type for Rcw*P+tcw and -Rcw.t()*tcw, cv::norm / Mat::dot in double,
// PredictScale's log in double; no FMA contraction.
#include <hip/hip_runtime.h>

#include "../../include/orbg.h"
#include "frame_device.h"
#include "orbg_device.h"
#include "orbg_internal.h"

#pragma clang fp contract(off)

namespace orbg {

// ---------------------------------------------------------------------------
// UndistortKeyPoints
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_undistort(const orbg_keypoint *__restrict__ kps,
                                                   const int32_t *__restrict__ counts, int fc,
                                                   orbg_camera cam,
                                                   orbg_keypoint *__restrict__ out)
{
    const int f = blockIdx.y;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= counts[f]) return;
    const size_t o = (size_t)f * fc + i;
    orbg_keypoint kp = kps[o];
    if (cam.k1 != 0.0f) undistort_point(cam, kp.x, kp.y, &kp.x, &kp.y);  // Frame.cc:544-548
    out[o] = kp;
}

int launch_undistort(hipStream_t st, const orbg_camera &cam, const orbg_keypoint *kps,
                     const int32_t *counts, int fc, int nframes, orbg_keypoint *out)
{
    if (nframes <= 0 || fc <= 0) return 0;
    hipLaunchKernelGGL(k_undistort, dim3((fc + 255) / 256, nframes), dim3(256), 0, st, kps,
                       counts, fc, cam, out);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

// ---------------------------------------------------------------------------
// ComputeStereoFromRGBD
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_rgbd(const uint8_t *__restrict__ depth, int u16,
                                              int scale, float factor, int w, int h,
                                              size_t pitch, size_t istride,
                                              const orbg_keypoint *__restrict__ kps,
                                              const orbg_keypoint *__restrict__ kps_un,
                                              const int32_t *__restrict__ counts, int fc, float mbf,
                                              float *__restrict__ uright, float *__restrict__ dout)
{
    const int f = blockIdx.y;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= counts[f]) return;
    const size_t o = (size_t)f * fc + i;
    const orbg_keypoint kp = kps[o];
    // imDepth.at<float>(v, u): the float position truncated to int
    const int u = (int)kp.x, v = (int)kp.y;
    float d = -1.0f;
    if (u >= 0 && u < w && v >= 0 && v < h) {
        const uint8_t *row = depth + (size_t)f * istride + (size_t)v * pitch;
        const float raw = u16 ? (float)((const uint16_t *)row)[u] : ((const float *)row)[u];
        d = scale ? raw * factor : raw;
    }
    float ur = -1.0f, dd = -1.0f;
    if (d > 0) {  // Frame.cc:851-855
        dd = d;
        ur = kps_un[o].x - mbf / d;
    }
    uright[o] = ur;
    dout[o] = dd;
}

int launch_rgbd(hipStream_t st, const void *depth, int u16, float factor, int w, int h,
                size_t pitch, size_t istride, const orbg_keypoint *kps,
                const orbg_keypoint *kps_un, const int32_t *counts, int fc, int nframes,
                float mbf, float *uright, float *dout)
{
    if (nframes <= 0 || fc <= 0) return 0;
    // Tracking.cc:233-234: converted (x * factor) unless already float with factor ~ 1
    const int scale = u16 || (double)fabsf(factor - 1.0f) > 1e-5;
    hipLaunchKernelGGL(k_rgbd, dim3((fc + 255) / 256, nframes), dim3(256), 0, st,
                       (const uint8_t *)depth, u16, scale, factor, w, h, pitch, istride, kps,
                       kps_un, counts, fc, mbf, uright, dout);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

// ---------------------------------------------------------------------------
// isInFrustum
// ---------------------------------------------------------------------------
// cv::gemm small-matrix pin (oracle orc_gemm3): (float)(alpha * op(R) x + c), double work
__device__ __forceinline__ float gemm_row(const float *T, int r, bool trans, const float x[3],
                                          double alpha, double c)
{
    double t = 0.0;
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const float a = trans ? T[4 * k + r] : T[4 * r + k];
        t += (double)a * (double)x[k];
    }
    t *= alpha;
    t += c;
    return (float)t;
}

__global__ __launch_bounds__(256) void k_frustum(const orbg_frustum_camera *__restrict__ cams,
                                                 const orbg_map_point *__restrict__ mps,
                                                 const int32_t *__restrict__ counts, int cap,
                                                 float cos_limit,
                                                 orbg_map_projection *__restrict__ out,
                                                 int32_t *__restrict__ nvisible)
{
    const int f = blockIdx.y;
    const int i = blockIdx.x * 256 + threadIdx.x;
    const int n = counts[f];
    // mOw = -mRcw.t()*mtcw (Frame::UpdatePoseMatrices, Frame.cc:334; gemm, alpha -1): once
    // per workgroup (it is the frame's), not per point
    __shared__ float sOw[3];
    if (threadIdx.x < 3) {
        const orbg_frustum_camera &C = cams[f];
        const int r = threadIdx.x;
        double t = 0.0;
#pragma unroll
        for (int k = 0; k < 3; k++) t += (double)C.Tcw[4 * k + r] * (double)C.Tcw[4 * k + 3];
        sOw[r] = (float)(t * -1.0);
    }
    __syncthreads();
    bool vis = false;
    if (i < n) {
        const orbg_frustum_camera &C = cams[f];
        const orbg_map_point mp = mps[(size_t)f * cap + i];
        orbg_map_projection o;
        o.flags = mp.flags & ORBG_MP_HAS_OBS;  // mbTrackInView = false
        if (mp.flags & ORBG_MP_VALID) {
            const float P[3] = {mp.x, mp.y, mp.z};
            const float tcw[3] = {C.Tcw[3], C.Tcw[7], C.Tcw[11]};
            const float PcX = gemm_row(C.Tcw, 0, false, P, 1.0, (double)tcw[0]);
            const float PcY = gemm_row(C.Tcw, 1, false, P, 1.0, (double)tcw[1]);
            const float PcZ = gemm_row(C.Tcw, 2, false, P, 1.0, (double)tcw[2]);
            do {
                if (PcZ < 0.0f) break;
                const float invz = 1.0f / PcZ;
                const float u = C.fx * PcX * invz + C.cx;
                const float v = C.fy * PcY * invz + C.cy;
                if (u < C.bounds.min_x || u > C.bounds.max_x) break;
                if (v < C.bounds.min_y || v > C.bounds.max_y) break;
                const float maxDistance = 1.2f * mp.max_dist;
                const float minDistance = 0.8f * mp.min_dist;
                const float Ow[3] = {sOw[0], sOw[1], sOw[2]};
                const float PO0 = P[0] - Ow[0], PO1 = P[1] - Ow[1], PO2 = P[2] - Ow[2];
                double s = 0.0;
                s += (double)PO0 * (double)PO0;
                s += (double)PO1 * (double)PO1;
                s += (double)PO2 * (double)PO2;
                const float dist = (float)sqrt(s);
                if (dist < minDistance || dist > maxDistance) break;
                double dot = 0.0;
                dot += (double)PO0 * (double)mp.nx;
                dot += (double)PO1 * (double)mp.ny;
                dot += (double)PO2 * (double)mp.nz;
                const float viewCos = (float)(dot / (double)dist);
                if (viewCos < cos_limit) break;
                const int ns = predict_scale(mp.max_dist, dist, C.log_scale_factor, C.nlevels);
                o.flags |= ORBG_MP_VALID;
                o.u = u;
                o.ur = u - C.bf * invz;
                o.v = v;
                o.level = ns;
                o.view_cos = viewCos;
                vis = true;
            } while (0);
        }
        if (vis)
            out[(size_t)f * cap + i] = o;
        else  // only the flags: the other mTrack* members keep their values (Frame.cc:350)
            out[(size_t)f * cap + i].flags = o.flags;
    }
    // per-frame count: one atomic per wave
    const unsigned long long m = __ballot(vis);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(&nvisible[f], (int)__popcll(m));
}

int launch_frustum(hipStream_t st, const orbg_frustum_camera *cams, const orbg_map_point *mps,
                   const int32_t *counts, int cap, int nframes, float cos_limit,
                   orbg_map_projection *out, int32_t *nvisible)
{
    if (nframes <= 0 || cap <= 0) return 0;
    if (hipMemsetAsync(nvisible, 0, (size_t)nframes * 4, st) != hipSuccess) return -5;
    hipLaunchKernelGGL(k_frustum, dim3((cap + 255) / 256, nframes), dim3(256), 0, st, cams, mps,
                       counts, cap, cos_limit, out, nvisible);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

// ---------------------------------------------------------------------------
// ComputeDistinctiveDescriptors
// ---------------------------------------------------------------------------
#define DD_WAVES 4
#ifndef ORBG_DD_GROUPS
#define ORBG_DD_GROUPS 1  // N <= 32: 16- / 32-lane groups, two or four rows per iteration (0: a row per iteration)
#endif
#define DD_CHUNKS 8  // observations kept as per-lane distances per row: 512

__device__ __forceinline__ void load_desc(const uint8_t *__restrict__ pool, int row, uint32_t d[8])
{
    const uint4 *p = (const uint4 *)(pool + (size_t)row * 32);
    const uint4 a = p[0], b = p[1];
    d[0] = a.x; d[1] = a.y; d[2] = a.z; d[3] = a.w;
    d[4] = b.x; d[5] = b.y; d[6] = b.z; d[7] = b.w;
}

__global__ __launch_bounds__(64 * DD_WAVES) void k_distinctive(
    const uint8_t *__restrict__ pool, const int32_t *__restrict__ rows,
    const int32_t *__restrict__ off, int npoints, int32_t *__restrict__ best_out,
    uint8_t *__restrict__ desc_out)
{
    const int lane = threadIdx.x & 63;
    const int p = blockIdx.x * DD_WAVES + (threadIdx.x >> 6);
    if (p >= npoints) return;  // wave-uniform
    const int o0 = off[p];
    const int N = off[p + 1] - o0;
    if (N <= 0) {  // no observation: the reference returns, mDescriptor untouched
        if (lane == 0) best_out[p] = -1;
        return;
    }
    const int32_t *R = rows + o0;
    const int k = (N - 1) >> 1;  // vDists[0.5*(N-1)]: (size_t)(0.5 * (N - 1)) = (N - 1) / 2
#if ORBG_DD_GROUPS
    if (N <= 32) {
        // G-lane groups (G = 16 or 32), one row per group: every group holds all N
        // observations (lane l: observation l % G), group g takes row i0 + g of each
        // iteration, its median by the ballot search restricted to the group's bits
        const int G = N <= 16 ? 16 : 32, R_ = 64 / G;
        const int g = lane / G, j = lane - g * G;
        uint32_t mine[8];
        if (j < N) load_desc(pool, R[j], mine);
        else
#pragma unroll
            for (int w = 0; w < 8; w++) mine[w] = 0;
        const unsigned long long gmask = (G == 64 ? ~0ull : ((1ull << G) - 1ull)) << (g * G);
        int best_median = 0x7fffffff, best = 0;
        for (int i0 = 0; i0 < N; i0 += R_) {
            const int r = i0 + g;  // this group's row (past N: a dead row, not compared)
            const int src = g * G + min(r, N - 1);
            uint32_t q[8];
#pragma unroll
            for (int w = 0; w < 8; w++) q[w] = (uint32_t)__shfl((int)mine[w], src, 64);
            int d = 0x7fff;
            if (j < N) {
                d = 0;
#pragma unroll
                for (int w = 0; w < 8; w++) d += __popc(q[w] ^ mine[w]);
            }
            int lo = 0, hi = 256;  // group-uniform
#pragma unroll
            for (int it = 0; it < 9; it++) {
                const int mid = (lo + hi) >> 1;
                const int cnt = __popcll(__ballot(d <= mid) & gmask);
                const bool up = cnt >= k + 1;
                hi = up ? mid : hi;
                lo = up ? lo : mid + 1;
            }
            // rows i0 .. i0 + R_ - 1 in order: strict <, the first row wins ties
            for (int gg = 0; gg < R_; gg++) {
                const int rr = i0 + gg;
                if (rr >= N) break;
                const int m = __builtin_amdgcn_readlane(lo, gg * G);
                if (m < best_median) {
                    best_median = m;
                    best = rr;
                }
            }
        }
        if (lane == 0) best_out[p] = best;
        if (desc_out && lane < 2) {
            const int rb = R[best];
            ((uint4 *)(desc_out + (size_t)p * 32))[lane] = ((const uint4 *)(pool + (size_t)rb * 32))[lane];
        }
        return;
    }
#endif
    // observations 0..63 register-resident, one per lane
    uint32_t mine[8];
    if (lane < N) load_desc(pool, R[lane], mine);
    else
#pragma unroll
        for (int w = 0; w < 8; w++) mine[w] = 0;
    int best_median = 0x7fffffff, best = 0;
    for (int i = 0; i < N; i++) {
        // row i's descriptor, wave-uniform (scalar registers)
        uint32_t qi[8];
        if (i < 64) {
#pragma unroll
            for (int w = 0; w < 8; w++) qi[w] = (uint32_t)__builtin_amdgcn_readlane((int)mine[w], i);
        } else {
            const int ri = __builtin_amdgcn_readfirstlane(R[i]);
            load_desc(pool, ri, qi);
#pragma unroll
            for (int w = 0; w < 8; w++) qi[w] = (uint32_t)__builtin_amdgcn_readfirstlane((int)qi[w]);
        }
        // d_ij per lane for j = lane + 64 c; past N: 0x7fff (never <= a candidate median)
        int dc[DD_CHUNKS];
#pragma unroll
        for (int c = 0; c < DD_CHUNKS; c++) {
            dc[c] = 0x7fff;
            const int j = c * 64 + lane;
            if (c * 64 < N && j < N) {
                uint32_t dj[8];
                if (c == 0) {
#pragma unroll
                    for (int w = 0; w < 8; w++) dj[w] = mine[w];
                } else {
                    load_desc(pool, R[j], dj);
                }
                int d = 0;
#pragma unroll
                for (int w = 0; w < 8; w++) d += __popc(qi[w] ^ dj[w]);
                dc[c] = d;
            }
        }
        // the median: the smallest v with #{j : d_ij <= v} >= k + 1 (a 9-step search)
        int lo = 0, hi = 256;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            int cnt = 0;
#pragma unroll
            for (int c = 0; c < DD_CHUNKS; c++)
                if (c * 64 < N) cnt += __popcll(__ballot(dc[c] <= mid));
            // observations past DD_CHUNKS * 64 (rare): re-read per step, L2-resident
            for (int c = DD_CHUNKS * 64; c < N; c += 64) {
                const int j = c + lane;
                bool le = false;
                if (j < N) {
                    uint32_t dj[8];
                    load_desc(pool, R[j], dj);
                    int d = 0;
#pragma unroll
                    for (int w = 0; w < 8; w++) d += __popc(qi[w] ^ dj[w]);
                    le = d <= mid;
                }
                cnt += __popcll(__ballot(le));
            }
            if (cnt >= k + 1)
                hi = mid;
            else
                lo = mid + 1;
        }
        if (lo < best_median) {  // strict <: the first row wins ties
            best_median = lo;
            best = i;
        }
    }
    if (lane == 0) best_out[p] = best;
    if (desc_out && lane < 2) {
        const int rb = R[best];
        ((uint4 *)(desc_out + (size_t)p * 32))[lane] = ((const uint4 *)(pool + (size_t)rb * 32))[lane];
    }
}

int launch_distinctive(hipStream_t st, const uint8_t *pool, const int32_t *rows,
                       const int32_t *off, int npoints, int32_t *best, uint8_t *desc_out)
{
    if (npoints <= 0) return 0;
    hipLaunchKernelGGL(k_distinctive, dim3((npoints + DD_WAVES - 1) / DD_WAVES),
                       dim3(64 * DD_WAVES), 0, st, pool, rows, off, npoints, best, desc_out);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

}  // namespace orbg
