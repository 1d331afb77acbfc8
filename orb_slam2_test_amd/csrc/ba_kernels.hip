// ba_kernels.hip -- per-edge arithmetic of Optimizer::LocalBundleAdjustment on gfx950.
//
// k_ba_edges: one thread per point over its edges, fp64 throughout (world coordinates reach
// hundreds of metres on KITTI; obs - proj cancels, SURVEY.md 7 hard part 5):
//   EdgeSE3ProjectXYZ / EdgeStereoSE3ProjectXYZ::computeError  types_six_dof_expmap.h:90-95,122-127
//   cam_project (stereo: float invz, float bf)                 types_six_dof_expmap.cpp:141-157
//   linearizeOplus                                             types_six_dof_expmap.cpp:103-139,188-234
//   chi2, Huber rho' (float dsqr)                              base_edge.h:58-61, robust_kernel_impl.cpp:65-91
//   constructQuadraticForm: H_pp += A^T W A, b_p += A^T w_r,   base_binary_edge.hpp:55-120
//       H_ll += B^T W B, b_l += B^T w_r, H_pl = A^T W B
// Point blocks are summed per point over its edge list in k_ba_edges itself (no atomics);
// pose blocks by k_ba_pose_mfma (MFMA f64 over slices of each pose's edges, rows recomputed).
#include <hip/hip_runtime.h>

#include <cstring>

#include "../../include/orbg.h"
#include "orbg_internal.h"

namespace orbg {

void prof_begin(void *prof, hipStream_t s, const char *n, hipEvent_t *a);
void prof_end(void *prof, hipStream_t s, const char *n, hipEvent_t a);

// LDS written by some lanes of a wave, then read by others (the hardware keeps one wave's
// LDS ops in order; the fence keeps the compiler from reordering them)
__device__ __forceinline__ void wave_sync_lds_ba()
{
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ void quat_rotate(const double q[4], const double v[3], double o[3])
{
    double uv[3] = {q[1] * v[2] - q[2] * v[1], q[2] * v[0] - q[0] * v[2],
                    q[0] * v[1] - q[1] * v[0]};
    uv[0] += uv[0];
    uv[1] += uv[1];
    uv[2] += uv[2];
    o[0] = v[0] + q[3] * uv[0] + (q[1] * uv[2] - q[2] * uv[1]);
    o[1] = v[1] + q[3] * uv[1] + (q[2] * uv[0] - q[0] * uv[2]);
    o[2] = v[2] + q[3] * uv[2] + (q[0] * uv[1] - q[1] * uv[0]);
}

// computeError (types_six_dof_expmap.h:90-95, 122-127): Xc = q X + t, then the mono
// projection in double, or the stereo cam_project with its float invz and float bf
// (types_six_dof_expmap.cpp:150-157); err[2] = 0 for a mono edge
__device__ __forceinline__ void ba_edge_error(const orbg_pose &P, const double X[3],
                                              const orbg_edge &e, double xc[3], double err[3])
{
    quat_rotate(P.q, X, xc);
    xc[0] += P.t[0];
    xc[1] += P.t[1];
    xc[2] += P.t[2];
    const double x = xc[0], y = xc[1], z = xc[2];
    err[2] = 0;
    if (!e.stereo) {
        err[0] = e.obs[0] - ((x / z) * e.fx + e.cx);
        err[1] = e.obs[1] - ((y / z) * e.fy + e.cy);
    } else {
        const float invz = (float)(1.0f / z);
        const float bf = (float)e.bf;
        const double u = x * invz * e.fx + e.cx;
        const double v = y * invz * e.fy + e.cy;
        err[0] = e.obs[0] - u;
        err[1] = e.obs[1] - v;
        err[2] = e.obs[2] - (u - (double)(bf * invz));
    }
}

// ---------------------------------------------------------------------------
// Edge sources: the kernels read an edge as an orbg_edge value, either from the ABI's
// 104-byte records or from an orbg_ba_graph's 24-byte packed edges, whose camera and
// (information, Huber delta) values sit in small deduplicated tables (an ORB-SLAM2 window has
// one camera and one pair per octave and edge type; the observations are float keypoint
// coordinates, exact in f32).  Same doubles either way, so the same bits out.
// ---------------------------------------------------------------------------
struct BaEdgeRecords {
    const orbg_edge *e;
    __device__ __forceinline__ orbg_edge operator()(int i) const { return e[i]; }
};
struct BaEdgePacked {
    const BaPackedEdge *e;
    const BaCam *cam;
    const BaInfo *info;
    __device__ __forceinline__ orbg_edge operator()(int i) const
    {
        const BaPackedEdge p = e[i];
        orbg_edge r;
        r.point = p.point;
        r.pose = p.pose;
        r.stereo = (int)(p.flags & 1u);
        r.robust = (int)((p.flags >> 1) & 1u);
        r.active = (int)((p.flags >> 2) & 1u);
        r.pad = 0;
        r.obs[0] = (double)p.obs[0];
        r.obs[1] = (double)p.obs[1];
        r.obs[2] = (double)p.obs[2];
        const BaCam c = cam[(p.flags >> 8) & 0xFFu];
        r.fx = c.fx;
        r.fy = c.fy;
        r.cx = c.cx;
        r.cy = c.cy;
        r.bf = c.bf;
        const BaInfo f = info[p.flags >> 16];
        r.inv_sigma2 = f.inv_sigma2;
        r.huber_delta = f.huber_delta;
        return r;
    }
};

// ---------------------------------------------------------------------------
// k_ba_errors: g2o's per-trial error pass (SparseOptimizer::computeActiveErrors,
// sparse_optimizer.cpp:61-76) and the terms activeRobustChi2 sums (:100-114): thread per
// edge, every edge given (active or not); err / rho0 / depth_ok may be NULL.
//   chi2 = e^T Omega e (base_edge.h:58-61), rho0 = RobustKernelHuber::robustify's rho[0]
//   with its float dsqr (robust_kernel_impl.cpp:78-91) or chi2 without a kernel,
//   depth_ok = isDepthPositive (types_six_dof_expmap.h:97-101, 129-133).
// 28 B out per edge (err as f64 x 3 only on request).
// ---------------------------------------------------------------------------
template <class ES>
__global__ __launch_bounds__(256) void k_ba_errors(const orbg_pose *__restrict__ poses,
                                                   const double *__restrict__ points,
                                                   const ES edges, int nedge,
                                                   double *__restrict__ err_out,
                                                   double *__restrict__ chi2_out,
                                                   double *__restrict__ rho0_out,
                                                   uint8_t *__restrict__ depth_ok)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nedge) return;
    const orbg_edge e = edges(i);
    const int ip = e.pose, iq = e.point;
    const orbg_pose P = poses[ip];
    const double X[3] = {points[3 * iq], points[3 * iq + 1], points[3 * iq + 2]};
    double xc[3], err[3];
    ba_edge_error(P, X, e, xc, err);
    const double info = e.inv_sigma2;
    double chi2 = 0;
#pragma unroll
    for (int k = 0; k < 3; k++) chi2 += err[k] * (info * err[k]);  // mono: + exact 0
    double rho0 = chi2;
    if (e.robust) {
        const float dsqr = (float)(e.huber_delta * e.huber_delta);
        if (!(chi2 <= dsqr)) rho0 = 2 * sqrt(chi2) * e.huber_delta - dsqr;
    }
    chi2_out[i] = chi2;
    if (rho0_out) rho0_out[i] = rho0;
    if (depth_ok) depth_ok[i] = xc[2] > 0.0;
    if (err_out)
#pragma unroll
        for (int k = 0; k < 3; k++) err_out[3 * (size_t)i + k] = err[k];
}

template <class ES>
static int launch_ba_errors_t(hipStream_t st, const orbg_pose *poses, const double *points,
                              ES edges, int nedge, double *err, double *chi2, double *rho0,
                              uint8_t *depth_ok, void *prof)
{
    if (nedge <= 0) return 0;
    hipEvent_t a = nullptr;
    prof_begin(prof, st, "ba_errors", &a);
    hipLaunchKernelGGL(k_ba_errors<ES>, dim3((nedge + 255) / 256), dim3(256), 0, st, poses,
                       points, edges, nedge, err, chi2, rho0, depth_ok);
    prof_end(prof, st, "ba_errors", a);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

int launch_ba_errors(hipStream_t st, const orbg_pose *poses, const double *points,
                     const orbg_edge *edges, int nedge, double *err, double *chi2, double *rho0,
                     uint8_t *depth_ok, void *prof)
{
    return launch_ba_errors_t(st, poses, points, BaEdgeRecords{edges}, nedge, err, chi2, rho0,
                              depth_ok, prof);
}

int launch_ba_errors_packed(hipStream_t st, const orbg_pose *poses, const double *points,
                            const BaPackedEdge *edges, const BaCam *cam, const BaInfo *info,
                            int nedge, double *err, double *chi2, double *rho0,
                            uint8_t *depth_ok, void *prof)
{
    return launch_ba_errors_t(st, poses, points, BaEdgePacked{edges, cam, info}, nedge, err,
                              chi2, rho0, depth_ok, prof);
}

// ---------------------------------------------------------------------------
// The linearisation of one edge (linearizeOplus types_six_dof_expmap.cpp:103-139 / 188-234,
// chi2 + Huber rho' base_edge.h:58-61, robust_kernel_impl.cpp:78-91), everything in
// registers; the third row of a mono edge is zero (adding it adds exact zeros, so the fixed
// 3-row loops give the same bits as the oracle's 2-row ones).
// ---------------------------------------------------------------------------
#ifndef ORBG_BA_JT_RCP
#define ORBG_BA_JT_RCP 1  // pose Jacobian by reciprocals (0: g2o's divisions, round 4)
#endif
struct BaLin {
    double err[3], jp[3][3], jt[3][6], chi2, rho1, w, info;
    int D;
};

__device__ __forceinline__ void ba_linearize_edge(const orbg_pose &P, const double X[3],
                                                  const orbg_edge &e, BaLin &L)
{
    double xc[3];
    ba_edge_error(P, X, e, xc, L.err);
    const double x = xc[0], y = xc[1], z = xc[2], z_2 = z * z;
    const double fx = e.fx, fy = e.fy;
    L.D = e.stereo ? 3 : 2;
    // rotation matrix (Eigen toRotationMatrix)
    const double *q = P.q;
    const double tx = 2 * q[0], ty = 2 * q[1], tz = 2 * q[2];
    const double twx = tx * q[3], twy = ty * q[3], twz = tz * q[3];
    const double txx = tx * q[0], txy = ty * q[0], txz = tz * q[0];
    const double tyy = ty * q[1], tyz = tz * q[1], tzz = tz * q[2];
    const double R[3][3] = {{1 - (tyy + tzz), txy - twz, txz + twy},
                            {txy + twz, 1 - (txx + tzz), tyz - twx},
                            {txz - twy, tyz + twx, 1 - (txx + tyy)}};
    if (!e.stereo) {
        const double t02 = -x / z * fx, t12 = -y / z * fy;
#pragma unroll
        for (int c = 0; c < 3; c++) {
            L.jp[0][c] = -1. / z * (fx * R[0][c] + t02 * R[2][c]);
            L.jp[1][c] = -1. / z * (fy * R[1][c] + t12 * R[2][c]);
            L.jp[2][c] = 0;
        }
    } else {
#pragma unroll
        for (int c = 0; c < 3; c++) {
            L.jp[0][c] = -fx * R[0][c] / z + fx * x * R[2][c] / z_2;
            L.jp[1][c] = -fy * R[1][c] / z + fy * y * R[2][c] / z_2;
            L.jp[2][c] = L.jp[0][c] - e.bf * R[2][c] / z_2;
        }
    }
#if ORBG_BA_JT_RCP
    // the pose Jacobian by two reciprocals and products instead of g2o's twelve divisions:
    // a few ulps from the divided form (tests hold it to 1e-9 relative of the oracle's; the
    // error, the point Jacobian and with it the point blocks keep g2o's exact expressions)
    const double iz = 1. / z, iz2 = 1. / z_2;
    const double xiz = x * iz, yiz = y * iz, xiz2 = x * iz2, yiz2 = y * iz2, xy2 = x * y * iz2;
    L.jt[0][0] = xy2 * fx;
    L.jt[0][1] = -(1 + x * xiz2) * fx;
    L.jt[0][2] = yiz * fx;
    L.jt[0][3] = -iz * fx;
    L.jt[0][4] = 0;
    L.jt[0][5] = xiz2 * fx;
    L.jt[1][0] = (1 + y * yiz2) * fy;
    L.jt[1][1] = -xy2 * fy;
    L.jt[1][2] = -xiz * fy;
    L.jt[1][3] = 0;
    L.jt[1][4] = -iz * fy;
    L.jt[1][5] = yiz2 * fy;
    if (e.stereo) {
        L.jt[2][0] = L.jt[0][0] - e.bf * yiz2;
        L.jt[2][1] = L.jt[0][1] + e.bf * xiz2;
        L.jt[2][2] = L.jt[0][2];
        L.jt[2][3] = L.jt[0][3];
        L.jt[2][4] = 0;
        L.jt[2][5] = L.jt[0][5] - e.bf * iz2;
    } else {
#else
    L.jt[0][0] = x * y / z_2 * fx;
    L.jt[0][1] = -(1 + (x * x / z_2)) * fx;
    L.jt[0][2] = y / z * fx;
    L.jt[0][3] = -1. / z * fx;
    L.jt[0][4] = 0;
    L.jt[0][5] = x / z_2 * fx;
    L.jt[1][0] = (1 + y * y / z_2) * fy;
    L.jt[1][1] = -x * y / z_2 * fy;
    L.jt[1][2] = -x / z * fy;
    L.jt[1][3] = 0;
    L.jt[1][4] = -1. / z * fy;
    L.jt[1][5] = y / z_2 * fy;
    if (e.stereo) {
        L.jt[2][0] = L.jt[0][0] - e.bf * y / z_2;
        L.jt[2][1] = L.jt[0][1] + e.bf * x / z_2;
        L.jt[2][2] = L.jt[0][2];
        L.jt[2][3] = L.jt[0][3];
        L.jt[2][4] = 0;
        L.jt[2][5] = L.jt[0][5] - e.bf / z_2;
    } else {
#endif
#pragma unroll
        for (int c = 0; c < 6; c++) L.jt[2][c] = 0;
    }
    L.info = e.inv_sigma2;
    double chi2 = 0;
#pragma unroll
    for (int k = 0; k < 3; k++) chi2 += L.err[k] * (L.info * L.err[k]);
    double rho1 = 1.0;
    if (e.robust) {
        const float dsqr = (float)(e.huber_delta * e.huber_delta);
        if (!(chi2 <= dsqr)) rho1 = e.huber_delta / sqrt(chi2);
    }
    L.chi2 = chi2;
    L.rho1 = rho1;
    L.w = rho1 * L.info;
}

// an active edge's share of its point block (base_binary_edge.hpp:55-120): c[0..8] =
// J_point^T W J_point row-major, c[9..11] = J_point^T (-rho' Omega e)
__device__ __forceinline__ void ba_point_share(const BaLin &L, double c[12])
{
    double wr[3];
#pragma unroll
    for (int k = 0; k < 3; k++) wr[k] = -L.info * L.err[k] * L.rho1;
#pragma unroll
    for (int r = 0; r < 3; r++) {
        double bs = 0;
#pragma unroll
        for (int k = 0; k < 3; k++) bs += L.jp[k][r] * wr[k];
        c[9 + r] = bs;
#pragma unroll
        for (int cc = 0; cc < 3; cc++) {
            double hs = 0;
#pragma unroll
            for (int k = 0; k < 3; k++) hs += L.jp[k][r] * L.w * L.jp[k][cc];
            c[r * 3 + cc] = hs;
        }
    }
}

// per-edge outputs: field pointers with a stride in doubles per edge (the orbg_edge_out
// records of the ABI, stride 50, or separate arrays); NULL = not stored
struct BaEdgeOut {
    double *err, *chi2, *rho1, *jp, *jt, *hpl;
    int stride;
};

// ---------------------------------------------------------------------------
// k_ba_edges: one thread per SLOT of the point-major edge order (CSR point_off / point_edges,
// a point's edges contiguous in ascending edge index), so every lane linearises exactly one
// edge (no per-lane loop over a point's edges: the wave's lanes do equal work).  Each lane
// writes its edge's H_pl = J_point^T W J_pose (base_binary_edge.hpp:105-117: the block the
// Schur step reads) plus the optional error terms / Jacobians, and stages its share of the
// point block H_ll | b_l in LDS; the lane holding a point's first slot then sums the shares
// in edge order (the oracle's order, same bits) and stores the block.  A point whose slots
// run past the workgroup's 256 is finished by fp64 atomics of the per-workgroup partial sums
// onto the zeroed block (two partials for any point with <= 256 edges: exact in either
// order).  The pose blocks are k_ba_pose_mfma's, which recomputes the pose rows it needs.
// ---------------------------------------------------------------------------
#define BA_EDGES_TPB ORBG_BA_EDGES_TPB

template <class ES, bool GRAPH>
__global__ __launch_bounds__(BA_EDGES_TPB) void k_ba_edges(const orbg_pose *__restrict__ poses,
                                                          const double *__restrict__ points,
                                                          const ES edges,
                                                          int nslot,
                                                          const int32_t *__restrict__ point_off,
                                                          const int32_t *__restrict__ point_edges,
                                                          BaEdgeOut o, double *__restrict__ hpoint,
                                                          double *__restrict__ bpoint)
{
    __shared__ double part[12][BA_EDGES_TPB];  // H_ll row-major (9), b_l (3) per slot
    const int t = threadIdx.x;
    const int base = blockIdx.x * BA_EDGES_TPB;
    const int a = base + t;
    const int bend = min(base + BA_EDGES_TPB, nslot);
    int q = -1;
    {
        double c[12];
#pragma unroll
        for (int k = 0; k < 12; k++) c[k] = 0;
        if (a < nslot) {
            const int ei = point_edges[a];
            const orbg_edge e = edges(ei);
            const size_t ob = (size_t)ei * o.stride;
            q = e.point;
            if (!e.active) {  // setLevel(1): no contribution, outputs zero
                if (o.hpl)
#pragma unroll
                    for (int k = 0; k < 18; k += 2)
                        *(double2 *)(o.hpl + ob + k) = make_double2(0.0, 0.0);
                if (o.err)
#pragma unroll
                    for (int k = 0; k < 3; k++) o.err[ob + k] = 0;
                if (o.chi2) o.chi2[ob] = 0;
                if (o.rho1) o.rho1[ob] = 0;
                if (o.jp)
#pragma unroll
                    for (int k = 0; k < 9; k++) o.jp[ob + k] = 0;
                if (o.jt)
#pragma unroll
                    for (int k = 0; k < 18; k++) o.jt[ob + k] = 0;
            } else {
                const orbg_pose P = poses[e.pose];
                const double X[3] = {points[3 * (size_t)q], points[3 * (size_t)q + 1],
                                     points[3 * (size_t)q + 2]};
                BaLin L;
                ba_linearize_edge(P, X, e, L);
                ba_point_share(L, c);
                if (o.hpl) {
                    double h[18];
#pragma unroll
                    for (int r = 0; r < 3; r++)
#pragma unroll
                        for (int cc = 0; cc < 6; cc++) {
                            double v = 0;
                            if (!P.fixed)
#pragma unroll
                                for (int k = 0; k < 3; k++) v += L.jp[k][r] * L.w * L.jt[k][cc];
                            h[r * 6 + cc] = v;
                        }
#pragma unroll
                    for (int k = 0; k < 18; k += 2)
                        *(double2 *)(o.hpl + ob + k) = make_double2(h[k], h[k + 1]);
                }
                if (o.err)
#pragma unroll
                    for (int k = 0; k < 3; k++) o.err[ob + k] = L.err[k];
                if (o.chi2) o.chi2[ob] = L.chi2;
                if (o.rho1) o.rho1[ob] = L.rho1;
                if (o.jp)
#pragma unroll
                    for (int k = 0; k < 9; k++) o.jp[ob + k] = L.jp[k / 3][k % 3];
                if (o.jt)
#pragma unroll
                    for (int k = 0; k < 18; k++) o.jt[ob + k] = L.jt[k / 6][k % 6];
            }
        }
#pragma unroll
        for (int k = 0; k < 12; k++) part[k][t] = c[k];
    }
    __syncthreads();
    if (a >= nslot) return;
    const int qs = point_off[q], qe = point_off[q + 1];
    if (a != qs && t != 0) return;  // not the first slot of its point in this workgroup
    const int end = min(qe, bend) - base;
    double acc[12];
#pragma unroll
    for (int k = 0; k < 12; k++) acc[k] = 0;
    for (int j = t; j < end; j++)
#pragma unroll
        for (int k = 0; k < 12; k++) acc[k] += part[k][j];
    double *hq = hpoint + 9 * (size_t)q, *bq = bpoint + 3 * (size_t)q;
    if (GRAPH && (qs < base || qe > bend)) return;  // k_ba_special sums it in edge order
    if (qs < base || qe > bend) {  // the point's slots span workgroups: partial sums
#pragma unroll
        for (int k = 0; k < 9; k++) atomicAdd(hq + k, acc[k]);
#pragma unroll
        for (int k = 0; k < 3; k++) atomicAdd(bq + k, acc[9 + k]);
    } else {
#pragma unroll
        for (int k = 0; k < 9; k++) hq[k] = acc[k];
#pragma unroll
        for (int k = 0; k < 3; k++) bq[k] = acc[9 + k];
    }
}

// ---------------------------------------------------------------------------
// k_ba_pose_mfma: one wave per 64-edge slice of one pose's edge list.  Lane l recomputes edge
// l's three pose rows v_r = [J_pose row | -e] (7 wide) and weight w_r = rho' invSigma2 (zero
// rows for the third row of mono edges and for inactive edges) into LDS, then
//     C = sum_r (w_r v_r)^T v_r   gives  H_pp = C[0:6][0:6],  b_p = C[0:6][6]
// (constructQuadraticForm's A^T W A and A^T omega_r, omega_r = -rho' Omega e), accumulated in
// fp64 by v_mfma_f64_16x16x4_f64: each instruction folds 4 rows, A[i][k] = w v[i] and
// B[k][j] = v[j] padded from 7 to 16.  Slices of one pose add by fp64 atomics.  Fixed poses
// get no block (g2o skips them).
// ---------------------------------------------------------------------------
typedef double v4d __attribute__((ext_vector_type(4)));

#define BA_SLICE ORBG_BA_SLICE  // edges per wave
#ifndef ORBG_BA_POSE_WG
#define ORBG_BA_POSE_WG 0  // 1: graph path with a workgroup per pose, no partials / reduce launch (measured slower: 0.100 vs 0.073 + 0.011 ms; r04s_ba_pose_wg_ab.txt)
#endif
#define BA_ROW 8     // doubles per staged pose row: J_pose (6), -e, w

#ifndef ORBG_BA_MFMA4
#define ORBG_BA_MFMA4 1  // v_mfma_f64_4x4x4f64 (0: round 4's v_mfma_f64_16x16x4f64)
#endif

#if ORBG_BA_MFMA4
// v_mfma_f64_4x4x4f64: four independent 4x4 blocks, K = 4, one f64 per lane in each operand
// (measured, tools/microbench/mfma_f64_rate.hip: A[b][i][k] at lane 16k + 4b + i,
// B[b][k][j] at lane 16k + 4b + j, C[b][i][j] at lane 16i + 4b + j).  The 8x8 [H | b | 0]
// tile is the four blocks: block b = 2I + J holds rows 4I + i, columns 4J + j, so 42 of
// the 64 lane results are H_pp | b_p (round 4's 16x16 tile used 42 of 256).  It issues a
// quarter of the 16x16x4 instruction's FLOPs at ~7x its rate (22 vs 154 cycles per
// instruction and SIMD, profiles/r05a_mfma_f64.txt).
typedef double BaAcc;
#else
typedef v4d BaAcc;
#endif

// every (row, column, value) of the slice accumulator a lane holds
template <class F>
__device__ __forceinline__ void ba_acc_entries(const BaAcc &C, int lane, F f)
{
#if ORBG_BA_MFMA4
    const int i = lane >> 4, b = (lane >> 2) & 3, j = lane & 3;
    f(4 * (b >> 1) + i, 4 * (b & 1) + j, C);
#else
    // D layout of v_mfma_f64_16x16x4f64 (measured): lane holds column j = lane % 16 of rows
    // lane / 16 + 4 v, v = 0..3
    const int j = lane & 15;
#pragma unroll
    for (int v = 0; v < 4; v++) f((lane >> 4) + 4 * v, j, C[v]);
#endif
}

#if ORBG_BA_MFMA4
// One 64-edge slice: lane l linearises edge l and stages its D nonzero pose rows (D = 2 mono,
// 3 stereo, 0 inactive: no zero rows) at row offset sum_{l' < l} D_l', each row = J_pose row
// (6), -e, w; rows up to the next multiple of 16 are zeroed.  Then
//     C += sum_r (w_r v_r)^T v_r   (H_pp = C[0:6][0:6], b_p = C[0:6][6])
// by v_mfma_f64_4x4x4f64, four independent accumulators (rows r0 + 4u + k, u = 0..3, added
// in a fixed order at the end: deterministic, the dependent-MFMA latency hidden)
template <class ES>
__device__ __forceinline__ void ba_pose_slice(const orbg_pose &P, const double *__restrict__ points,
                                              const ES &edges,
                                              const int32_t *__restrict__ pose_edges, int e0,
                                              int ne, double *rl, int lane, BaAcc &C)
{
    int nr16;
    {
        double v[3][BA_ROW];
#pragma unroll
        for (int k = 0; k < 3; k++)
#pragma unroll
            for (int c = 0; c < BA_ROW; c++) v[k][c] = 0;
        int D = 0;
        if (lane < ne) {
            const orbg_edge e = edges(pose_edges[e0 + lane]);
            if (e.active) {
                const double X[3] = {points[3 * (size_t)e.point], points[3 * (size_t)e.point + 1],
                                     points[3 * (size_t)e.point + 2]};
                BaLin L;
                ba_linearize_edge(P, X, e, L);
                D = L.D;
#pragma unroll
                for (int k = 0; k < 3; k++) {
#pragma unroll
                    for (int c = 0; c < 6; c++) v[k][c] = L.jt[k][c];
                    v[k][6] = -L.err[k];
                    v[k][7] = L.w;
                }
            }
        }
        const unsigned long long m2 = __ballot(D >= 2), m3 = __ballot(D == 3);
        const int off =
            2 * __builtin_amdgcn_mbcnt_hi((uint32_t)(m2 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m2, 0)) +
            __builtin_amdgcn_mbcnt_hi((uint32_t)(m3 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m3, 0));
        const int nrow = 2 * __popcll(m2) + __popcll(m3);
        nr16 = (nrow + 15) & ~15;
        wave_sync_lds_ba();  // the previous slice's reads of rl are done (in-order LDS)
#pragma unroll
        for (int k = 0; k < 3; k++)
            if (k < D)
#pragma unroll
                for (int c = 0; c < BA_ROW; c += 2)
                    *(double2 *)(rl + (off + k) * BA_ROW + c) = make_double2(v[k][c], v[k][c + 1]);
        if (nrow + lane < nr16)
#pragma unroll
            for (int c = 0; c < BA_ROW; c += 2)
                *(double2 *)(rl + (nrow + lane) * BA_ROW + c) = make_double2(0.0, 0.0);
    }
    wave_sync_lds_ba();
    const int k = lane >> 4, b = (lane >> 2) & 3, t = lane & 3;
    const int ia = 4 * (b >> 1) + t, ib = 4 * (b & 1) + t;  // column 7 is the weight slot: 0
    double c4[4] = {0, 0, 0, 0};
    for (int r0 = 0; r0 < nr16; r0 += 16) {
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const double *row = rl + (r0 + 4 * u + k) * BA_ROW;
            const double w = row[7];
            const double va = ia < 7 ? row[ia] : 0.0;
            const double vb = ib < 7 ? row[ib] : 0.0;
            c4[u] = __builtin_amdgcn_mfma_f64_4x4x4f64(va * w, vb, c4[u], 0, 0, 0);
        }
    }
    C += (c4[0] + c4[1]) + (c4[2] + c4[3]);
}
#else
// One 64-edge slice into LDS rows (lane l: edge l -> rows 3l .. 3l+2: J_pose row, -e, w; zero
// rows for the third row of a mono edge and for inactive edges or lanes past the slice), then
// C += sum_r (w_r v_r)^T v_r by v_mfma_f64_16x16x4f64 (A[i][k] = w v[i], B[k][j] = v[j], 7
// columns padded to 16)
template <class ES>
__device__ __forceinline__ void ba_pose_slice(const orbg_pose &P, const double *__restrict__ points,
                                              const ES &edges,
                                              const int32_t *__restrict__ pose_edges, int e0,
                                              int ne, double *rl, int lane, BaAcc &C)
{
    {
        double v[3][BA_ROW];
#pragma unroll
        for (int k = 0; k < 3; k++)
#pragma unroll
            for (int c = 0; c < BA_ROW; c++) v[k][c] = 0;
        if (lane < ne) {
            const orbg_edge e = edges(pose_edges[e0 + lane]);
            if (e.active) {
                const double X[3] = {points[3 * (size_t)e.point], points[3 * (size_t)e.point + 1],
                                     points[3 * (size_t)e.point + 2]};
                BaLin L;
                ba_linearize_edge(P, X, e, L);
#pragma unroll
                for (int k = 0; k < 3; k++) {
                    const bool on = k < L.D;
#pragma unroll
                    for (int c = 0; c < 6; c++) v[k][c] = on ? L.jt[k][c] : 0.0;
                    v[k][6] = on ? -L.err[k] : 0.0;
                    v[k][7] = on ? L.w : 0.0;
                }
            }
        }
        wave_sync_lds_ba();  // the previous slice's reads of rl are done (in-order LDS)
#pragma unroll
        for (int k = 0; k < 3; k++)
#pragma unroll
            for (int c = 0; c < BA_ROW; c += 2)
                *(double2 *)(rl + (3 * lane + k) * BA_ROW + c) = make_double2(v[k][c], v[k][c + 1]);
    }
    wave_sync_lds_ba();
    const int nrow = 3 * ne;
    const int i = lane & 15, k = lane >> 4;  // A: (row i of the 16x4 tile, k); B: (k, column i)
    const int col = i < 7 ? i : 7;           // padded columns read the weight and are zeroed
    for (int r0 = 0; r0 < nrow; r0 += 4 * 4) {
        double va[4], vb[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int r = min(r0 + 4 * u + k, 3 * BA_SLICE - 1);  // rows past nrow are zero rows or
            const double vv = rl[r * BA_ROW + col];               // beyond: weight zeroed below
            const double w = r0 + 4 * u + k < nrow ? rl[r * BA_ROW + 7] : 0.0;
            vb[u] = i < 7 ? vv : 0.0;
            va[u] = vb[u] * w;
        }
#pragma unroll
        for (int u = 0; u < 4; u++) C = __builtin_amdgcn_mfma_f64_16x16x4f64(va[u], vb[u], C, 0, 0, 0);
    }
}
#endif

// record path: one wave per slice, the slices of one pose added by fp64 atomics onto the
// zeroed blocks.  Fixed poses get no block (g2o skips them).
template <class ES>
__global__ __launch_bounds__(256) void k_ba_pose_mfma(const orbg_pose *__restrict__ poses,
                                                      const double *__restrict__ points,
                                                      const ES edges,
                                                      const int32_t *__restrict__ pose_off,
                                                      const int32_t *__restrict__ pose_edges,
                                                      const int32_t *__restrict__ slice_off,
                                                      const int32_t *__restrict__ slice_pose,
                                                      int nslice, double *__restrict__ hpose,
                                                      double *__restrict__ bpose)
{
    __shared__ double rows_lds[4][3 * BA_SLICE * BA_ROW];  // 12 KB per wave
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int sl = blockIdx.x * 4 + wv;
    if (sl >= nslice) return;    // wave-uniform; no workgroup barrier below
    const int p = slice_pose[sl];
    if (p < 0) return;           // past the last slice (table filled with -1)
    const orbg_pose P = poses[p];
    if (P.fixed) return;         // stays zero (memset)
    double *H = hpose + 36 * (size_t)p, *bv = bpose + 6 * (size_t)p;
    const int e0p = pose_off[p], nep = pose_off[p + 1] - e0p;
    const int ks = sl - slice_off[p];
    BaAcc C = {};
    ba_pose_slice(P, points, edges, pose_edges, e0p + ks * BA_SLICE,
                  min(BA_SLICE, nep - ks * BA_SLICE), rows_lds[wv], lane, C);
    ba_acc_entries(C, lane, [&](int row, int col, double val) {
        if (row < 6 && col < 6) atomicAdd(&H[row * 6 + col], val);
        if (row < 6 && col == 6) atomicAdd(&bv[row], val);
    });
}

// graph path, pass 1: one wave per slice (the graph's slice tables, built once), the
// slice's [H | b] partial (6 x 7) stored -- no fills, no atomics
template <class ES>
__device__ __forceinline__ void ba_slice_part(const orbg_pose *__restrict__ poses,
                                              const double *__restrict__ points, const ES &edges,
                                              const int32_t *__restrict__ pose_off,
                                              const int32_t *__restrict__ pose_edges,
                                              const int32_t *__restrict__ slice_off,
                                              const int32_t *__restrict__ slice_pose, int sl,
                                              double *__restrict__ part, double *rows, int lane)
{
    const int p = slice_pose[sl];
    const orbg_pose P = poses[p];
    if (P.fixed) return;  // pass 2 writes the zero block
    const int e0p = pose_off[p], nep = pose_off[p + 1] - e0p;
    const int ks = sl - slice_off[p];
    BaAcc C = {};
    ba_pose_slice(P, points, edges, pose_edges, e0p + ks * BA_SLICE,
                  min(BA_SLICE, nep - ks * BA_SLICE), rows, lane, C);
    ba_acc_entries(C, lane, [&](int row, int col, double val) {
        if (row < 6 && col < 7) part[42 * (size_t)sl + row * 7 + col] = val;
    });
}

// graph path, pass 2: thread per (pose, block entry): the slice partials summed in slice order
// (the next launch: stream order makes pass 1's stores visible), zero for fixed poses and poses
// without edges; every block written, the same bits every build
__global__ __launch_bounds__(256) void k_ba_pose_reduce(const orbg_pose *__restrict__ poses,
                                                        int npose,
                                                        const int32_t *__restrict__ slice_off,
                                                        const double *__restrict__ part,
                                                        double *__restrict__ hpose,
                                                        double *__restrict__ bpose)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= 42 * npose) return;
    const int p = t / 42, e = t - 42 * p;
    double acc = 0;
    if (!poses[p].fixed) {
        // eight independent loads in flight, added in slice order (the same bits as one by one)
        const int s1 = slice_off[p + 1];
        int s = slice_off[p];
        for (; s + 8 <= s1; s += 8) {
            double v[8];
#pragma unroll
            for (int u = 0; u < 8; u++) v[u] = part[42 * (size_t)(s + u) + e];
#pragma unroll
            for (int u = 0; u < 8; u++) acc += v[u];
        }
        for (; s < s1; s++) acc += part[42 * (size_t)s + e];
    }
    const int row = e / 7, col = e - 7 * row;
    if (col < 6)
        hpose[36 * (size_t)p + row * 6 + col] = acc;
    else
        bpose[6 * (size_t)p + row] = acc;
}

// orbg_ba_graph's special points, one wave each: points whose slots span two k_ba_edges
// workgroups (their block summed here in edge order, the oracle's, instead of two partials)
// and points without edges (zero block).  Lane l computes edge l's share (chunks of 64),
// lanes 0..11 sum one block entry each over the edges in order.
template <class ES>
__device__ __forceinline__ void ba_special_point(const orbg_pose *__restrict__ poses,
                                                 const double *__restrict__ points,
                                                 const ES &edges,
                                                 const int32_t *__restrict__ point_off,
                                                 const int32_t *__restrict__ point_edges, int q,
                                                 double *__restrict__ hpoint,
                                                 double *__restrict__ bpoint, double (*sh)[64],
                                                 int lane)
{
    const double X[3] = {points[3 * (size_t)q], points[3 * (size_t)q + 1], points[3 * (size_t)q + 2]};
    const int a0 = point_off[q], a1 = point_off[q + 1];
    double acc = 0;  // lanes 0..11: entry `lane` of [H_ll | b_l]
    for (int c0 = a0; c0 < a1; c0 += 64) {
        double c[12];
#pragma unroll
        for (int k = 0; k < 12; k++) c[k] = 0;
        if (c0 + lane < a1) {
            const orbg_edge e = edges(point_edges[c0 + lane]);
            if (e.active) {
                BaLin L;
                ba_linearize_edge(poses[e.pose], X, e, L);
                ba_point_share(L, c);
            }
        }
        wave_sync_lds_ba();
#pragma unroll
        for (int k = 0; k < 12; k++) sh[k][lane] = c[k];
        wave_sync_lds_ba();
        const int n = min(64, a1 - c0);
        if (lane < 12)
            for (int j = 0; j < n; j++) acc += sh[lane][j];
    }
    if (lane < 9)
        hpoint[9 * (size_t)q + lane] = acc;
    else if (lane < 12)
        bpoint[3 * (size_t)q + lane - 9] = acc;
}

// graph path, pass 1: one launch, a wave per task -- the special points first (waves
// [0, 4 * nb_special): their chains of 64-edge chunks are the longest), then one wave per
// 64-edge slice of a pose (MFMA f64 partial of [H_pp | b_p]).  Both read only the graph and
// the estimate; merging them hides the special points' latency behind the slices.
template <class ES>
__global__ __launch_bounds__(256) void k_ba_slices_special(
    const orbg_pose *__restrict__ poses, const double *__restrict__ points, const ES edges,
    const int32_t *__restrict__ pose_off, const int32_t *__restrict__ pose_edges,
    const int32_t *__restrict__ slice_off, const int32_t *__restrict__ slice_pose, int nslice,
    double *__restrict__ part, const int32_t *__restrict__ point_off,
    const int32_t *__restrict__ point_edges, const int32_t *__restrict__ special, int nsp,
    int nb_special, double *__restrict__ hpoint, double *__restrict__ bpoint, int npose,
    double *__restrict__ hpose, double *__restrict__ bpose)
{
    __shared__ double rows_lds[4][3 * BA_SLICE * BA_ROW];  // 12 KB per wave (special: 6 KB)
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if ((int)blockIdx.x < nb_special) {
        const int i = blockIdx.x * 4 + wv;
        if (i >= nsp) return;  // wave-uniform; no workgroup barrier in either path
        ba_special_point(poses, points, edges, point_off, point_edges, special[i], hpoint, bpoint,
                         (double(*)[64])rows_lds[wv], lane);
        return;
    }
#if ORBG_BA_POSE_WG
    // a workgroup per pose: wave w accumulates the pose's slices w, w + 4, ... in its MFMA
    // tile, the four tiles are added in wave order through LDS and the block stored -- no
    // partials, no reduce launch; every pose block written (zero for fixed / edgeless poses)
    __shared__ double tiles[4][42];
    const int p = (int)blockIdx.x - nb_special;
    if (p >= npose) return;  // workgroup-uniform
    const orbg_pose P = poses[p];
    BaAcc C = {};
    if (!P.fixed) {
        const int e0p = pose_off[p], nep = pose_off[p + 1] - e0p;
        const int ns = (nep + BA_SLICE - 1) / BA_SLICE;
        for (int ks = wv; ks < ns; ks += 4)
            ba_pose_slice(P, points, edges, pose_edges, e0p + ks * BA_SLICE,
                          min(BA_SLICE, nep - ks * BA_SLICE), rows_lds[wv], lane, C);
    }
    ba_acc_entries(C, lane, [&](int row, int col, double val) {
        if (row < 6 && col < 7) tiles[wv][row * 7 + col] = val;
    });
    __syncthreads();
    if (threadIdx.x < 42) {
        const int e = threadIdx.x;
        const double acc = ((tiles[0][e] + tiles[1][e]) + tiles[2][e]) + tiles[3][e];
        const int row = e / 7, col = e - 7 * row;
        if (col < 6)
            hpose[36 * (size_t)p + row * 6 + col] = acc;
        else
            bpose[6 * (size_t)p + row] = acc;
    }
    (void)slice_off;
    (void)slice_pose;
    (void)nslice;
    (void)part;
#else
    const int sl = ((int)blockIdx.x - nb_special) * 4 + wv;
    if (sl >= nslice) return;
    ba_slice_part(poses, points, edges, pose_off, pose_edges, slice_off, slice_pose, sl, part,
                  rows_lds[wv], lane);
#endif
}

// slice -> pose table: pose p owns ceil(edges_p / BA_SLICE) consecutive slices
__global__ __launch_bounds__(256) void k_ba_slices(const int32_t *__restrict__ pose_off,
                                                   int npose, int32_t *__restrict__ slice_off,
                                                   int32_t *__restrict__ slice_pose, int *nslice)
{
    // single workgroup: exclusive scan of per-pose slice counts, then fill
    __shared__ int run;
    if (threadIdx.x == 0) run = 0;
    __syncthreads();
    for (int p0 = 0; p0 < npose; p0 += 256) {
        const int p = p0 + threadIdx.x;
        const int n = p < npose ? (pose_off[p + 1] - pose_off[p] + BA_SLICE - 1) / BA_SLICE : 0;
        int x = n;  // inclusive block scan (simple, npose is small)
        __shared__ int sc[256];
        sc[threadIdx.x] = x;
        __syncthreads();
        for (int o = 1; o < 256; o <<= 1) {
            const int y = threadIdx.x >= o ? sc[threadIdx.x - o] : 0;
            __syncthreads();
            sc[threadIdx.x] += y;
            __syncthreads();
        }
        const int excl = run + sc[threadIdx.x] - n;
        if (p < npose) {
            slice_off[p] = excl;
            for (int q = 0; q < n; q++) slice_pose[excl + q] = p;
        }
        __syncthreads();
        if (threadIdx.x == 255) run += sc[255];
        __syncthreads();
    }
    if (threadIdx.x == 0) *nslice = run;
}

static size_t al(size_t x) { return (x + 255) & ~(size_t)255; }

// slice tables (upper bound: one slice per pose plus one per BA_SLICE edges)
size_t ba_rows_bytes(int nedge, int npose)
{
    const size_t ns = (size_t)(npose > 0 ? npose : 1) + (size_t)(nedge > 0 ? nedge : 1) / BA_SLICE;
    return al((npose + 1) * 4) + al(ns * 4) + 256;
}

size_t ba_scratch_bytes(int npose, int npoint, int nedge)
{
    const size_t np = (size_t)(npose > 0 ? npose : 1), nq = (size_t)(npoint > 0 ? npoint : 1),
                 ne = (size_t)(nedge > 0 ? nedge : 1);
    return al(np * sizeof(orbg_pose)) + al(nq * 24) + al(ne * sizeof(orbg_edge)) +
           al(ne * sizeof(orbg_edge_out)) + al(np * 36 * 8) + al(np * 6 * 8) + al(nq * 9 * 8) +
           al(nq * 3 * 8) + al((np + 1) * 4) + 2 * al(ne * 4) + al((nq + 1) * 4) +
           ba_rows_bytes(nedge, npose);
}

// the orbg_edge_out records (include/orbg.h) as strided fields
static BaEdgeOut eout_fields(orbg_edge_out *eout, bool jacobians, bool errors)
{
    BaEdgeOut o{};
    if (!eout) return o;
    o.stride = (int)(sizeof(orbg_edge_out) / sizeof(double));
    o.hpl = &eout[0].hpl[0][0];
    if (errors) {
        o.err = &eout[0].err[0];
        o.chi2 = &eout[0].chi2;
        o.rho1 = &eout[0].rho1;
    }
    if (jacobians) {
        o.jp = &eout[0].jp[0][0];
        o.jt = &eout[0].jt[0][0];
    }
    return o;
}

// device-resident linearisation: every pointer is device memory; scratch = ba_rows_bytes.
// hpl != NULL: H_pl goes there as [nedge][3][6] (orbg_ba_build_system_device) and eout is
// not used.
template <class ES>
static int launch_ba_device_t(hipStream_t st, const orbg_pose *poses, int npose,
                              const double *points, int npoint, ES edges, int nedge,
                              const int32_t *pose_off, const int32_t *pose_edges,
                              const int32_t *point_off, const int32_t *point_edges,
                              orbg_edge_out *eout, double *hpose, double *bpose, double *hpoint,
                              double *bpoint, double *scr, void *prof, bool jacobians,
                              bool errors, double *hpl)
{
    BaEdgeOut o = eout_fields(eout, jacobians, errors);
    if (hpl) {
        o = BaEdgeOut{};
        o.hpl = hpl;
        o.stride = 18;
    }
    if (npoint) {
        // points without edges keep zero blocks; points spanning workgroups are summed onto
        // zero by atomics
        if (hipMemsetAsync(hpoint, 0, (size_t)npoint * 9 * 8, st) != hipSuccess ||
            hipMemsetAsync(bpoint, 0, (size_t)npoint * 3 * 8, st) != hipSuccess)
            return -5;
    }
    if (nedge) {
        hipEvent_t a = nullptr;
        prof_begin(prof, st, "ba_edges", &a);
        hipLaunchKernelGGL((k_ba_edges<ES, false>), dim3((nedge + BA_EDGES_TPB - 1) / BA_EDGES_TPB),
                           dim3(BA_EDGES_TPB), 0, st, poses, points, edges, nedge, point_off,
                           point_edges, o, hpoint, bpoint);
        prof_end(prof, st, "ba_edges", a);
    }
    if (npose) {
        // scratch: slice_off[npose+1], slice_pose[max], nslice
        uint8_t *t = (uint8_t *)scr;
        int32_t *slice_off = (int32_t *)t;
        t += al((npose + 1) * 4);
        int32_t *slice_pose = (int32_t *)t;
        const int max_slices = npose + (nedge > 0 ? nedge : 1) / BA_SLICE;
        t += al((size_t)max_slices * 4);
        int *d_nslice = (int *)t;
        if (hipMemsetAsync(hpose, 0, (size_t)npose * 36 * 8, st) != hipSuccess ||
            hipMemsetAsync(bpose, 0, (size_t)npose * 6 * 8, st) != hipSuccess)
            return -5;
        if (hipMemsetAsync(slice_pose, 0xFF, (size_t)max_slices * 4, st) != hipSuccess) return -5;
        hipLaunchKernelGGL(k_ba_slices, dim3(1), dim3(256), 0, st, pose_off, npose, slice_off,
                           slice_pose, d_nslice);
        hipEvent_t a = nullptr;
        prof_begin(prof, st, "ba_pose_mfma", &a);
        // the grid covers the bound; waves past the actual slice count exit at once
        hipLaunchKernelGGL(k_ba_pose_mfma<ES>, dim3((max_slices + 3) / 4), dim3(256), 0, st,
                           poses, points, edges, pose_off, pose_edges, slice_off, slice_pose,
                           max_slices, hpose, bpose);
        prof_end(prof, st, "ba_pose_mfma", a);
    }
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

int launch_ba_device(hipStream_t st, const orbg_pose *poses, int npose, const double *points,
                     int npoint, const orbg_edge *edges, int nedge, const int32_t *pose_off,
                     const int32_t *pose_edges, const int32_t *point_off,
                     const int32_t *point_edges, orbg_edge_out *eout, double *hpose,
                     double *bpose, double *hpoint, double *bpoint, double *scr, void *prof,
                     bool jacobians, bool errors, double *hpl)
{
    return launch_ba_device_t(st, poses, npose, points, npoint, BaEdgeRecords{edges}, nedge,
                              pose_off, pose_edges, point_off, point_edges, eout, hpose, bpose,
                              hpoint, bpoint, scr, prof, jacobians, errors, hpl);
}

// precomputed once per graph (BaGraphDev): the exact slice tables, the special vertices, the
// pose partials -- no zero fills, no slice-table kernel, no atomics on the blocks per build.
// Three launches: the edge pass, the special points + pose slices, the pose reduce.  (Round 4
// measured the pose blocks or the special points on a second stream beside the edge pass:
// slower, the edge pass fills the chip; profiles/r04n_ba_overlap_ab.txt.)
int launch_ba_graph(hipStream_t st, const orbg_pose *poses, int npose, const double *points,
                    int npoint, const BaPackedEdge *edges, const BaCam *cam, const BaInfo *info,
                    int nedge, const int32_t *pose_off, const int32_t *pose_edges,
                    const int32_t *point_off, const int32_t *point_edges, const BaGraphDev &gd,
                    double *hpl, double *hpose, double *bpose, double *hpoint, double *bpoint,
                    void *prof)
{
    const BaEdgePacked es{edges, cam, info};
    BaEdgeOut o{};
    o.hpl = hpl;
    o.stride = 18;
    if (nedge) {
        hipEvent_t a = nullptr;
        prof_begin(prof, st, "ba_edges", &a);
        hipLaunchKernelGGL((k_ba_edges<BaEdgePacked, true>),
                           dim3((nedge + BA_EDGES_TPB - 1) / BA_EDGES_TPB), dim3(BA_EDGES_TPB), 0,
                           st, poses, points, es, nedge, point_off, point_edges, o, hpoint, bpoint);
        prof_end(prof, st, "ba_edges", a);
    }
    const int nb_special = (gd.nspecial + 3) / 4;
#if ORBG_BA_POSE_WG
    const int nb_slice = npose;  // a workgroup per pose
#else
    const int nb_slice = npose ? (gd.nslice + 3) / 4 : 0;
#endif
    if (nb_special + nb_slice) {
        hipEvent_t a = nullptr;
        prof_begin(prof, st, "ba_pose_mfma", &a);
        hipLaunchKernelGGL(k_ba_slices_special<BaEdgePacked>, dim3(nb_special + nb_slice),
                           dim3(256), 0, st, poses, points, es, pose_off, pose_edges,
                           gd.slice_off, gd.slice_pose, npose ? gd.nslice : 0, gd.part, point_off,
                           point_edges, gd.special, gd.nspecial, nb_special, hpoint, bpoint,
                           npose, hpose, bpose);
        prof_end(prof, st, "ba_pose_mfma", a);
    }
    if (npose && !ORBG_BA_POSE_WG) {
        hipEvent_t a = nullptr;
        prof_begin(prof, st, "ba_pose_reduce", &a);
        hipLaunchKernelGGL(k_ba_pose_reduce, dim3((42 * npose + 255) / 256), dim3(256), 0, st,
                           poses, npose, gd.slice_off, gd.part, hpose, bpose);
        prof_end(prof, st, "ba_pose_reduce", a);
    }
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

// host arrays in/out: upload, build nothing on the device but the blocks, download
int launch_ba(hipStream_t st, const orbg_pose *poses, int npose, const double *points,
              int npoint, const orbg_edge *edges, int nedge, const int32_t *pose_off,
              const int32_t *pose_edges, const int32_t *point_off, const int32_t *point_edges,
              orbg_edge_out *eout, double *hpose, double *bpose, double *hpoint, double *bpoint,
              void *scratch, void *prof)
{
    uint8_t *s = (uint8_t *)scratch;
    const size_t np = (size_t)(npose > 0 ? npose : 1), nq = (size_t)(npoint > 0 ? npoint : 1),
                 ne = (size_t)(nedge > 0 ? nedge : 1);
    orbg_pose *d_pose = (orbg_pose *)s;
    s += al(np * sizeof(orbg_pose));
    double *d_pts = (double *)s;
    s += al(nq * 24);
    orbg_edge *d_edges = (orbg_edge *)s;
    s += al(ne * sizeof(orbg_edge));
    orbg_edge_out *d_eout = (orbg_edge_out *)s;
    s += al(ne * sizeof(orbg_edge_out));
    double *d_hpose = (double *)s;
    s += al(np * 36 * 8);
    double *d_bpose = (double *)s;
    s += al(np * 6 * 8);
    double *d_hpt = (double *)s;
    s += al(nq * 9 * 8);
    double *d_bpt = (double *)s;
    s += al(nq * 3 * 8);
    int32_t *d_off = (int32_t *)s;
    s += al((np + 1) * 4);
    int32_t *d_pe = (int32_t *)s;
    s += al(ne * 4);
    int32_t *d_qoff = (int32_t *)s;
    s += al((nq + 1) * 4);
    int32_t *d_qe = (int32_t *)s;
    s += al(ne * 4);
    double *d_rows = (double *)s;
#define CK(x)                                                                              \
    if ((x) != hipSuccess) return -5
    if (npose) CK(hipMemcpyAsync(d_pose, poses, npose * sizeof(orbg_pose), hipMemcpyHostToDevice, st));
    if (npoint) CK(hipMemcpyAsync(d_pts, points, (size_t)npoint * 24, hipMemcpyHostToDevice, st));
    if (nedge) CK(hipMemcpyAsync(d_edges, edges, nedge * sizeof(orbg_edge), hipMemcpyHostToDevice, st));
    if (npose) CK(hipMemcpyAsync(d_off, pose_off, (npose + 1) * 4, hipMemcpyHostToDevice, st));
    if (nedge) CK(hipMemcpyAsync(d_pe, pose_edges, nedge * 4, hipMemcpyHostToDevice, st));
    if (npoint) CK(hipMemcpyAsync(d_qoff, point_off, (npoint + 1) * 4, hipMemcpyHostToDevice, st));
    if (nedge) CK(hipMemcpyAsync(d_qe, point_edges, nedge * 4, hipMemcpyHostToDevice, st));
    const int rc = launch_ba_device(st, d_pose, npose, d_pts, npoint, d_edges, nedge, d_off, d_pe,
                                    d_qoff, d_qe, d_eout, d_hpose, d_bpose, d_hpt, d_bpt, d_rows,
                                    prof, true, true, nullptr);
    if (rc) return rc;
    if (eout && nedge)
        CK(hipMemcpyAsync(eout, d_eout, nedge * sizeof(orbg_edge_out), hipMemcpyDeviceToHost, st));
    if (npose) {
        CK(hipMemcpyAsync(hpose, d_hpose, (size_t)npose * 36 * 8, hipMemcpyDeviceToHost, st));
        CK(hipMemcpyAsync(bpose, d_bpose, (size_t)npose * 6 * 8, hipMemcpyDeviceToHost, st));
    }
    if (npoint) {
        CK(hipMemcpyAsync(hpoint, d_hpt, (size_t)npoint * 9 * 8, hipMemcpyDeviceToHost, st));
        CK(hipMemcpyAsync(bpoint, d_bpt, (size_t)npoint * 3 * 8, hipMemcpyDeviceToHost, st));
    }
#undef CK
    return 0;
}

}  // namespace orbg
