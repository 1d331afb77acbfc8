// ba_kernels.hip -- per-edge arithmetic of Optimizer::LocalBundleAdjustment on gfx950.
//
// k_ba_edges: one thread per edge, fp64 throughout (world coordinates reach hundreds of
// metres on KITTI; obs - proj cancels, SURVEY.md 7 hard part 5):
//   EdgeSE3ProjectXYZ / EdgeStereoSE3ProjectXYZ::computeError  types_six_dof_expmap.h:90-95,122-127
//   cam_project (stereo: float invz, float bf)                 types_six_dof_expmap.cpp:141-157
//   linearizeOplus                                             types_six_dof_expmap.cpp:103-139,188-234
//   chi2, Huber rho' (float dsqr)                              base_edge.h:58-61, robust_kernel_impl.cpp:65-91
//   constructQuadraticForm: H_pp += A^T W A, b_p += A^T w_r,   base_binary_edge.hpp:55-120
//       H_ll += B^T W B, b_l += B^T w_r, H_pl = A^T W B
// Point blocks are accumulated with fp64 global atomics (no-return global_atomic_add_f64);
// pose blocks by k_ba_pose_mfma (MFMA f64 over each pose's edge rows).
#include <hip/hip_runtime.h>

#include <cstring>

#include "../../include/orbg.h"

namespace orbg {

void prof_begin(void *prof, hipStream_t s, const char *n, hipEvent_t *a);
void prof_end(void *prof, hipStream_t s, const char *n, hipEvent_t a);

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

// ---------------------------------------------------------------------------
// k_ba_edges: thread per edge.  Per-edge outputs go straight to global (no 400-byte live
// struct); point blocks are accumulated with fp64 atomics (a point has ~4-5 observations,
// so contention is low); the pose side is left to k_ba_pose_mfma through three rows per
// edge: rows[e][k] = {J_pose[k][0..5], -e[k], w} (w = rho' * invSigma2; mono edges have a
// zero third row, inactive edges zero rows).
// ---------------------------------------------------------------------------
#define BA_ROW 8  // doubles per pose row

__global__ __launch_bounds__(256) void k_ba_edges(const orbg_pose *__restrict__ poses,
                                                  const double *__restrict__ points,
                                                  const orbg_edge *__restrict__ edges, int nedge,
                                                  orbg_edge_out *__restrict__ eout,
                                                  double *__restrict__ rows,
                                                  double *__restrict__ hpoint,
                                                  double *__restrict__ bpoint)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nedge) return;
    const orbg_edge e = edges[i];
    orbg_edge_out *o = eout + i;
    double *row = rows + (size_t)i * 3 * BA_ROW;
    if (!e.active) {
        memset(o, 0, sizeof(*o));
        for (int k = 0; k < 3 * BA_ROW; k++) row[k] = 0;
        return;
    }
    const orbg_pose P = poses[e.pose];
    const double X[3] = {points[3 * e.point], points[3 * e.point + 1], points[3 * e.point + 2]};
    double xc[3];
    quat_rotate(P.q, X, xc);
    xc[0] += P.t[0];
    xc[1] += P.t[1];
    xc[2] += P.t[2];
    const double x = xc[0], y = xc[1], z = xc[2], z_2 = z * z;
    const double fx = e.fx, fy = e.fy;
    const int D = e.stereo ? 3 : 2;
    double err[3] = {0, 0, 0};
    if (!e.stereo) {
        err[0] = e.obs[0] - ((x / z) * fx + e.cx);
        err[1] = e.obs[1] - ((y / z) * fy + e.cy);
    } else {
        const float invz = (float)(1.0f / z);
        const float bf = (float)e.bf;
        const double u = x * invz * fx + e.cx;
        const double v = y * invz * fy + e.cy;
        err[0] = e.obs[0] - u;
        err[1] = e.obs[1] - v;
        err[2] = e.obs[2] - (u - (double)(bf * invz));
    }
    // rotation matrix (Eigen toRotationMatrix)
    const double *q = P.q;
    const double tx = 2 * q[0], ty = 2 * q[1], tz = 2 * q[2];
    const double twx = tx * q[3], twy = ty * q[3], twz = tz * q[3];
    const double txx = tx * q[0], txy = ty * q[0], txz = tz * q[0];
    const double tyy = ty * q[1], tyz = tz * q[1], tzz = tz * q[2];
    const double R[3][3] = {{1 - (tyy + tzz), txy - twz, txz + twy},
                            {txy + twz, 1 - (txx + tzz), tyz - twx},
                            {txz - twy, tyz + twx, 1 - (txx + tyy)}};
    double jp[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
    if (!e.stereo) {
        const double t02 = -x / z * fx, t12 = -y / z * fy;
        for (int c = 0; c < 3; c++) {
            jp[0][c] = -1. / z * (fx * R[0][c] + t02 * R[2][c]);
            jp[1][c] = -1. / z * (fy * R[1][c] + t12 * R[2][c]);
        }
    } else {
        for (int c = 0; c < 3; c++) {
            jp[0][c] = -fx * R[0][c] / z + fx * x * R[2][c] / z_2;
            jp[1][c] = -fy * R[1][c] / z + fy * y * R[2][c] / z_2;
            jp[2][c] = jp[0][c] - e.bf * R[2][c] / z_2;
        }
    }
    double jt[3][6];
    jt[0][0] = x * y / z_2 * fx;
    jt[0][1] = -(1 + (x * x / z_2)) * fx;
    jt[0][2] = y / z * fx;
    jt[0][3] = -1. / z * fx;
    jt[0][4] = 0;
    jt[0][5] = x / z_2 * fx;
    jt[1][0] = (1 + y * y / z_2) * fy;
    jt[1][1] = -x * y / z_2 * fy;
    jt[1][2] = -x / z * fy;
    jt[1][3] = 0;
    jt[1][4] = -1. / z * fy;
    jt[1][5] = y / z_2 * fy;
    if (e.stereo) {
        jt[2][0] = jt[0][0] - e.bf * y / z_2;
        jt[2][1] = jt[0][1] + e.bf * x / z_2;
        jt[2][2] = jt[0][2];
        jt[2][3] = jt[0][3];
        jt[2][4] = 0;
        jt[2][5] = jt[0][5] - e.bf / z_2;
    } else {
        for (int c = 0; c < 6; c++) jt[2][c] = 0;
    }
    const double info = e.inv_sigma2;
    // fixed trip counts (the third row of a mono edge is zero: adding it adds exact zeros)
    // keep every array in registers
    double chi2 = 0;
#pragma unroll
    for (int k = 0; k < 3; k++) chi2 += err[k] * (info * err[k]);
    double rho1 = 1.0;
    if (e.robust) {
        const float dsqr = (float)(e.huber_delta * e.huber_delta);
        if (!(chi2 <= dsqr)) rho1 = e.huber_delta / sqrt(chi2);
    }
    const double w = rho1 * info;
    for (int k = 0; k < 3; k++) o->err[k] = err[k];
    o->chi2 = chi2;
    o->rho1 = rho1;
    for (int k = 0; k < 3; k++)
        for (int c = 0; c < 3; c++) o->jp[k][c] = jp[k][c];
    for (int k = 0; k < 3; k++)
        for (int c = 0; c < 6; c++) o->jt[k][c] = jt[k][c];
    // point (vertex 0) block
    double wr[3];
#pragma unroll
    for (int k = 0; k < 3; k++) wr[k] = -info * err[k] * rho1;
    double *hp = hpoint + 9 * (size_t)e.point, *bp = bpoint + 3 * (size_t)e.point;
#pragma unroll
    for (int r = 0; r < 3; r++) {
        double acc = 0;
#pragma unroll
        for (int k = 0; k < 3; k++) acc += jp[k][r] * wr[k];
        atomicAdd(&bp[r], acc);
#pragma unroll
        for (int c = 0; c < 3; c++) {
            double a2 = 0;
#pragma unroll
            for (int k = 0; k < 3; k++) a2 += jp[k][r] * w * jp[k][c];
            atomicAdd(&hp[r * 3 + c], a2);
        }
    }
    // H_pl = J_point^T W J_pose (stored per edge, base_binary_edge.hpp:105-117)
#pragma unroll
    for (int r = 0; r < 3; r++)
#pragma unroll
        for (int c = 0; c < 6; c++) {
            double a2 = 0;
            if (!P.fixed)
#pragma unroll
                for (int k = 0; k < 3; k++) a2 += jp[k][r] * w * jt[k][c];
            o->hpl[r][c] = a2;
        }
    // pose rows for k_ba_pose_mfma
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const bool on = k < D;
        for (int c = 0; c < 6; c++) row[k * BA_ROW + c] = on ? jt[k][c] : 0.0;
        row[k * BA_ROW + 6] = on ? -err[k] : 0.0;
        row[k * BA_ROW + 7] = on ? w : 0.0;
    }
}

// ---------------------------------------------------------------------------
// k_ba_pose_mfma: one wave per pose.  With v_r = [J_pose row | -e] (7 wide) and weight w_r
// over the pose's rows r (3 per edge, from the pose's edge list),
//     C = sum_r (w_r v_r)^T v_r   gives  H_pp = C[0:6][0:6],  b_p = C[0:6][6]
// (constructQuadraticForm's A^T W A and A^T omega_r, omega_r = -rho' Omega e), accumulated
// in fp64 by v_mfma_f64_16x16x4_f64: each instruction folds 4 rows, A[i][k] = w v[i] and
// B[k][j] = v[j] padded from 7 to 16.  Fixed poses get no block (g2o skips them).
// ---------------------------------------------------------------------------
typedef double v4d __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_ba_pose_mfma(const orbg_pose *__restrict__ poses,
                                                      int npose,
                                                      const int32_t *__restrict__ pose_off,
                                                      const int32_t *__restrict__ pose_edges,
                                                      const double *__restrict__ rows,
                                                      double *__restrict__ hpose,
                                                      double *__restrict__ bpose)
{
    const int lane = threadIdx.x & 63;
    const int p = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (p >= npose) return;
    double *H = hpose + 36 * (size_t)p, *bv = bpose + 6 * (size_t)p;
    if (poses[p].fixed) {
        if (lane < 36) H[lane] = 0;
        if (lane < 6) bv[lane] = 0;
        return;
    }
    const int e0 = pose_off[p], ne = pose_off[p + 1] - e0;
    const int nrow = 3 * ne;
    const int i = lane & 15, k = lane >> 4;  // A: (row i of the 16x4 tile, k); B: (k, column i)
    const int col = i < 7 ? i : 7;           // padded columns read the weight and are zeroed
    v4d C = {0, 0, 0, 0};
    for (int r0 = 0; r0 < nrow; r0 += 4 * 4) {
        double va[4], vb[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {  // four MFMA steps' loads in flight
            const int r = r0 + 4 * u + k;
            double v = 0, w = 0;
            if (r < nrow) {
                const double *rw = rows + ((size_t)pose_edges[e0 + r / 3] * 3 + r % 3) * BA_ROW;
                v = rw[col];
                w = rw[7];
            }
            vb[u] = i < 7 ? v : 0.0;
            va[u] = vb[u] * w;
        }
#pragma unroll
        for (int u = 0; u < 4; u++) C = __builtin_amdgcn_mfma_f64_16x16x4f64(va[u], vb[u], C, 0, 0, 0);
    }
    // D layout of v_mfma_f64_16x16x4f64 (measured): lane holds column j = lane % 16 of rows
    // lane / 16 + 4 v, v = 0..3
    const int j = lane & 15;
#pragma unroll
    for (int v = 0; v < 4; v++) {
        const int row = (lane >> 4) + 4 * v;
        if (row < 6 && j < 6) H[row * 6 + j] = C[v];
        if (row < 6 && j == 6) bv[row] = C[v];
    }
}

static size_t al(size_t x) { return (x + 255) & ~(size_t)255; }

size_t ba_scratch_bytes(int npose, int npoint, int nedge)
{
    const size_t np = (size_t)(npose > 0 ? npose : 1), nq = (size_t)(npoint > 0 ? npoint : 1),
                 ne = (size_t)(nedge > 0 ? nedge : 1);
    return al(np * sizeof(orbg_pose)) + al(nq * 24) + al(ne * sizeof(orbg_edge)) +
           al(ne * sizeof(orbg_edge_out)) + al(np * 36 * 8) + al(np * 6 * 8) + al(nq * 9 * 8) +
           al(nq * 3 * 8) + al((np + 1) * 4) + al(ne * 4) + al(ne * 3 * BA_ROW * 8);
}

size_t ba_rows_bytes(int nedge) { return (size_t)(nedge > 0 ? nedge : 1) * 3 * BA_ROW * 8; }

// device-resident linearisation: every pointer is device memory; rows = ba_rows_bytes(nedge)
int launch_ba_device(hipStream_t st, const orbg_pose *poses, int npose, const double *points,
                     int npoint, const orbg_edge *edges, int nedge, const int32_t *pose_off,
                     const int32_t *pose_edges, orbg_edge_out *eout, double *hpose, double *bpose,
                     double *hpoint, double *bpoint, double *rows, void *prof)
{
    if (npoint && (hipMemsetAsync(hpoint, 0, (size_t)npoint * 9 * 8, st) != hipSuccess ||
                   hipMemsetAsync(bpoint, 0, (size_t)npoint * 3 * 8, st) != hipSuccess))
        return -5;
    if (nedge) {
        hipEvent_t a = nullptr;
        prof_begin(prof, st, "ba_edges", &a);
        hipLaunchKernelGGL(k_ba_edges, dim3((nedge + 255) / 256), dim3(256), 0, st, poses, points,
                           edges, nedge, eout, rows, hpoint, bpoint);
        prof_end(prof, st, "ba_edges", a);
    }
    if (npose) {
        hipEvent_t a = nullptr;
        prof_begin(prof, st, "ba_pose_mfma", &a);
        hipLaunchKernelGGL(k_ba_pose_mfma, dim3((npose + 3) / 4), dim3(256), 0, st, poses, npose,
                           pose_off, pose_edges, rows, hpose, bpose);
        prof_end(prof, st, "ba_pose_mfma", a);
    }
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

// host arrays in/out: upload, build nothing on the device but the blocks, download
int launch_ba(hipStream_t st, const orbg_pose *poses, int npose, const double *points,
              int npoint, const orbg_edge *edges, int nedge, const int32_t *pose_off,
              const int32_t *pose_edges, orbg_edge_out *eout, double *hpose, double *bpose,
              double *hpoint, double *bpoint, void *scratch, void *prof)
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
    double *d_rows = (double *)s;
#define CK(x)                                                                              \
    if ((x) != hipSuccess) return -5
    if (npose) CK(hipMemcpyAsync(d_pose, poses, npose * sizeof(orbg_pose), hipMemcpyHostToDevice, st));
    if (npoint) CK(hipMemcpyAsync(d_pts, points, (size_t)npoint * 24, hipMemcpyHostToDevice, st));
    if (nedge) CK(hipMemcpyAsync(d_edges, edges, nedge * sizeof(orbg_edge), hipMemcpyHostToDevice, st));
    if (npose) CK(hipMemcpyAsync(d_off, pose_off, (npose + 1) * 4, hipMemcpyHostToDevice, st));
    if (nedge) CK(hipMemcpyAsync(d_pe, pose_edges, nedge * 4, hipMemcpyHostToDevice, st));
    const int rc = launch_ba_device(st, d_pose, npose, d_pts, npoint, d_edges, nedge, d_off, d_pe,
                                    d_eout, d_hpose, d_bpose, d_hpt, d_bpt, d_rows, prof);
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
