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
// Per-vertex blocks are accumulated with fp64 global atomics (no-return
// global_atomic_add_f64); the per-edge outputs are written coalesced as SoA.
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

__global__ __launch_bounds__(256) void k_ba_edges(const orbg_pose *__restrict__ poses,
                                                  const double *__restrict__ points,
                                                  const orbg_edge *__restrict__ edges, int nedge,
                                                  orbg_edge_out *__restrict__ eout,
                                                  double *__restrict__ hpose,
                                                  double *__restrict__ bpose,
                                                  double *__restrict__ hpoint,
                                                  double *__restrict__ bpoint)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nedge) return;
    const orbg_edge e = edges[i];
    orbg_edge_out o;
    memset(&o, 0, sizeof(o));
    if (!e.active) {
        if (eout) eout[i] = o;
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
    if (!e.stereo) {
        o.err[0] = e.obs[0] - ((x / z) * fx + e.cx);
        o.err[1] = e.obs[1] - ((y / z) * fy + e.cy);
    } else {
        const float invz = (float)(1.0f / z);
        const float bf = (float)e.bf;
        const double u = x * invz * fx + e.cx;
        const double v = y * invz * fy + e.cy;
        o.err[0] = e.obs[0] - u;
        o.err[1] = e.obs[1] - v;
        o.err[2] = e.obs[2] - (u - (double)(bf * invz));
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
    if (!e.stereo) {
        const double t02 = -x / z * fx, t12 = -y / z * fy;
        for (int c = 0; c < 3; c++) {
            o.jp[0][c] = -1. / z * (fx * R[0][c] + t02 * R[2][c]);
            o.jp[1][c] = -1. / z * (fy * R[1][c] + t12 * R[2][c]);
        }
    } else {
        for (int c = 0; c < 3; c++) {
            o.jp[0][c] = -fx * R[0][c] / z + fx * x * R[2][c] / z_2;
            o.jp[1][c] = -fy * R[1][c] / z + fy * y * R[2][c] / z_2;
            o.jp[2][c] = o.jp[0][c] - e.bf * R[2][c] / z_2;
        }
    }
    o.jt[0][0] = x * y / z_2 * fx;
    o.jt[0][1] = -(1 + (x * x / z_2)) * fx;
    o.jt[0][2] = y / z * fx;
    o.jt[0][3] = -1. / z * fx;
    o.jt[0][4] = 0;
    o.jt[0][5] = x / z_2 * fx;
    o.jt[1][0] = (1 + y * y / z_2) * fy;
    o.jt[1][1] = -x * y / z_2 * fy;
    o.jt[1][2] = -x / z * fy;
    o.jt[1][3] = 0;
    o.jt[1][4] = -1. / z * fy;
    o.jt[1][5] = y / z_2 * fy;
    if (e.stereo) {
        o.jt[2][0] = o.jt[0][0] - e.bf * y / z_2;
        o.jt[2][1] = o.jt[0][1] + e.bf * x / z_2;
        o.jt[2][2] = o.jt[0][2];
        o.jt[2][3] = o.jt[0][3];
        o.jt[2][4] = 0;
        o.jt[2][5] = o.jt[0][5] - e.bf / z_2;
    }
    const double info = e.inv_sigma2;
    double chi2 = 0;
    for (int k = 0; k < D; k++) chi2 += o.err[k] * (info * o.err[k]);
    o.chi2 = chi2;
    double rho1 = 1.0;
    if (e.robust) {
        const float dsqr = (float)(e.huber_delta * e.huber_delta);
        if (!(chi2 <= dsqr)) rho1 = e.huber_delta / sqrt(chi2);
    }
    o.rho1 = rho1;
    const double w = rho1 * info;
    double wr[3] = {0, 0, 0};
    for (int k = 0; k < D; k++) wr[k] = -info * o.err[k] * rho1;
    // point (vertex 0) block
    double *hp = hpoint + 9 * (size_t)e.point, *bp = bpoint + 3 * (size_t)e.point;
    for (int r = 0; r < 3; r++) {
        double acc = 0;
        for (int k = 0; k < D; k++) acc += o.jp[k][r] * wr[k];
        atomicAdd(&bp[r], acc);
        for (int c = 0; c < 3; c++) {
            double a2 = 0;
            for (int k = 0; k < D; k++) a2 += o.jp[k][r] * w * o.jp[k][c];
            atomicAdd(&hp[r * 3 + c], a2);
        }
    }
    if (!P.fixed) {
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 6; c++) {
                double a2 = 0;
                for (int k = 0; k < D; k++) a2 += o.jp[k][r] * w * o.jt[k][c];
                o.hpl[r][c] = a2;
            }
        double *ht = hpose + 36 * (size_t)e.pose, *bt = bpose + 6 * (size_t)e.pose;
        for (int r = 0; r < 6; r++) {
            double acc = 0;
            for (int k = 0; k < D; k++) acc += o.jt[k][r] * wr[k];
            atomicAdd(&bt[r], acc);
            for (int c = 0; c < 6; c++) {
                double a2 = 0;
                for (int k = 0; k < D; k++) a2 += o.jt[k][r] * w * o.jt[k][c];
                atomicAdd(&ht[r * 6 + c], a2);
            }
        }
    }
    if (eout) eout[i] = o;
}

static size_t al(size_t x) { return (x + 255) & ~(size_t)255; }

size_t ba_scratch_bytes(int npose, int npoint, int nedge)
{
    const size_t np = (size_t)(npose > 0 ? npose : 1), nq = (size_t)(npoint > 0 ? npoint : 1),
                 ne = (size_t)(nedge > 0 ? nedge : 1);
    return al(np * sizeof(orbg_pose)) + al(nq * 24) + al(ne * sizeof(orbg_edge)) +
           al(ne * sizeof(orbg_edge_out)) + al(np * 36 * 8) + al(np * 6 * 8) + al(nq * 9 * 8) +
           al(nq * 3 * 8);
}

int launch_ba(hipStream_t st, const orbg_pose *poses, int npose, const double *points,
              int npoint, const orbg_edge *edges, int nedge, orbg_edge_out *eout, double *hpose,
              double *bpose, double *hpoint, double *bpoint, void *scratch, void *prof)
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
#define CK(x)                                                                              \
    if ((x) != hipSuccess) return -5
    if (npose) CK(hipMemcpyAsync(d_pose, poses, npose * sizeof(orbg_pose), hipMemcpyHostToDevice, st));
    if (npoint) CK(hipMemcpyAsync(d_pts, points, (size_t)npoint * 24, hipMemcpyHostToDevice, st));
    if (nedge) CK(hipMemcpyAsync(d_edges, edges, nedge * sizeof(orbg_edge), hipMemcpyHostToDevice, st));
    CK(hipMemsetAsync(d_hpose, 0, np * 36 * 8, st));
    CK(hipMemsetAsync(d_bpose, 0, np * 6 * 8, st));
    CK(hipMemsetAsync(d_hpt, 0, nq * 9 * 8, st));
    CK(hipMemsetAsync(d_bpt, 0, nq * 3 * 8, st));
    if (nedge) {
        hipEvent_t a = nullptr;
        prof_begin(prof, st, "ba_edges", &a);
        hipLaunchKernelGGL(k_ba_edges, dim3((nedge + 255) / 256), dim3(256), 0, st, d_pose, d_pts,
                           d_edges, nedge, eout ? d_eout : nullptr, d_hpose, d_bpose, d_hpt,
                           d_bpt);
        prof_end(prof, st, "ba_edges", a);
        CK(hipGetLastError());
    }
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
