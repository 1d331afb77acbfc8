// schur_kernels.hip -- g2o BlockSolver<6,3>::solve with the Schur complement
// (Thirdparty/g2o/g2o/core/block_solver.hpp:354-486) for one LocalBundleAdjustment window,
// on gfx950, fp64.  Inputs are orbg_ba_linearize's blocks (H_pp, b_p per pose; H_ll, b_l per
// point; H_pl per edge) after setLambda(lambda); outputs the pose and point increments.
//
//   k_schur_points   thread per landmark: D^-1 = (H_ll + lambda I)^-1 (Eigen's cofactor
//                    3x3 inverse), D^-1 b_l, and per active edge to a free pose
//                    B D^-1 (6x3) and B D^-1 b_l (6)
//   k_schur_blocks   thread per (pose pair i1 <= i2, element): S = H_pp + lambda I (diagonal
//                    blocks) minus B_i D^-1 B_j^T landmark by landmark, then b_schur
//   k_schur_mirror   lower triangle = upper
//   k_schur_ldlt     one workgroup: dense LDLT (no pivoting) of S and the two triangular
//                    solves -- 6 x (free poses) unknowns, a few hundred at most
//   k_schur_backsub  thread per landmark: x_l = D^-1 (b_l - B^T x_p)
// Every sum runs in the order oracle/ba_oracle.c (orc_ba_schur_solve) pins, so the
// increments are bit-identical to it.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>

#include "../../include/orbg.h"
#include "orbg_device.h"
#include "schur_args.h"

#pragma clang fp contract(off)

namespace orbg {

void prof_begin(void *prof, hipStream_t s, const char *n, hipEvent_t *a);
void prof_end(void *prof, hipStream_t s, const char *n, hipEvent_t a);

__global__ void k_schur_points(SchurArgs A)
{
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= A.npoint) return;
    const int a0 = A.pt_off[p], a1 = A.pt_off[p + 1];
    double *Di = A.dinv + 9 * (size_t)p;
    if (a0 == a1) {
        for (int k = 0; k < 9; k++) Di[k] = 0;
        return;
    }
    double m[9];
    for (int k = 0; k < 9; k++) m[k] = A.hpoint[9 * (size_t)p + k];
    m[0] += A.lambda;
    m[4] += A.lambda;
    m[8] += A.lambda;
#define M(i, j) m[(i) * 3 + (j)]
#define COF(i, j) (M(((i) + 1) % 3, ((j) + 1) % 3) * M(((i) + 2) % 3, ((j) + 2) % 3) - \
                   M(((i) + 1) % 3, ((j) + 2) % 3) * M(((i) + 2) % 3, ((j) + 1) % 3))
    const double c0 = COF(0, 0), c1 = COF(1, 0), c2 = COF(2, 0);
    const double det = (c0 * M(0, 0) + c1 * M(1, 0)) + c2 * M(2, 0);
    const double invdet = 1.0 / det;
    double d[9];
    d[0] = c0 * invdet;
    d[1] = c1 * invdet;
    d[2] = c2 * invdet;
    d[3] = COF(0, 1) * invdet;
    d[4] = COF(1, 1) * invdet;
    d[5] = COF(2, 1) * invdet;
    d[6] = COF(0, 2) * invdet;
    d[7] = COF(1, 2) * invdet;
    d[8] = COF(2, 2) * invdet;
#undef COF
#undef M
    for (int k = 0; k < 9; k++) Di[k] = d[k];
    const double *bl = A.bpoint + 3 * (size_t)p;
    double db[3];
    for (int r = 0; r < 3; r++) db[r] = (d[r * 3] * bl[0] + d[r * 3 + 1] * bl[1]) + d[r * 3 + 2] * bl[2];
    for (int a = a0; a < a1; a++) {
        const int e = A.pt_edges[a];
        if (A.pidx[A.edge_pose[e]] < 0) continue;
        const double(*h)[6] = A.eout[e].hpl;  // B = h^T (6 x 3)
        double *bd = A.bd + 18 * (size_t)e;
        double *cf = A.cf + 6 * (size_t)e;
        for (int r = 0; r < 6; r++) {
            for (int c = 0; c < 3; c++)
                bd[r * 3 + c] = (h[0][r] * d[c] + h[1][r] * d[3 + c]) + h[2][r] * d[6 + c];
            cf[r] = (h[0][r] * db[0] + h[1][r] * db[1]) + h[2][r] * db[2];
        }
    }
}

// thread per (upper block, element): blocks of the free-pose pairs (i1 <= i2) that share a
// landmark, plus every diagonal block
__global__ void k_schur_blocks(SchurArgs A)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= A.nblk * 36) return;
    const int bk = t / 36, rc = t - bk * 36, r = rc / 6, c = rc - r * 6;
    const int i1 = A.blk_i1[bk], i2 = A.blk_i2[bk];
    double acc = 0.0;
    if (i1 == i2) {
        // the pose index of free pose i1 (pidx inverse is monotone: search)
        int pose = 0;
        for (int q = 0; q < A.npose; q++)
            if (A.pidx[q] == i1) pose = q;
        acc = A.hpose[36 * (size_t)pose + rc] + (r == c ? A.lambda : 0.0);
    }
    for (int k = A.blk_off[bk]; k < A.blk_off[bk + 1]; k++) {
        const int2 pr = A.blk_pairs[k];
        const double *bd = A.bd + 18 * (size_t)pr.x;
        const double(*h2)[6] = A.eout[pr.y].hpl;
        acc -= (bd[r * 3] * h2[0][c] + bd[r * 3 + 1] * h2[1][c]) + bd[r * 3 + 2] * h2[2][c];
    }
    A.S[(size_t)(6 * i1 + r) * A.n + 6 * i2 + c] = acc;
}

// b_schur = b_p - coefficients (coefficients summed per free pose in landmark order)
__global__ void k_schur_rhs(SchurArgs A)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= A.n) return;
    const int i = t / 6, r = t - i * 6;
    int pose = 0;
    for (int q = 0; q < A.npose; q++)
        if (A.pidx[q] == i) pose = q;
    double coef = 0.0;
    for (int k = A.pose_off[i]; k < A.pose_off[i + 1]; k++) coef += A.cf[6 * (size_t)A.pose_edges[k] + r];
    A.x[t] = A.bpose[6 * (size_t)pose + r] - coef;
}

__global__ void k_schur_mirror(SchurArgs A)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= A.n * A.n) return;
    const int r = t / A.n, c = t - r * A.n;
    if (r > c) A.S[(size_t)r * A.n + c] = A.S[(size_t)c * A.n + r];
}

// dense LDLT without pivoting + solves, one 256-thread workgroup (orc_ldlt_dense_solve)
__global__ __launch_bounds__(256) void k_schur_ldlt(SchurArgs A)
{
    const int n = A.n, tid = threadIdx.x;
    double *S = A.S, *x = A.x;
    __shared__ int bad;
    if (tid == 0) bad = 0;
    __syncthreads();
    for (int j = 0; j < n; j++) {
        if (tid == 0) {
            double d = S[(size_t)j * n + j];
            for (int k = 0; k < j; k++) d -= S[(size_t)j * n + k] * S[(size_t)j * n + k] * S[(size_t)k * n + k];
            S[(size_t)j * n + j] = d;
            if (d == 0.0 || !isfinite(d)) bad = 1;
        }
        __syncthreads();
        if (bad) break;
        const double d = S[(size_t)j * n + j];
        for (int i = j + 1 + tid; i < n; i += 256) {
            double s = S[(size_t)i * n + j];
            for (int k = 0; k < j; k++) s -= S[(size_t)i * n + k] * S[(size_t)j * n + k] * S[(size_t)k * n + k];
            S[(size_t)i * n + j] = s / d;
        }
        __syncthreads();
    }
    if (tid == 0) {
        if (!bad) {
            for (int i = 0; i < n; i++) {
                double s = x[i];
                for (int k = 0; k < i; k++) s -= S[(size_t)i * n + k] * x[k];
                x[i] = s;
            }
            for (int i = 0; i < n; i++) x[i] /= S[(size_t)i * n + i];
            for (int i = n - 1; i >= 0; i--) {
                double s = x[i];
                for (int k = i + 1; k < n; k++) s -= S[(size_t)k * n + i] * x[k];
                x[i] = s;
            }
        }
        *A.ok = !bad;
    }
}

// x_l = D^-1 (b_l - B^T x_p); pose increments scattered out
__global__ void k_schur_backsub(SchurArgs A)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const bool ok = *A.ok != 0;
    if (t < A.npose * 6) {
        const int i = A.pidx[t / 6];
        A.dx_pose[t] = (ok && i >= 0) ? A.x[6 * i + t % 6] : 0.0;
    }
    if (t >= A.npoint) return;
    const int p = t;
    double *xl = A.dx_point + 3 * (size_t)p;
    const int a0 = A.pt_off[p], a1 = A.pt_off[p + 1];
    if (!ok || a0 == a1) {
        xl[0] = xl[1] = xl[2] = 0.0;
        return;
    }
    const double *bl = A.bpoint + 3 * (size_t)p;
    double cl[3] = {bl[0], bl[1], bl[2]};
    for (int a = a0; a < a1; a++) {
        const int e = A.pt_edges[a], i1 = A.pidx[A.edge_pose[e]];
        if (i1 < 0) continue;
        const double(*h)[6] = A.eout[e].hpl;
        for (int k = 0; k < 3; k++) {
            double s = 0;
            for (int r = 0; r < 6; r++) s += h[k][r] * -A.x[6 * i1 + r];
            cl[k] += s;
        }
    }
    const double *Di = A.dinv + 9 * (size_t)p;
    for (int r = 0; r < 3; r++) xl[r] = (Di[r * 3] * cl[0] + Di[r * 3 + 1] * cl[1]) + Di[r * 3 + 2] * cl[2];
}

int launch_schur(hipStream_t st, const SchurArgs &A, void *prof)
{
    hipEvent_t ev = nullptr;
    prof_begin(prof, st, "schur", &ev);
    const int T = 256;
    hipLaunchKernelGGL(k_schur_points, dim3((A.npoint + T - 1) / T), dim3(T), 0, st, A);
    if (A.n > 0) {
        hipLaunchKernelGGL(k_schur_blocks, dim3((A.nblk * 36 + T - 1) / T), dim3(T), 0, st, A);
        hipLaunchKernelGGL(k_schur_rhs, dim3((A.n + T - 1) / T), dim3(T), 0, st, A);
        hipLaunchKernelGGL(k_schur_mirror, dim3((A.n * A.n + T - 1) / T), dim3(T), 0, st, A);
    }
    hipLaunchKernelGGL(k_schur_ldlt, dim3(1), dim3(256), 0, st, A);
    const int m = std::max(A.npoint, A.npose * 6);
    hipLaunchKernelGGL(k_schur_backsub, dim3((m + T - 1) / T), dim3(T), 0, st, A);
    prof_end(prof, st, "schur", ev);
    return hipGetLastError() == hipSuccess ? ORBG_OK : ORBG_EIO;
}

}  // namespace orbg
