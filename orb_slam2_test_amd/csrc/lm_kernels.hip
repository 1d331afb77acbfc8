// lm_kernels.hip -- the rest of g2o's Levenberg-Marquardt iteration over device-resident
// LocalBundleAdjustment state (OptimizationAlgorithmLevenberg::solve,
// Thirdparty/g2o/g2o/core/optimization_algorithm_levenberg.cpp:61-164), beside the build
// (ba_kernels.hip), the error pass and the Schur solve (schur_kernels.hip):
//   k_ba_update    SparseOptimizer::update (sparse_optimizer.cpp): thread per pose,
//                  VertexSE3Expmap::oplusImpl (types_six_dof_expmap.h:73-76: estimate =
//                  SE3Quat::exp(dx) * estimate, se3_device.h; fixed poses untouched), and per
//                  point coordinate, VertexSBAPointXYZ::oplusImpl (estimate += dx)
//   k_lm_partial   the scalars the LM reads, each a deterministic two-level reduction:
//   k_lm_final       activeRobustChi2 (sum of rho over the active edges), computeScale
//                    (sum of x (lambda x + b)), computeLambdaInit's max |H_jj|; LM_RG
//                    workgroups walk the vector grid-stride in index order, a tree per
//                    workgroup, then one tree over the workgroups: a fixed order, so a run
//                    repeats bit for bit (g2o sums sequentially; the LM only compares these)
#include <hip/hip_runtime.h>

#include "../../include/orbg.h"
#include "orbg_internal.h"
#include "orbg_device.h"
#include "se3_device.h"

#pragma clang fp contract(off)

namespace orbg {

#define LM_RG 64   // reduction workgroups
#define LM_RT 256  // threads per reduction workgroup

// pout / qout may alias poses / points (the LM updates in place, orbg.h): no __restrict__ on
// those pairs; each thread reads its element before writing it
__global__ __launch_bounds__(256) void k_ba_update(const orbg_pose *poses, int npose,
                                                   const double *points, int npoint,
                                                   const double *__restrict__ dxp,
                                                   const double *__restrict__ dxq,
                                                   orbg_pose *pout, double *qout)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < npose) {
        orbg_pose p = poses[t];
        if (!p.fixed) {
            double upd[6];
#pragma unroll
            for (int k = 0; k < 6; k++) upd[k] = dxp[6 * (size_t)t + k];
            se3_oplus(p.q, p.t, upd);
        }
        pout[t] = p;
    }
    const int j = t - npose;
    if (j >= 0 && j < 3 * npoint) qout[j] = points[j] + dxq[j];
}

// term i of the reduction's vector (mode: LM_CHI2, LM_SCALE, LM_MAXDIAG)
struct LmArgs {
    int mode, n1, n2;  // vector = [part 1 (n1), part 2 (n2)]
    double lambda;
    const double *a1, *a2, *b1, *b2;
    const BaPackedEdge *edges;  // LM_CHI2: active = flags & 4
};

__device__ __forceinline__ double lm_term(const LmArgs &A, int i)
{
    if (A.mode == 0) return (A.edges[i].flags & 4u) ? A.a1[i] : 0.0;
    if (A.mode == 1) {
        const double x = i < A.n1 ? A.a1[i] : A.a2[i - A.n1];
        const double b = i < A.n1 ? A.b1[i] : A.b2[i - A.n1];
        return x * (A.lambda * x + b);
    }
    // |H_jj|: pose j -> H_pp[36 (j / 6) + 7 (j % 6)], point j -> H_ll[9 (j / 3) + 4 (j % 3)]
    if (i < A.n1) return fabs(A.a1[36 * (size_t)(i / 6) + 7 * (i % 6)]);
    const int k = i - A.n1;
    return fabs(A.a2[9 * (size_t)(k / 3) + 4 * (k % 3)]);
}

__device__ __forceinline__ double lm_comb(int mode, double a, double b)
{
    return mode == 2 ? fmax(a, b) : a + b;
}

__global__ __launch_bounds__(LM_RT) void k_lm_partial(LmArgs A, double *__restrict__ part)
{
    __shared__ double v[LM_RT];
    const int tid = threadIdx.x, n = A.n1 + A.n2;
    double acc = 0.0;
    for (int i = blockIdx.x * LM_RT + tid; i < n; i += LM_RG * LM_RT) acc = lm_comb(A.mode, acc, lm_term(A, i));
    v[tid] = acc;
    __syncthreads();
    for (int s = LM_RT / 2; s > 0; s >>= 1) {
        if (tid < s) v[tid] = lm_comb(A.mode, v[tid], v[tid + s]);
        __syncthreads();
    }
    if (tid == 0) part[blockIdx.x] = v[0];
}

__global__ __launch_bounds__(LM_RG) void k_lm_final(int mode, const double *__restrict__ part,
                                                    double *__restrict__ out)
{
    __shared__ double v[LM_RG];
    const int tid = threadIdx.x;
    v[tid] = part[tid];
    __syncthreads();
    for (int s = LM_RG / 2; s > 0; s >>= 1) {
        if (tid < s) v[tid] = lm_comb(mode, v[tid], v[tid + s]);
        __syncthreads();
    }
    if (tid == 0) *out = v[0];
}

int launch_ba_update(hipStream_t st, const orbg_pose *poses, int npose, const double *points,
                     int npoint, const double *dxp, const double *dxq, orbg_pose *pout,
                     double *qout)
{
    const int n = npose + 3 * npoint;
    if (n <= 0) return 0;
    hipLaunchKernelGGL(k_ba_update, dim3((n + 255) / 256), dim3(256), 0, st, poses, npose,
                       points, npoint, dxp, dxq, pout, qout);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

// mode 0: sum of a1[e] over active edges (n1 = nedge); 1: sum x (lambda x + b) over
// [a1 (n1), a2 (n2)] with b = [b1, b2]; 2: max |H_jj| (a1 = H_pp, n1 = 6 npose; a2 = H_ll,
// n2 = 3 npoint).  part: LM_RG doubles of scratch; out: one double
int launch_lm_reduce(hipStream_t st, int mode, int n1, int n2, double lambda, const double *a1,
                     const double *a2, const double *b1, const double *b2,
                     const BaPackedEdge *edges, double *part, double *out)
{
    LmArgs A{mode, n1, n2, lambda, a1, a2, b1, b2, edges};
    hipLaunchKernelGGL(k_lm_partial, dim3(LM_RG), dim3(LM_RT), 0, st, A, part);
    hipLaunchKernelGGL(k_lm_final, dim3(1), dim3(LM_RG), 0, st, mode, part, out);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

int lm_reduce_groups() { return LM_RG; }

}  // namespace orbg
