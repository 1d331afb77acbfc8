// triangulate_kernels.hip -- LocalMapping::CreateNewMapPoints on the device: the per-pair
// geometry (ComputeF12, src/LocalMapping.cc:690-707, + pKF1's camera centre: the
// orbg_triangulation_pair SearchForTriangulation reads) and the triangulation of every matched
// pair (:395-560: parallax, linear triangulation or UnprojectStereo, the two cheirality tests,
// the chi-square reprojection gates, scale consistency).
//
//   k_tri_geometry   thread per KeyFrame pair
//   k_triangulate    thread per pKF1 feature i of a pair (grid y = pair): its matched pKF2
//                    feature, status + x3D written for every i < N, the new points counted
//                    per pair (ballot + one atomic per wave)
//
// Pure per-thread float / double arithmetic in the reference's order (the oracle's, oracle/
// mapping_oracle.c orc_tri_geometry / orc_triangulate, bit for bit): cv::gemm and Mat::dot in
// double with one rounding, A.inv()*B as the float LU solve, invert()'s 3x3 closed form, glibc
// atan2f / cosf restated; cv::SVD::compute of the 4x4 system is the null vector of A^T A by the
// oracle's cyclic Jacobi in double.  Branch-divergent (the reference's `continue`s), ~1 us of
// ALU per pair and ~100 B read: latency- and launch-bound, not HBM-bound, at KeyFrame rates.
#include <hip/hip_runtime.h>

#include <cmath>

#include "../../include/orbg.h"
#include "orbg_device.h"

#pragma clang fp contract(off)

namespace orbg {

struct TriLevelTabs {
    float scale[ORBG_MAX_LEVELS];   // mvScaleFactors
    float sigma2[ORBG_MAX_LEVELS];  // mvLevelSigma2
    float ratio;                    // 1.5f * mfScaleFactor
};

// ---- float helpers (glibc's atan2f: fdlibm e_atan2f.c / s_atanf.c, atanf's 2^25 bound) ----
static __constant__ const float tri_atanhi[4] = {4.6364760399e-01f, 7.8539812565e-01f,
                                                 9.8279368877e-01f, 1.5707962513e+00f};
static __constant__ const float tri_atanlo[4] = {5.0121582440e-09f, 3.7748947079e-08f,
                                                 3.4473217170e-08f, 7.5497894159e-08f};
static __constant__ const float tri_aT[11] = {
    3.3333334327e-01f, -2.0000000298e-01f, 1.4285714924e-01f, -1.1111110449e-01f,
    9.0908870101e-02f, -7.6918758452e-02f, 6.6610731184e-02f, -5.8335702866e-02f,
    4.9768779427e-02f, -3.6531571299e-02f, 1.6285819933e-02f};

__device__ __forceinline__ float glibc_atanf(float x)
{
    const int32_t hx = (int32_t)__float_as_uint(x), ix = hx & 0x7fffffff;
    int id;
    if (ix >= 0x4c000000) {
        if (ix > 0x7f800000) return x + x;
        return hx > 0 ? tri_atanhi[3] + tri_atanlo[3] : -tri_atanhi[3] - tri_atanlo[3];
    }
    if (ix < 0x3ee00000) {
        if (ix < 0x31000000) return x;
        id = -1;
    } else {
        x = fabsf(x);
        if (ix < 0x3f980000) {
            if (ix < 0x3f300000) {
                id = 0;
                x = (2.0f * x - 1.0f) / (2.0f + x);
            } else {
                id = 1;
                x = (x - 1.0f) / (x + 1.0f);
            }
        } else if (ix < 0x401c0000) {
            id = 2;
            x = (x - 1.5f) / (1.0f + 1.5f * x);
        } else {
            id = 3;
            x = -1.0f / x;
        }
    }
    const float z = x * x, w = z * z;
    const float s1 = z * (tri_aT[0] + w * (tri_aT[2] + w * (tri_aT[4] + w * (tri_aT[6] + w * (tri_aT[8] + w * tri_aT[10])))));
    const float s2 = w * (tri_aT[1] + w * (tri_aT[3] + w * (tri_aT[5] + w * (tri_aT[7] + w * tri_aT[9]))));
    if (id < 0) return x - x * (s1 + s2);
    const float r = tri_atanhi[id] - ((x * (s1 + s2) - tri_atanlo[id]) - x);
    return hx < 0 ? -r : r;
}

__device__ __forceinline__ float glibc_atan2f(float y, float x)
{
    const float tiny = 1.0e-30f, pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f,
                pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f;
    const int32_t hx = (int32_t)__float_as_uint(x), ix = hx & 0x7fffffff;
    const int32_t hy = (int32_t)__float_as_uint(y), iy = hy & 0x7fffffff;
    if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;
    if (hx == 0x3f800000) return glibc_atanf(y);
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
    if (iy == 0) return m < 2 ? y : (m == 2 ? pi + tiny : -pi - tiny);
    if (ix == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    if (ix == 0x7f800000) {
        if (iy == 0x7f800000) {
            const float r[4] = {pi_o_4 + tiny, -pi_o_4 - tiny, 3.0f * pi_o_4 + tiny, -3.0f * pi_o_4 - tiny};
            return r[m];
        }
        const float r[4] = {0.0f, -0.0f, pi + tiny, -pi - tiny};
        return r[m];
    }
    if (iy == 0x7f800000) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    const int k = (iy - ix) >> 23;
    float z;
    if (k > 60)
        z = pi_o_2 + 0.5f * pi_lo;
    else if (hx < 0 && k < -60)
        z = 0.0f;
    else
        z = glibc_atanf(fabsf(y / x));
    switch (m) {
    case 0: return z;
    case 1: return __uint_as_float(__float_as_uint(z) ^ 0x80000000u);
    case 2: return pi - (z - pi_lo);
    default: return (z - pi_lo) - pi;
    }
}

__device__ __forceinline__ float glibc_cosf(float y)
{
    float s, c;
    glibc_sincosf(y, &s, &c);
    return c;
}

// ---- small matrices (row-major 3x4 poses: rotation R[4 r + k], translation R[4 r + 3]) ----
// cv::gemm of the rotation (transposed if tr) with a float 3-vector: double sums, alpha, + c
__device__ __forceinline__ void tri_gemm3(const float *R, bool tr, const float *x, double alpha,
                                          const float *c, float *out)
{
#pragma unroll
    for (int r = 0; r < 3; r++) {
        double t = 0.0;
#pragma unroll
        for (int k = 0; k < 3; k++) t += (double)(tr ? R[4 * k + r] : R[4 * r + k]) * (double)x[k];
        t *= alpha;
        if (c) t += (double)c[r];
        out[r] = (float)t;
    }
}

__device__ __forceinline__ double tri_dot3(const float *a, const float *b)
{
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < 3; k++) s += (double)a[k] * (double)b[k];
    return s;
}

__device__ __forceinline__ void tri_mm3(const float *A, const float *B, float *C)
{
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) {
            double t = 0.0;
#pragma unroll
            for (int k = 0; k < 3; k++) t += (double)A[3 * i + k] * (double)B[3 * k + j];
            C[3 * i + j] = (float)t;
        }
}

// solve(A, B) for 3x3 floats (hal::LU32f, partial pivoting, eps 10 FLT_EPSILON): X into B
__device__ void tri_solve3_lu(const float *A0, float *B)
{
    float A[9];
#pragma unroll
    for (int k = 0; k < 9; k++) A[k] = A0[k];
    const float eps = 10.0f * 1.19209290e-07f;
#pragma unroll
    for (int i = 0; i < 3; i++) {
        int k = i;
#pragma unroll
        for (int j = i + 1; j < 3; j++)
            if (fabsf(A[3 * j + i]) > fabsf(A[3 * k + i])) k = j;
        float piv = A[3 * i + i];
#pragma unroll
        for (int j = i + 1; j < 3; j++)
            if (k == j) piv = A[3 * j + i];
        if (fabsf(piv) < eps) {
#pragma unroll
            for (int q = 0; q < 9; q++) B[q] = 0.0f;
            return;
        }
        // row swap i <-> k (k >= i), columns >= i of A, all of B: selects, no dynamic index
#pragma unroll
        for (int j = i + 1; j < 3; j++)
            if (k == j) {
#pragma unroll
                for (int c = 0; c < 3; c++) {
                    if (c >= i) {
                        const float t = A[3 * i + c];
                        A[3 * i + c] = A[3 * j + c];
                        A[3 * j + c] = t;
                    }
                    const float t = B[3 * i + c];
                    B[3 * i + c] = B[3 * j + c];
                    B[3 * j + c] = t;
                }
            }
        const float d = -1.0f / A[3 * i + i];
#pragma unroll
        for (int j = i + 1; j < 3; j++) {
            const float alpha = A[3 * j + i] * d;
#pragma unroll
            for (int c = i + 1; c < 3; c++) A[3 * j + c] += alpha * A[3 * i + c];
#pragma unroll
            for (int c = 0; c < 3; c++) B[3 * j + c] += alpha * B[3 * i + c];
        }
        A[3 * i + i] = -d;
    }
#pragma unroll
    for (int i = 2; i >= 0; i--)
#pragma unroll
        for (int j = 0; j < 3; j++) {
            float s = B[3 * i + j];
#pragma unroll
            for (int c = i + 1; c < 3; c++) s -= A[3 * i + c] * B[3 * c + j];
            B[3 * i + j] = s * A[3 * i + i];
        }
}

// invert() of a 3x3 float: det3 and the cofactors in double, times 1/det, rounded
__device__ __forceinline__ void tri_inv3f(const float *S, float *D)
{
#define Sf(y, x) ((double)S[3 * (y) + (x)])
    double d = Sf(0, 0) * (Sf(1, 1) * Sf(2, 2) - Sf(1, 2) * Sf(2, 1)) -
               Sf(0, 1) * (Sf(1, 0) * Sf(2, 2) - Sf(1, 2) * Sf(2, 0)) +
               Sf(0, 2) * (Sf(1, 0) * Sf(2, 1) - Sf(1, 1) * Sf(2, 0));
    if (d == 0.0) {
#pragma unroll
        for (int k = 0; k < 9; k++) D[k] = 0.0f;
        return;
    }
    d = 1.0 / d;
    D[0] = (float)((Sf(1, 1) * Sf(2, 2) - Sf(1, 2) * Sf(2, 1)) * d);
    D[1] = (float)((Sf(0, 2) * Sf(2, 1) - Sf(0, 1) * Sf(2, 2)) * d);
    D[2] = (float)((Sf(0, 1) * Sf(1, 2) - Sf(0, 2) * Sf(1, 1)) * d);
    D[3] = (float)((Sf(1, 2) * Sf(2, 0) - Sf(1, 0) * Sf(2, 2)) * d);
    D[4] = (float)((Sf(0, 0) * Sf(2, 2) - Sf(0, 2) * Sf(2, 0)) * d);
    D[5] = (float)((Sf(0, 2) * Sf(1, 0) - Sf(0, 0) * Sf(1, 2)) * d);
    D[6] = (float)((Sf(1, 0) * Sf(2, 1) - Sf(1, 1) * Sf(2, 0)) * d);
    D[7] = (float)((Sf(0, 1) * Sf(2, 0) - Sf(0, 0) * Sf(2, 1)) * d);
    D[8] = (float)((Sf(0, 0) * Sf(1, 1) - Sf(0, 1) * Sf(1, 0)) * d);
#undef Sf
}

// KeyFrame::SetPose's camera centre Ow = -Rcw^T tcw (gemm, alpha -1)
__device__ __forceinline__ void tri_center(const float *T, float *Ow)
{
    const float t[3] = {T[3], T[7], T[11]};
    tri_gemm3(T, true, t, -1.0, nullptr, Ow);
}

__global__ __launch_bounds__(256) void k_tri_geometry(const orbg_kf_camera *__restrict__ cams,
                                                      const int32_t *__restrict__ kf1,
                                                      const int32_t *__restrict__ kf2, int npairs,
                                                      orbg_triangulation_pair *__restrict__ geo)
{
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= npairs) return;
    const orbg_kf_camera c1 = cams[kf1[p]], c2 = cams[kf2[p]];
    const float *T1 = c1.Tcw, *T2 = c2.Tcw;
    float R12[9], nR12[9];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) {
            double t = 0.0;
#pragma unroll
            for (int k = 0; k < 3; k++) t += (double)T1[4 * i + k] * (double)T2[4 * j + k];
            R12[3 * i + j] = (float)t;
            nR12[3 * i + j] = (float)(t * -1.0);
        }
    float t12[3];
#pragma unroll
    for (int i = 0; i < 3; i++) {
        double t = 0.0;
#pragma unroll
        for (int k = 0; k < 3; k++) t += (double)nR12[3 * i + k] * (double)T2[4 * k + 3];
        t += (double)T1[4 * i + 3];
        t12[i] = (float)t;
    }
    float X[9] = {0.0f, -t12[2], t12[1], t12[2], 0.0f, -t12[0], -t12[1], t12[0], 0.0f};
    const float K1t[9] = {c1.fx, 0.0f, 0.0f, 0.0f, c1.fy, 0.0f, c1.cx, c1.cy, 1.0f};
    const float K2[9] = {c2.fx, 0.0f, c2.cx, 0.0f, c2.fy, c2.cy, 0.0f, 0.0f, 1.0f};
    tri_solve3_lu(K1t, X);
    float Y[9], K2i[9], F[9], Cw1[3];
    tri_mm3(X, R12, Y);
    tri_inv3f(K2, K2i);
    tri_mm3(Y, K2i, F);
    tri_center(T1, Cw1);
    orbg_triangulation_pair g;
#pragma unroll
    for (int k = 0; k < 9; k++) g.F12[k] = F[k];
#pragma unroll
    for (int k = 0; k < 3; k++) g.Cw1[k] = Cw1[k];
#pragma unroll
    for (int k = 0; k < 12; k++) g.Tcw2[k] = T2[k];
    g.fx2 = c2.fx;
    g.fy2 = c2.fy;
    g.cx2 = c2.cx;
    g.cy2 = c2.cy;
    geo[p] = g;
}

// the null vector of the 4x4 float A (row-major) in double: cyclic Jacobi on A^T A, 12
// sweeps at most, the column of V at the least diagonal entry (orc_tri_nullvec)
__device__ void tri_nullvec(const float *A, double *v)
{
    double B[16], V[16];
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j < 4; j++) {
            double t = 0.0;
#pragma unroll
            for (int k = 0; k < 4; k++) t += (double)A[4 * k + i] * (double)A[4 * k + j];
            B[4 * i + j] = t;
            V[4 * i + j] = i == j ? 1.0 : 0.0;
        }
    for (int sweep = 0; sweep < 12; sweep++) {
        double off = 0.0;
#pragma unroll
        for (int p = 0; p < 3; p++)
#pragma unroll
            for (int q = p + 1; q < 4; q++) off += fabs(B[4 * p + q]);
        if (off == 0.0) break;
#pragma unroll
        for (int p = 0; p < 3; p++)
#pragma unroll
            for (int q = p + 1; q < 4; q++) {
                const double apq = B[4 * p + q];
                if (apq == 0.0) continue;
                const double theta = (B[4 * q + q] - B[4 * p + p]) / (2.0 * apq);
                double t = 1.0 / (fabs(theta) + sqrt(theta * theta + 1.0));
                if (theta < 0.0) t = -t;
                const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const double bkp = B[4 * k + p], bkq = B[4 * k + q];
                    B[4 * k + p] = c * bkp - s * bkq;
                    B[4 * k + q] = s * bkp + c * bkq;
                }
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const double bpk = B[4 * p + k], bqk = B[4 * q + k];
                    B[4 * p + k] = c * bpk - s * bqk;
                    B[4 * q + k] = s * bpk + c * bqk;
                }
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const double vkp = V[4 * k + p], vkq = V[4 * k + q];
                    V[4 * k + p] = c * vkp - s * vkq;
                    V[4 * k + q] = s * vkp + c * vkq;
                }
            }
    }
    int m = 0;
    double bm = B[0];
#pragma unroll
    for (int i = 1; i < 4; i++)
        if (B[4 * i + i] < bm) {
            bm = B[4 * i + i];
            m = i;
        }
#pragma unroll
    for (int k = 0; k < 4; k++) v[k] = m == 0 ? V[4 * k] : m == 1 ? V[4 * k + 1] : m == 2 ? V[4 * k + 2] : V[4 * k + 3];
}

struct TriSide {
    const orbg_kf_camera *c;
    orbg_keypoint kp;
    float ur, depth;
    const orbg_keypoint *raw;  // mvKeys[idx] (UnprojectStereo)
};

__device__ __forceinline__ int tri_level(int o) { return min(max(o, 0), ORBG_MAX_LEVELS - 1); }

// one match (orc_triangulate_one): the status, X = x3D when NEW
__device__ int tri_one(const TriSide &s1, const TriSide &s2, const float *Ow1, const float *Ow2,
                       const TriLevelTabs &L, float *X)
{
    const orbg_kf_camera &c1 = *s1.c, &c2 = *s2.c;
    const float *T1 = c1.Tcw, *T2 = c2.Tcw;
    const bool bStereo1 = s1.ur >= 0, bStereo2 = s2.ur >= 0;
    const float xn1[3] = {(s1.kp.x - c1.cx) * c1.invfx, (s1.kp.y - c1.cy) * c1.invfy, 1.0f};
    const float xn2[3] = {(s2.kp.x - c2.cx) * c2.invfx, (s2.kp.y - c2.cy) * c2.invfy, 1.0f};
    float ray1[3], ray2[3];
    tri_gemm3(T1, true, xn1, 1.0, nullptr, ray1);
    tri_gemm3(T2, true, xn2, 1.0, nullptr, ray2);
    const float cosParallaxRays =
        (float)(tri_dot3(ray1, ray2) / (sqrt(tri_dot3(ray1, ray1)) * sqrt(tri_dot3(ray2, ray2))));
    float cosParallaxStereo = cosParallaxRays + 1;
    float cosParallaxStereo1 = cosParallaxStereo, cosParallaxStereo2 = cosParallaxStereo;
    if (bStereo1)
        cosParallaxStereo1 = glibc_cosf(2 * glibc_atan2f(c1.mb / 2, s1.depth));
    else if (bStereo2)
        cosParallaxStereo2 = glibc_cosf(2 * glibc_atan2f(c2.mb / 2, s2.depth));
    cosParallaxStereo = cosParallaxStereo2 < cosParallaxStereo1 ? cosParallaxStereo2 : cosParallaxStereo1;
    float x3D[3];
    if (cosParallaxRays < cosParallaxStereo && cosParallaxRays > 0 &&
        (bStereo1 || bStereo2 || cosParallaxRays < 0.9998)) {
        float A[16];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            A[k] = (T1[8 + k] * xn1[0] + T1[k] * -1.0f) + 0.0f;
            A[4 + k] = (T1[8 + k] * xn1[1] + T1[4 + k] * -1.0f) + 0.0f;
            A[8 + k] = (T2[8 + k] * xn2[0] + T2[k] * -1.0f) + 0.0f;
            A[12 + k] = (T2[8 + k] * xn2[1] + T2[4 + k] * -1.0f) + 0.0f;
        }
        double v[4];
        tri_nullvec(A, v);
        const float vf3 = (float)v[3];
        if (vf3 == 0) return ORBG_TRI_W0;
        const float a = (float)(1.0 / (double)vf3);
#pragma unroll
        for (int k = 0; k < 3; k++) x3D[k] = (float)v[k] * a + 0.0f;
    } else if (bStereo1 && cosParallaxStereo1 < cosParallaxStereo2) {
        const float z = s1.depth;
        if (!(z > 0)) return ORBG_TRI_PARALLAX;
        const float xc[3] = {(s1.raw->x - c1.cx) * z * c1.invfx, (s1.raw->y - c1.cy) * z * c1.invfy, z};
        tri_gemm3(T1, true, xc, 1.0, Ow1, x3D);
    } else if (bStereo2 && cosParallaxStereo2 < cosParallaxStereo1) {
        const float z = s2.depth;
        if (!(z > 0)) return ORBG_TRI_PARALLAX;
        const float xc[3] = {(s2.raw->x - c2.cx) * z * c2.invfx, (s2.raw->y - c2.cy) * z * c2.invfy, z};
        tri_gemm3(T2, true, xc, 1.0, Ow2, x3D);
    } else {
        return ORBG_TRI_PARALLAX;
    }
    const float z1 = (float)(tri_dot3(&T1[8], x3D) + (double)T1[11]);
    if (z1 <= 0) return ORBG_TRI_Z1;
    const float z2 = (float)(tri_dot3(&T2[8], x3D) + (double)T2[11]);
    if (z2 <= 0) return ORBG_TRI_Z2;
    {
        const float sigmaSquare1 = L.sigma2[tri_level(s1.kp.octave)];
        const float x1 = (float)(tri_dot3(&T1[0], x3D) + (double)T1[3]);
        const float y1 = (float)(tri_dot3(&T1[4], x3D) + (double)T1[7]);
        const float invz1 = (float)(1.0 / (double)z1);
        const float u1 = c1.fx * x1 * invz1 + c1.cx;
        const float v1 = c1.fy * y1 * invz1 + c1.cy;
        const float errX1 = u1 - s1.kp.x, errY1 = v1 - s1.kp.y;
        if (!bStereo1) {
            if ((double)(errX1 * errX1 + errY1 * errY1) > 5.991 * (double)sigmaSquare1)
                return ORBG_TRI_REPROJ1;
        } else {
            const float errX1_r = (u1 - c1.mbf * invz1) - s1.ur;
            if ((double)(errX1 * errX1 + errY1 * errY1 + errX1_r * errX1_r) > 7.8 * (double)sigmaSquare1)
                return ORBG_TRI_REPROJ1;
        }
    }
    {
        const float sigmaSquare2 = L.sigma2[tri_level(s2.kp.octave)];
        const float x2 = (float)(tri_dot3(&T2[0], x3D) + (double)T2[3]);
        const float y2 = (float)(tri_dot3(&T2[4], x3D) + (double)T2[7]);
        const float invz2 = (float)(1.0 / (double)z2);
        const float u2 = c2.fx * x2 * invz2 + c2.cx;
        const float v2 = c2.fy * y2 * invz2 + c2.cy;
        const float errX2 = u2 - s2.kp.x, errY2 = v2 - s2.kp.y;
        if (!bStereo2) {
            if ((double)(errX2 * errX2 + errY2 * errY2) > 5.991 * (double)sigmaSquare2)
                return ORBG_TRI_REPROJ2;
        } else {
            // the current KeyFrame's mbf (LocalMapping.cc:528)
            const float errX2_r = (u2 - c1.mbf * invz2) - s2.ur;
            if ((double)(errX2 * errX2 + errY2 * errY2 + errX2_r * errX2_r) > 7.8 * (double)sigmaSquare2)
                return ORBG_TRI_REPROJ2;
        }
    }
    const float n1[3] = {x3D[0] - Ow1[0], x3D[1] - Ow1[1], x3D[2] - Ow1[2]};
    const float n2[3] = {x3D[0] - Ow2[0], x3D[1] - Ow2[1], x3D[2] - Ow2[2]};
    const float dist1 = (float)sqrt(tri_dot3(n1, n1)), dist2 = (float)sqrt(tri_dot3(n2, n2));
    if (dist1 == 0 || dist2 == 0) return ORBG_TRI_DIST0;
    const float ratioDist = dist2 / dist1;
    const float ratioOctave = L.scale[tri_level(s1.kp.octave)] / L.scale[tri_level(s2.kp.octave)];
    if (ratioDist * L.ratio < ratioOctave || ratioDist > ratioOctave * L.ratio) return ORBG_TRI_SCALE;
    X[0] = x3D[0];
    X[1] = x3D[1];
    X[2] = x3D[2];
    return ORBG_TRI_NEW;
}

__global__ __launch_bounds__(256) void k_triangulate(orbg_keyframes K,
                                                     const orbg_keypoint *__restrict__ kps_raw,
                                                     const float *__restrict__ depth, int cap,
                                                     const orbg_kf_camera *__restrict__ cams,
                                                     const int32_t *__restrict__ kf1,
                                                     const int32_t *__restrict__ kf2,
                                                     const int32_t *__restrict__ m12,
                                                     TriLevelTabs L, float *__restrict__ x3d,
                                                     int8_t *__restrict__ status,
                                                     int32_t *__restrict__ nnew)
{
    const int p = blockIdx.y, i = blockIdx.x * 256 + threadIdx.x;
    const int a = kf1[p], b = kf2[p];
    const int n1 = min(max(K.counts[a], 0), cap), n2 = min(max(K.counts[b], 0), cap);
    if (blockIdx.x * 256 >= n1) return;  // uniform per workgroup
    int st = ORBG_TRI_NONE;
    float X[3] = {0.0f, 0.0f, 0.0f};
    const size_t o = (size_t)p * cap + i;
    if (i < n1) {
        const int j = m12[o];
        if (j >= 0 && j < n2) {
            const size_t ia = (size_t)a * cap + i, jb = (size_t)b * cap + j;
            TriSide s1, s2;
            s1.c = cams + a;
            s2.c = cams + b;
            s1.kp = K.kps[ia];
            s2.kp = K.kps[jb];
            s1.ur = K.uright ? K.uright[ia] : -1.0f;
            s2.ur = K.uright ? K.uright[jb] : -1.0f;
            s1.depth = (s1.ur >= 0) ? depth[ia] : 0.0f;
            s2.depth = (s2.ur >= 0) ? depth[jb] : 0.0f;
            s1.raw = kps_raw ? kps_raw + ia : K.kps + ia;
            s2.raw = kps_raw ? kps_raw + jb : K.kps + jb;
            float Ow1[3], Ow2[3];
            tri_center(s1.c->Tcw, Ow1);
            tri_center(s2.c->Tcw, Ow2);
            st = tri_one(s1, s2, Ow1, Ow2, L, X);
        }
        status[o] = (int8_t)st;
        x3d[3 * o] = X[0];
        x3d[3 * o + 1] = X[1];
        x3d[3 * o + 2] = X[2];
    }
    const unsigned long long bal = __ballot(st == ORBG_TRI_NEW);
    if ((threadIdx.x & 63) == 0 && bal) atomicAdd(nnew + p, (int)__popcll(bal));
}

int launch_tri_geometry(hipStream_t st, const orbg_kf_camera *cams, const int32_t *kf1,
                        const int32_t *kf2, int npairs, orbg_triangulation_pair *geo)
{
    if (npairs <= 0) return 0;
    hipLaunchKernelGGL(k_tri_geometry, dim3((npairs + 255) / 256), dim3(256), 0, st, cams, kf1,
                       kf2, npairs, geo);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

int launch_triangulate(hipStream_t st, const orbg_keyframes &K, const orbg_keypoint *kps_raw,
                       const float *depth, int cap, const orbg_kf_camera *cams, const int32_t *kf1,
                       const int32_t *kf2, const int32_t *m12, int npairs, const float *scale,
                       const float *sigma2, int nlevels, float scale_factor, float *x3d,
                       int8_t *status, int32_t *nnew)
{
    if (npairs <= 0) return 0;
    if (npairs > 65535) return -22;
    if (hipMemsetAsync(nnew, 0, (size_t)npairs * sizeof(int32_t), st) != hipSuccess) return -5;
    TriLevelTabs L{};
    for (int l = 0; l < ORBG_MAX_LEVELS; l++) {
        const int s = l < nlevels ? l : nlevels - 1;
        L.scale[l] = scale[s];
        L.sigma2[l] = sigma2[s];
    }
    L.ratio = 1.5f * scale_factor;
    hipLaunchKernelGGL(k_triangulate, dim3((cap + 255) / 256, npairs), dim3(256), 0, st, K,
                       kps_raw, depth, cap, cams, kf1, kf2, m12, L, x3d, status, nnew);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

}  // namespace orbg
