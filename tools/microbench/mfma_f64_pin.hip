// mfma_f64_pin.hip -- the exact arithmetic of v_mfma_f64_4x4x4f64 (pins the Schur solve's
// oracle order, oracle/ba_oracle.c): random operands with wide exponent ranges, every C
// element compared bitwise against host emulations of the K = 4 reduction:
//   chain  : c = fma(a3,b3, fma(a2,b2, fma(a1,b1, fma(a0,b0,c))))   (k ascending)
//   rchain : the same, k descending
//   prod   : c + ((p0 + p1) + (p2 + p3)), products rounded
//   exact  : the exact sum rounded once (long double approximation, flagged by mismatch)
// hipcc --offload-arch=gfx950 -O3 mfma_f64_pin.hip -o mfma_f64_pin && ./mfma_f64_pin
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

__global__ void k4(const double *A, const double *B, const double *C, double *D, int n)
{
    const int w = blockIdx.x, l = threadIdx.x;
    if (w >= n) return;
    double c = __builtin_amdgcn_mfma_f64_4x4x4f64(A[64 * w + l], B[64 * w + l], C[64 * w + l], 0, 0, 0);
    D[64 * w + l] = c;
}

static bool same(double a, double b) { return memcmp(&a, &b, 8) == 0; }

int main()
{
    const int n = 20000;  // waves
    std::vector<double> A(64 * n), B(64 * n), C(64 * n), D(64 * n);
    std::mt19937_64 g(7);
    std::uniform_real_distribution<double> u(-1, 1);
    std::uniform_int_distribution<int> ex(-30, 30);
    for (size_t i = 0; i < A.size(); i++) {
        A[i] = std::ldexp(u(g), ex(g) / 3);
        B[i] = std::ldexp(u(g), ex(g) / 3);
        C[i] = std::ldexp(u(g), ex(g));
    }
    double *dA, *dB, *dC, *dD;
    hipMalloc(&dA, A.size() * 8);
    hipMalloc(&dB, A.size() * 8);
    hipMalloc(&dC, A.size() * 8);
    hipMalloc(&dD, A.size() * 8);
    hipMemcpy(dA, A.data(), A.size() * 8, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), A.size() * 8, hipMemcpyHostToDevice);
    hipMemcpy(dC, C.data(), A.size() * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k4, dim3(n), dim3(64), 0, 0, dA, dB, dC, dD, n);
    hipMemcpy(D.data(), dD, A.size() * 8, hipMemcpyDeviceToHost);
    long m_chain = 0, m_rchain = 0, m_prod = 0, m_exact = 0, tot = 0;
    for (int w = 0; w < n; w++)
        for (int l = 0; l < 64; l++) {
            // C[b][i][j] at lane 16 i + 4 b + j; A[b][i][k] at 16 k + 4 b + i; B[b][k][j] at 16 k + 4 b + j
            const int i = l >> 4, b = (l >> 2) & 3, j = l & 3;
            double a[4], bb[4];
            for (int k = 0; k < 4; k++) {
                a[k] = A[64 * w + 16 * k + 4 * b + i];
                bb[k] = B[64 * w + 16 * k + 4 * b + j];
            }
            const double c = C[64 * w + l], d = D[64 * w + l];
            double x = c;
            for (int k = 0; k < 4; k++) x = std::fma(a[k], bb[k], x);
            double y = c;
            for (int k = 3; k >= 0; k--) y = std::fma(a[k], bb[k], y);
            const double p = c + ((a[0] * bb[0] + a[1] * bb[1]) + (a[2] * bb[2] + a[3] * bb[3]));
            long double e = (long double)c;
            for (int k = 0; k < 4; k++) e += (long double)a[k] * (long double)bb[k];
            m_chain += same(x, d);
            m_rchain += same(y, d);
            m_prod += same(p, d);
            m_exact += same((double)e, d);
            tot++;
        }
    printf("4x4x4f64 bitwise matches of %ld: chain %ld rchain %ld prod %ld exact(long double) %ld\n",
           tot, m_chain, m_rchain, m_prod, m_exact);
    return 0;
}
