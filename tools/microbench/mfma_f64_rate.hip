// mfma_f64_rate.hip -- issue rate of gfx950's two f64 MFMA shapes, one wave per SIMD on every
// CU, 4 independent accumulators per wave (the BA pose-block pass chooses between them):
//   v_mfma_f64_16x16x4f64   (one 16x16 block, K = 4: 2048 FLOP)
//   v_mfma_f64_4x4x4f64     (four 4x4 blocks, K = 4: 512 FLOP)
// hipcc --offload-arch=gfx950 -O3 mfma_f64_rate.hip -o mfma_f64_rate && ./mfma_f64_rate
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double v4d __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k16(double *out, int iters, double a0)
{
    double a = a0 + threadIdx.x * 1e-9, b = a0 - threadIdx.x * 1e-9;
    v4d c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    for (int i = 0; i < iters; i++) {
        c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
    }
    out[blockIdx.x * 256 + threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
}

__global__ __launch_bounds__(256) void k4(double *out, int iters, double a0)
{
    double a = a0 + threadIdx.x * 1e-9, b = a0 - threadIdx.x * 1e-9;
    double c0 = 0, c1 = 0, c2 = 0, c3 = 0;
    for (int i = 0; i < iters; i++) {
        c0 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c3, 0, 0, 0);
    }
    out[blockIdx.x * 256 + threadIdx.x] = c0 + c1 + c2 + c3;
}

// one wave per SIMD, a single dependent chain: the latency
__global__ __launch_bounds__(64) void k4_chain(double *out, int iters, double a0)
{
    double a = a0 + threadIdx.x * 1e-9, b = a0 - threadIdx.x * 1e-9, c = 0;
    for (int i = 0; i < iters; i++) c = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
    out[blockIdx.x * 64 + threadIdx.x] = c;
}
__global__ __launch_bounds__(64) void k16_chain(double *out, int iters, double a0)
{
    double a = a0 + threadIdx.x * 1e-9, b = a0 - threadIdx.x * 1e-9;
    v4d c = {0, 0, 0, 0};
    for (int i = 0; i < iters; i++) c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    out[blockIdx.x * 64 + threadIdx.x] = c[0];
}

// 4x4x4 block layout probe: A = lane id, B = 1 -> which lanes' A values sum into each C lane
__global__ void k4_layout(double *out)
{
    const int l = threadIdx.x;
    const double a = (double)(1ull << (l % 16)) + 65536.0 * (l / 16);
    double c = __builtin_amdgcn_mfma_f64_4x4x4f64(a, 1.0, 0.0, 0, 0, 0);
    out[l] = c;
    double c2 = __builtin_amdgcn_mfma_f64_4x4x4f64(1.0, a, 0.0, 0, 0, 0);
    out[64 + l] = c2;
}

int main()
{
    double *d;
    hipMalloc(&d, 1 << 24);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 4096, cus = 256;
    float ms;
    for (int rep = 0; rep < 2; rep++) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(k16, dim3(cus), dim3(256), 0, 0, d, iters, 1.0);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        double fl = 2048.0 * 4 * iters * cus * 4;
        printf("16x16x4f64: %.3f ms  %.1f TFLOP/s  %.2f cyc/instr/SIMD @2.4GHz\n", ms, fl / ms / 1e9,
               ms * 1e-3 * 2.4e9 / (4.0 * iters));
        hipEventRecord(e0);
        hipLaunchKernelGGL(k4, dim3(cus), dim3(256), 0, 0, d, iters, 1.0);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        fl = 512.0 * 4 * iters * cus * 4;
        printf("4x4x4f64:   %.3f ms  %.1f TFLOP/s  %.2f cyc/instr/SIMD @2.4GHz\n", ms, fl / ms / 1e9,
               ms * 1e-3 * 2.4e9 / (4.0 * iters));
        hipEventRecord(e0);
        hipLaunchKernelGGL(k4_chain, dim3(cus * 4), dim3(64), 0, 0, d, iters, 1.0);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        printf("4x4x4f64 dependent chain: %.2f cyc/instr\n", ms * 1e-3 * 2.4e9 / iters);
        hipEventRecord(e0);
        hipLaunchKernelGGL(k16_chain, dim3(cus * 4), dim3(64), 0, 0, d, iters, 1.0);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        printf("16x16x4f64 dependent chain: %.2f cyc/instr\n", ms * 1e-3 * 2.4e9 / iters);
    }
    hipLaunchKernelGGL(k4_layout, dim3(1), dim3(64), 0, 0, d);
    double h[128];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("layout A=lane-code,B=1:");
    for (int l = 0; l < 64; l++) printf(" %d:%.0f", l, h[l]);
    printf("\nlayout A=1,B=lane-code:");
    for (int l = 0; l < 64; l++) printf(" %d:%.0f", l, h[64 + l]);
    printf("\n");
    return 0;
}
