// valu_rate.hip -- issue rate of the VALU instructions the hot kernels lean on (gfx950).
// 8 waves/SIMD of 8 independent dependency chains each; reports cycles per wave64
// instruction per SIMD.   hipcc --offload-arch=gfx950 -O3 valu_rate.hip -o valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>

typedef short v2s __attribute__((ext_vector_type(2)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));

#define N_IT 4096

template <int OP>
__global__ __launch_bounds__(256) void k(uint32_t *out, uint32_t seed)
{
    uint32_t r[8];
#pragma unroll
    for (int i = 0; i < 8; i++) r[i] = seed * (threadIdx.x + 1) + i * 0x9E3779B9u;
    for (int it = 0; it < N_IT; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            uint32_t a = r[i], b = r[(i + 1) & 7], c = r[(i + 2) & 7];
            if (OP == 0) {
                asm volatile("v_add_u32 %0, %1, %2" : "=v"(a) : "v"(a), "v"(b));
            } else if (OP == 1) {
                asm volatile("v_pk_max_i16 %0, %1, %2" : "=v"(a) : "v"(a), "v"(b));
            } else if (OP == 2) {
                asm volatile("v_pk_maximum3_f16 %0, %1, %2, %3" : "=v"(a) : "v"(a), "v"(b), "v"(c));
            } else if (OP == 3) {
                asm volatile("v_perm_b32 %0, %1, %2, %3" : "=v"(a) : "v"(a), "v"(b), "v"(c));
            } else if (OP == 4) {
                asm volatile("v_bcnt_u32_b32 %0, %1, %2" : "=v"(a) : "v"(a), "v"(b));
            } else if (OP == 5) {
                asm volatile("v_xor_b32 %0, %1, %2" : "=v"(a) : "v"(a), "v"(b));
            } else if (OP == 6) {
                asm volatile("v_pk_mad_u16 %0, %1, %2, %3" : "=v"(a) : "v"(a), "v"(b), "v"(c));
            } else if (OP == 7) {
                asm volatile("v_max3_u32 %0, %1, %2, %3" : "=v"(a) : "v"(a), "v"(b), "v"(c));
            }
            r[i] = a;
        }
    }
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) x ^= r[i];
    out[blockIdx.x * 256 + threadIdx.x] = x;
}

template <int OP>
static void run(const char *name, uint32_t *d, int blocks)
{
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, 1u);
    hipEventRecord(a);
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, 2u);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    int dev, clk, cus;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);  // kHz
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const double waves = blocks * 4.0, instr = waves * N_IT * 8;
    const double simd_cycles = ms * 1e-3 * clk * 1e3 * cus * 4;
    printf("%-20s %.2f cycles per wave64 instruction per SIMD (%.3f ms, clock %d MHz)\n", name,
           simd_cycles / instr, ms, clk / 1000);
}

int main()
{
    uint32_t *d;
    int dev, cus;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int blocks = cus * 8;  // 8 waves per SIMD
    hipMalloc(&d, (size_t)blocks * 256 * 4);
    run<0>("v_add_u32", d, blocks);
    run<1>("v_pk_max_i16", d, blocks);
    run<2>("v_pk_maximum3_f16", d, blocks);
    run<3>("v_perm_b32", d, blocks);
    run<4>("v_bcnt_u32_b32", d, blocks);
    run<5>("v_xor_b32", d, blocks);
    run<6>("v_pk_mad_u16", d, blocks);
    run<7>("v_max3_u32", d, blocks);
    hipFree(d);
    return 0;
}
