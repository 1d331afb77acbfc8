// orbg_device.h -- small wave64 helpers shared by the kernel translation units.
#pragma once

#include <hip/hip_runtime.h>

namespace orbg {

__device__ __forceinline__ int wave_incl_scan(int x)
{
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    return x;
}

// inclusive wave prefix of small counts 0 <= x < 8 from three ballots (no shuffles);
// *total = wave total
__device__ __forceinline__ int wave_incl_scan_small(int x, int *total)
{
    int incl = 0, tot = 0;
#pragma unroll
    for (int b = 0; b < 3; b++) {
        const unsigned long long m = __ballot((x >> b) & 1);
        const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
        incl += (below + ((x >> b) & 1)) << b;
        tot += __popcll(m) << b;
    }
    *total = tot;
    return incl;
}

__device__ __forceinline__ int wave_sum(int x)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}

// LDS written by some lanes of a wave, then read by others: keep the compiler from
// reordering (the hardware keeps one wave's LDS ops in order).
__device__ __forceinline__ void wave_sync_lds()
{
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// XCD-aware block remap (cdna_hip_programming.md T1, bijective for nwg % 8 != 0).
// The dispatcher deals workgroups round-robin over the 8 XCDs (orig % 8 shares an L2);
// the remap hands each XCD a contiguous run of logical blocks, so neighbouring cells /
// tiles / keypoints of one frame (which share halo lines and pyramid levels) hit in the
// same 4 MiB L2 instead of being fetched once per XCD.  Speed only, never correctness.
__device__ __forceinline__ int xcd_remap(int orig, int nwg)
{
    const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

}  // namespace orbg
