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

__device__ __forceinline__ int wave_sum(int x)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}

}  // namespace orbg
