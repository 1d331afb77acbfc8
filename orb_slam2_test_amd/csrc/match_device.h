// match_device.h -- device helpers shared by the matcher kernels (match_kernels.hip,
// track_kernels.hip): Hamming distance, the Frame grid window of GetFeaturesInArea
// (Frame.cc:421-504) and its candidate enumeration order.
#pragma once

#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

#include "../../include/orbg.h"
#include "orbg_internal.h"

#pragma clang fp contract(off)

namespace orbg {

__device__ __forceinline__ int wave_isum(int x)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}

__device__ __forceinline__ int hamming8(const uint32_t a[8], const uint32_t *b)
{
    int d = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) d += __popc(a[i] ^ b[i]);
    return d;
}

struct GridPrm {
    float min_x, min_y, inv_w, inv_h;
};

__device__ __forceinline__ GridPrm grid_prm(orbg_bounds b)
{
    GridPrm g;
    g.min_x = b.min_x;
    g.min_y = b.min_y;
    // Frame.cc:273-274
    g.inv_w = (float)ORBG_GRID_COLS / (float)(b.max_x - b.min_x);
    g.inv_h = (float)ORBG_GRID_ROWS / (float)(b.max_y - b.min_y);
    return g;
}

struct Window {
    int cx0, cx1, cy0, cy1;
    float x, y, r;
    bool empty;
};

// GetFeaturesInArea's cell range (Frame.cc:446-460)
__device__ __forceinline__ Window make_window(const GridPrm &g, float x, float y, float r)
{
    Window w;
    w.x = x;
    w.y = y;
    w.r = r;
    w.cx0 = max(0, (int)floorf((x - g.min_x - r) * g.inv_w));
    w.cx1 = min(ORBG_GRID_COLS - 1, (int)ceilf((x - g.min_x + r) * g.inv_w));
    w.cy0 = max(0, (int)floorf((y - g.min_y - r) * g.inv_h));
    w.cy1 = min(ORBG_GRID_ROWS - 1, (int)ceilf((y - g.min_y + r) * g.inv_h));
    w.empty = w.cx0 >= ORBG_GRID_COLS || w.cx1 < 0 || w.cy0 >= ORBG_GRID_ROWS || w.cy1 < 0;
    return w;
}

// candidate test for key (kx, ky, octave 0) with grid position (PosInGrid, round()).
// returns the grid-enumeration order key (cell major: ix, iy) or -1
__device__ __forceinline__ int cand_order(const GridPrm &g, const Window &w, float kx, float ky)
{
    const int px = (int)roundf((kx - g.min_x) * g.inv_w);
    const int py = (int)roundf((ky - g.min_y) * g.inv_h);
    if (px < 0 || px >= ORBG_GRID_COLS || py < 0 || py >= ORBG_GRID_ROWS) return -1;
    if (px < w.cx0 || px > w.cx1 || py < w.cy0 || py > w.cy1) return -1;
    const float dx = kx - w.x, dy = ky - w.y;
    if (!(fabsf(dx) < w.r && fabsf(dy) < w.r)) return -1;
    return px * ORBG_GRID_ROWS + py;
}

__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long u = __shfl_xor(v, o, 64);
        v = u < v ? u : v;
    }
    return v;
}


}  // namespace orbg
