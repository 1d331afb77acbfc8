// fast_device.h -- FAST-9 device helpers of k_fast2 (fast_kernels.hip): packed u16
// pixel-pair gathers and the cornerScore<16> arc
// extremes (cv::FAST TYPE_9_16).
#pragma once

#include <hip/hip_runtime.h>

#include <type_traits>

#pragma clang fp contract(off)

namespace orbg {

// ---------------------------------------------------------------------------
// FAST-9 score (cornerScore<16> semantics): s = M - 1, M = max over the 16 contiguous
// 9-arcs of the circle of max(min d, min -d), d = centre - circle pixel.  "Corner at
// threshold th" <=> s >= th; the score is stored as u8 max(s, 0) (0 = no corner or score
// 0, which FAST's NMS treats identically: it keeps a pixel only if score > 0-filled
// neighbours).  Two pixels per register: u8 -> u16 lanes with v_perm_b32, then
// v_pk_sub/min/max_i16.  Arc minima use OpenCV's structure: for even k the 8-run
// d[k+1..k+8] extended by d[k] or d[k+9] (all 16 starts).
// ---------------------------------------------------------------------------
typedef short v2s __attribute__((ext_vector_type(2)));

__device__ __forceinline__ v2s pmin(v2s a, v2s b) { return __builtin_elementwise_min(a, b); }
__device__ __forceinline__ v2s pmax(v2s a, v2s b) { return __builtin_elementwise_max(a, b); }

// bytes OFF and OFF+1 of the 12-byte window {w0, w1, w2} as two zero-extended u16 lanes
template <int OFF>
__device__ __forceinline__ v2s gather2(uint32_t w0, uint32_t w1, uint32_t w2)
{
    static_assert(OFF >= 0 && OFF + 1 < 12, "window");
    uint32_t r;
    // a word none of whose bytes is selected is not passed (so its LDS load is dead code)
    if (OFF + 1 < 4) {
        r = __builtin_amdgcn_perm(w0, w0, 0x0c000c00u | (OFF + 1) << 16 | OFF);
    } else if (OFF >= 4 && OFF + 1 < 8) {
        r = __builtin_amdgcn_perm(w1, w1, 0x0c000c00u | (OFF - 3) << 16 | (OFF - 4));
    } else if (OFF >= 8) {
        r = __builtin_amdgcn_perm(w2, w2, 0x0c000c00u | (OFF - 7) << 16 | (OFF - 8));
    } else if (OFF == 3) {  // straddles w0 / w1
        r = __builtin_amdgcn_perm(w1, w0, 0x0c040c03u);
    } else {  // OFF == 7: straddles w1 / w2
        r = __builtin_amdgcn_perm(w2, w1, 0x0c040c03u);
    }
    return __builtin_bit_cast(v2s, r);
}

struct Rows7 {
    uint32_t w[7][3];
};

// Arc extrema use gfx950's 3-input packed v_pk_maximum3_f16 / v_pk_minimum3_f16: the u16
// lanes (values 0..255) are read as f16 bit patterns, i.e. +0 and positive denormals,
// whose IEEE order is the integer order (f16 denormals are preserved; nothing is
// computed in f16, only ordered).
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ h2 hmax3(h2 a, h2 b, h2 c)
{
    return __builtin_elementwise_maximum(__builtin_elementwise_maximum(a, b), c);
}
__device__ __forceinline__ h2 hmin3(h2 a, h2 b, h2 c)
{
    return __builtin_elementwise_minimum(__builtin_elementwise_minimum(a, b), c);
}
__device__ __forceinline__ h2 as_h2(v2s v) { return __builtin_bit_cast(h2, v); }
__device__ __forceinline__ v2s as_v2s(h2 v) { return __builtin_bit_cast(v2s, v); }

// bytes OFF + s and OFF + s + 1 of the 12-byte window {w0, w1, w2}, s = 0 or 2 per lane,
// as two zero-extended u16 lanes: one v_perm_b32 whose selector is sel[OFF] = the s = 0
// selector + (s, s) in its two index bytes (the caller adds s once per task).  OFF <= 4
// picks from w0:w1 (bytes OFF + s + 1 <= 7), OFF >= 5 from w1:w2 (bytes 5 .. 9).
template <int OFF>
__device__ __forceinline__ constexpr uint32_t gather2_rt_sel()
{
    static_assert(OFF >= 0 && OFF <= 6, "window");
    return OFF <= 4 ? (0x0c000c00u | (uint32_t)(OFF + 1) << 16 | (uint32_t)OFF)
                    : (0x0c000c00u | (uint32_t)(OFF - 3) << 16 | (uint32_t)(OFF - 4));
}
template <int OFF>
__device__ __forceinline__ v2s gather2_rt(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t sel)
{
    const uint32_t r = OFF <= 4 ? __builtin_amdgcn_perm(w1, w0, sel) : __builtin_amdgcn_perm(w2, w1, sel);
    return __builtin_bit_cast(v2s, r);
}

// One side of the score of two pixels, the bright side: M = max_k min(x[k .. k+8]) - v, u8
// score max(M - 1, 0).  The dark side is the bright side of the complemented pixels
// (255 - x and 255 - v: v - min_k max(x[k .. k+8]) = max_k min(255 - x) - (255 - v)), so
// callers pass `flip` = 0xFFFFFFFF to complement the raw window bytes.  The 16 arc minima
// are paired: for even k, max(a_k, a_{k+1}) = min(l_{k+1}, max(x_k, x_{k+9})) with
// l_j = min(x[j .. j+7]) built from pairs and quads (8 + 8 ops) -- 36 packed ops per side
// instead of 40.  A pixel is never a corner on both sides at one threshold (9 + 9 > 16
// circle pixels), so the side below threshold contributes nothing: its true score is < th.
// Pixel pair s / 2 (s = 0: pixels 0-1, s = 2: pixels 2-3) of the unit whose rows R hold
// window bytes 0 .. 11 (pixel 0 at byte 3), s per lane: the seven selectors
// gather2_rt_sel<0..6>() + (s, s) are built once per task.  circle (dx, dy) of
// makeOffsets(16): row index = 3 + dy, byte offset = 3 + dx (+ pixel i).
__device__ __forceinline__ v2s fast_score_side_rt(const Rows7 &R, uint32_t sadd)
{
    uint32_t sel[7];
    sel[0] = gather2_rt_sel<0>() + sadd;
    sel[1] = gather2_rt_sel<1>() + sadd;
    sel[2] = gather2_rt_sel<2>() + sadd;
    sel[3] = gather2_rt_sel<3>() + sadd;
    sel[4] = gather2_rt_sel<4>() + sadd;
    sel[5] = gather2_rt_sel<5>() + sadd;
    sel[6] = gather2_rt_sel<6>() + sadd;
#define GB(row, dx) as_h2(gather2_rt<3 + (dx)>(R.w[row][0], R.w[row][1], R.w[row][2], sel[3 + (dx)]))
    const v2s v = gather2_rt<3>(R.w[3][0], R.w[3][1], R.w[3][2], sel[3]);
    h2 x[16];
    x[0] = GB(6, 0);
    x[1] = GB(6, 1);
    x[2] = GB(5, 2);
    x[3] = GB(4, 3);
    x[4] = GB(3, 3);
    x[5] = GB(2, 3);
    x[6] = GB(1, 2);
    x[7] = GB(0, 1);
    x[8] = GB(0, 0);
    x[9] = GB(0, -1);
    x[10] = GB(1, -2);
    x[11] = GB(2, -3);
    x[12] = GB(3, -3);
    x[13] = GB(4, -3);
    x[14] = GB(5, -2);
    x[15] = GB(6, -1);
#undef GB
    h2 p[8], q[8], m[8];
#pragma unroll
    for (int j = 0; j < 8; j++) p[j] = __builtin_elementwise_minimum(x[2 * j + 1], x[(2 * j + 2) & 15]);
#pragma unroll
    for (int j = 0; j < 8; j++) q[j] = __builtin_elementwise_minimum(p[j], p[(j + 1) & 7]);
#pragma unroll
    for (int j = 0; j < 8; j++)
        m[j] = hmin3(q[j], q[(j + 2) & 7], __builtin_elementwise_maximum(x[2 * j], x[(2 * j + 9) & 15]));
    const h2 amax = __builtin_elementwise_maximum(
        hmax3(hmax3(m[0], m[1], m[2]), hmax3(m[3], m[4], m[5]), m[6]), m[7]);
    const v2s zero = (v2s){0, 0}, one = (v2s){1, 1};
    return pmax(as_v2s(amax) - v - one, zero);
}

}  // namespace orbg
