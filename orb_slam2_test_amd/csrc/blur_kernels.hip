// blur_kernels.hip -- k_blur2: GaussianBlur(7x7, sigma 2, BORDER_REFLECT_101) of every pyramid
// level (ORBextractor.cc:1375-1377, cv::GaussianBlur 8U bit-exact fixed point:
// out = sat((sum_v k_v * sum_h k_h * p + 2^15) >> 16)), same bytes as k_blur
// (extract_kernels.hip), without LDS and without workgroup barriers.
//
// One wave owns a 256-column x SEG-row output tile of one (frame, level); lane j owns columns
// gx .. gx+3 (gx = tile x + 4j) and walks the SEG + 6 input rows top to bottom:
//   row pass   the 12 source bytes gx-4 .. gx+7 of the row (one dwordx4 + v_alignbyte) against
//              byte-shifted weight words: ten v_dot4_u32_u8 give the four row sums s (<= 256 * 255);
//   column     a register window over the last rows: P[r] = s[r] | s[r+1] << 16 per column, and
//              output row o = dot2(P[o], (k0,k1)) + dot2(P[o+2], (k2,k3)) + dot2(P[o+4], (k4,k5))
//              + k6 * s[o+6], the rounding term 2^15 as the chain's start value;
//   store      with weights summing to 256 the output is byte 2 of the sum: four pixels packed by
//              two v_perm, one dword store (legacy 257-sum weights saturate instead).
// Source rows are loaded ROWPF rows ahead (a register ring).  The rows above / below the level
// reflect (wave-uniform); lanes whose 12-byte window leaves the row gather bytes with
// REFLECT_101 (the two ends of a row only).  Every wave is independent: no LDS, no barrier.
#include <hip/hip_runtime.h>

#include "orbg_internal.h"
#include "orbg_device.h"

#pragma clang fp contract(off)

namespace orbg {

#ifndef ORBG_BLUR2_DPP
#define ORBG_BLUR2_DPP 1  // one dword per lane per row, neighbours by DPP wave shifts
#endif
// output columns per wave (4 per lane): with DPP the last 3 lanes only supply their dwords
#define BLUR2_TW (ORBG_BLUR2_DPP ? 244 : 256)
#ifndef ORBG_BLUR2_SEG
#define ORBG_BLUR2_SEG 32  // output rows per k_blur2 wave
#endif
#ifndef ORBG_BLUR2_EPF
#define ORBG_BLUR2_EPF 2  // edge-lane source rows in flight (51 VGPRs; 4: 65)
#endif
#ifndef ORBG_BLUR2_ROWPF
#define ORBG_BLUR2_ROWPF 8  // source rows in flight per lane
#endif

__device__ __forceinline__ uint32_t b2_udot2(uint32_t a, uint32_t b, uint32_t c)
{
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    return __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b), c,
                                  false);
}

__device__ __forceinline__ int b2_reflect101(int i, int n)
{
    i = i < 0 ? -i : i;
    return i >= n ? 2 * n - 2 - i : i;
}

// The row / column arithmetic of one 4-column group over SEG output rows.  Loader(i, w0, w1,
// w2) yields the 12 window bytes gx-4 .. gx+7 of source row i (image row y0 - 3 + i); Store(o,
// word) stores output row y0 + o.
struct Blur2Weights {
    uint32_t K00, K01, K10, K11, K12, K20, K21, K22, K31, K32, E0, E1, E2, k6, c0;
    bool norm256;
    __device__ Blur2Weights(const OrbgGeom *g)
    {
        const uint32_t k0 = g->gk[0], k1 = g->gk[1], k2 = g->gk[2], k3 = g->gk[3],
                       k4 = g->gk[4], k5 = g->gk[5];
        k6 = g->gk[6];
        norm256 = k0 + k1 + k2 + k3 + k4 + k5 + k6 == 256u;
        // row pass weight words (as k_blur): output x = gx + i needs window bytes 1+i .. 7+i
        K00 = k0 << 8 | k1 << 16 | k2 << 24;
        K01 = k3 | k4 << 8 | k5 << 16 | k6 << 24;
        K10 = k0 << 16 | k1 << 24;
        K11 = k2 | k3 << 8 | k4 << 16 | k5 << 24;
        K12 = k6;
        K20 = k0 << 24;
        K21 = k1 | k2 << 8 | k3 << 16 | k4 << 24;
        K22 = k5 | k6 << 8;
        K31 = k0 | k1 << 8 | k2 << 16 | k3 << 24;
        K32 = k4 | k5 << 8 | k6 << 16;
        E0 = k0 | k1 << 16;
        E1 = k2 | k3 << 16;
        E2 = k4 | k5 << 16;
        c0 = norm256 ? (1u << 15) : 0u;
    }
};

template <int SEG, typename Loader, typename Store>
__device__ __forceinline__ void blur2_column(const Blur2Weights &k, Loader &&load, Store &&store)
{
    constexpr int NR = SEG + 6;
    uint32_t s[NR][4];  // row sums (fully unrolled: only the live window stays in registers)
    uint32_t P[NR][4];  // P[r] = s[r] | s[r+1] << 16
#pragma unroll
    for (int i = 0; i < NR; i++) {
        uint32_t w0, w1, w2;
        load(i, w0, w1, w2);
        s[i][0] = __builtin_amdgcn_udot4(w1, k.K01, __builtin_amdgcn_udot4(w0, k.K00, 0u, false), false);
        s[i][1] = __builtin_amdgcn_udot4(w2, k.K12, __builtin_amdgcn_udot4(w1, k.K11, __builtin_amdgcn_udot4(w0, k.K10, 0u, false), false), false);
        s[i][2] = __builtin_amdgcn_udot4(w2, k.K22, __builtin_amdgcn_udot4(w1, k.K21, __builtin_amdgcn_udot4(w0, k.K20, 0u, false), false), false);
        s[i][3] = __builtin_amdgcn_udot4(w2, k.K32, __builtin_amdgcn_udot4(w1, k.K31, 0u, false), false);
        if (i >= 1) {
#pragma unroll
            for (int c = 0; c < 4; c++) P[i - 1][c] = s[i - 1][c] | s[i][c] << 16;
        }
        if (i >= 6) {
            const int o = i - 6;
            uint32_t a[4];
#pragma unroll
            for (int c = 0; c < 4; c++) {
                uint32_t v = b2_udot2(P[o][c], k.E0, k.c0);
                v = b2_udot2(P[o + 2][c], k.E1, v);
                v = b2_udot2(P[o + 4][c], k.E2, v);
                a[c] = __umul24(k.k6, s[o + 6][c]) + v;  // v_mad_u32_u24
            }
            uint32_t word;
            if (k.norm256) {
                // byte 2 of each sum (the output, no saturation possible): two v_perm
                word = __builtin_amdgcn_perm(a[1], a[0], 0x0c0c0602u) |
                       __builtin_amdgcn_perm(a[3], a[2], 0x06020c0cu);
            } else {
                word = 0;
#pragma unroll
                for (int c = 0; c < 4; c++) word |= min((a[c] + (1u << 15)) >> 16, 255u) << (8 * c);
            }
            store(o, word);
        }
    }
}

__device__ __forceinline__ void blur2_store(uint8_t *dst, int pitch, int W, int H, int gx, int gy,
                                            uint32_t word)
{
    if (gy >= H || gx >= W) return;
    uint8_t *d = dst + (int64_t)gy * pitch + gx;
    if (gx + 4 <= W) {
        *(uint32_t *)d = word;  // pitch is a multiple of 64, gx of 4: aligned
    } else {
        for (int c = 0; c < 4 && gx + c < W; c++) d[c] = (uint8_t)(word >> (8 * c));
    }
}

// k_blur2: after the edge waves (blur2_edge_lane), wave w is a tile (frame-major, then the
// tiles [t_begin, t_begin + t_count) in level order, BLUR2_TW x SEG each); its lanes whose
// window gx-4 .. gx+11 leaves the row skip their stores (the edge lanes' columns).
#define BLUR2_ECOLS 16  // k_blur2_edge column slots per row segment (4 left, 12 right)
#define BLUR2_EROWS 8   // output rows per k_blur2_edge lane
#define BLUR2_NEG (BLUR2_ECOLS * (ORBG_BLUR2_SEG / BLUR2_EROWS))  // lanes per row segment

// The row-end columns of levels [l_begin, l_end) that no tile lane stores (x < 4, and the
// columns after the last group with gx + 12 <= W), lane-level: lane = (frame, level, row
// segment, 8-row chunk, column slot), 16 column slots (4 left, up to 12 right) per chunk,
// level-major (edge_base).  A lane walks its chunk's 8 + 6 source rows: row sum of its
// column over the 7 REFLECT_101 columns (rows loaded 4 ahead), then the 7-row column sum; the 16
// lanes of a chunk read the same row, 16 bytes per lane and row.
__device__ __forceinline__ void blur2_edge_lane(const OrbgGeom *__restrict__ g,
                                             const int32_t *__restrict__ edge_base,
                                             const uint8_t *__restrict__ img0, int64_t img_fs,
                                             int img_pitch, const uint8_t *__restrict__ pyr,
                                             uint8_t *__restrict__ blur, int l_begin, int l_end,
                                             int nframes, int e0)
{
    const int ne = edge_base[l_end] - edge_base[l_begin];
    if (e0 >= ne * nframes) return;
    const int f = e0 / ne;
    const int e = edge_base[l_begin] + e0 - f * ne;
    int l = l_begin;
    while (l + 1 < l_end && e >= edge_base[l + 1]) l++;
    const int r = e - edge_base[l], ty = r / BLUR2_NEG, rcs = r - ty * BLUR2_NEG;
    const int rc = rcs / BLUR2_ECOLS, cs = rcs - rc * BLUR2_ECOLS;  // row chunk, column slot
    const OrbgLevel &lv = g->lv[l];
    const int W = lv.w, H = lv.h;
    const int gx_last = (W - 12) & ~3;  // last tile group with gx + 12 <= W
    const int x = cs < 4 ? cs : gx_last + cs;
    const int y0 = ty * ORBG_BLUR2_SEG + rc * BLUR2_EROWS;
    if ((cs >= 4 && x >= W) || y0 >= H) return;
    const uint8_t *src = l == 0 ? img0 + f * img_fs : pyr + f * g->pyr_frame + lv.pyr_off;
    const int pitch = l == 0 ? img_pitch : lv.pitch;
    uint8_t *dst = blur + f * g->blur_frame + lv.blur_off;
    // the 7 REFLECT_101 taps of column x all lie in the 16 bytes [wb, wb + 16) of a row (left:
    // columns 0..6; right: W-14 .. W-1): the row sum is four v_dot4_u32_u8 of those bytes
    // against per-lane weight words (taps folded onto the same byte add up, <= 96)
    const int wb = cs < 4 ? 0 : W - 16;
    uint32_t kw[4] = {0, 0, 0, 0};
#pragma unroll
    for (int t = 0; t < 7; t++) {
        const int bpos = b2_reflect101(x - 3 + t, W) - wb;  // 0 .. 15
        const uint32_t v = (uint32_t)g->gk[t] << (8 * (bpos & 3));
#pragma unroll
        for (int q = 0; q < 4; q++) kw[q] += (bpos >> 2) == q ? v : 0u;
    }
    const uint32_t k0 = g->gk[0], k1 = g->gk[1], k2 = g->gk[2], k3 = g->gk[3], k4 = g->gk[4],
                   k5 = g->gk[5], k6 = g->gk[6];
    // bounds-checked loads (the level's last row may end the caller's image buffer: the
    // aligned over-read past byte W-1 of that row returns 0 instead of faulting)
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void *)src, (short)0, (H - 1) * pitch + W, 0x00020000);
    const int sh0 = (int)((uintptr_t)src & 3);
    typedef unsigned int b2_v4u __attribute__((ext_vector_type(4)));
    constexpr int NRE = BLUR2_EROWS + 6, EPF = ORBG_BLUR2_EPF;  // source rows; rows in flight
    b2_v4u dq[EPF];
    uint32_t d4[EPF], dsh[EPF];
    auto issue = [&](int i) {
        const int y = b2_reflect101(min(y0 - 3 + i, H + 2), H);
        const int off = y * pitch + wb, sh = (off + sh0) & 3;
        dq[i % EPF] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off - sh, 0, 0);
        d4[i % EPF] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, off - sh + 16, 0, 0);
        dsh[i % EPF] = (uint32_t)sh;
    };
#pragma unroll
    for (int i = 0; i < EPF; i++) issue(i);
    uint32_t rs[NRE];
#pragma unroll
    for (int i = 0; i < NRE; i++) {
        const b2_v4u d = dq[i % EPF];
        const uint32_t e4 = d4[i % EPF], sh = dsh[i % EPF];
        if (i + EPF < NRE) issue(i + EPF);
        uint32_t v = __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(d.y, d.x, sh), kw[0], 0u, false);
        v = __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(d.z, d.y, sh), kw[1], v, false);
        v = __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(d.w, d.z, sh), kw[2], v, false);
        v = __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(e4, d.w, sh), kw[3], v, false);
        rs[i] = v;
        if (i >= 6 && y0 + i - 6 < H) {
            const int o = i - 6;
            uint32_t a = 1u << 15;
            a = __umul24(k0, rs[o]) + a;
            a = __umul24(k1, rs[o + 1]) + a;
            a = __umul24(k2, rs[o + 2]) + a;
            a = __umul24(k3, rs[o + 3]) + a;
            a = __umul24(k4, rs[o + 4]) + a;
            a = __umul24(k5, rs[o + 5]) + a;
            a = __umul24(k6, rs[o + 6]) + a;
            dst[(int64_t)(y0 + o) * lv.pitch + x] = (uint8_t)min(a >> 16, 255u);
        }
    }
}

template <int SEG>
__global__ __launch_bounds__(256) void k_blur2(
    const OrbgGeom *__restrict__ g, const int32_t *__restrict__ task_base,
    const uint8_t *__restrict__ img0, int64_t img_fs, int img_pitch,
    const uint8_t *__restrict__ pyr, uint8_t *__restrict__ blur, int t_begin, int t_count,
    const int32_t *__restrict__ edge_base, int l_begin, int l_end, int edge_waves, int nframes)
{
    constexpr int PF = ORBG_BLUR2_ROWPF;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    // the first edge_waves waves are the row-end lanes (dispatched first, short), then tiles
#ifdef ORBG_BLUR2_EDGE_LAST  // developer A/B: edge waves after the tile waves
    const int wraw0 = blockIdx.x * 4 + wv, ntw = (int)gridDim.x * 4 - edge_waves;
    const int wraw = wraw0 >= ntw ? wraw0 - ntw : wraw0 + edge_waves;
#else
    const int wraw = blockIdx.x * 4 + wv;
#endif
    if (wraw < edge_waves) {
#ifdef ORBG_BLUR2_EDGE_NOP  // developer what-if: edge waves launched but idle (wrong results)
        return;
#endif
        blur2_edge_lane(g, edge_base, img0, img_fs, img_pitch, pyr, blur, l_begin, l_end,
                        nframes, wraw * 64 + lane);
        return;
    }
    const int nb = gridDim.x - edge_waves / 4, bt = wraw / 4 - edge_waves / 4;
    const int wid = __builtin_amdgcn_readfirstlane(xcd_remap(bt, nb) * 4 + wv);
    if (wid >= t_count * nframes) return;  // wave-uniform
    const Blur2Weights k(g);
    {
        // ---- interior tile (wave-uniform frame / level / tile) ----
        const int f = wid / t_count, t = t_begin + wid - f * t_count;
        int l = 0;
        while (l + 1 < g->L && t >= task_base[l + 1]) l++;
        const int tt = t - task_base[l];
        const OrbgLevel &lv = g->lv[l];
        const int W = lv.w, H = lv.h;
        const int ntx = (W + BLUR2_TW - 1) / BLUR2_TW;
        const int ty = tt / ntx;
        const int gx = (tt - ty * ntx) * BLUR2_TW + 4 * lane, y0 = ty * SEG;
        const uint8_t *src = l == 0 ? img0 + f * img_fs : pyr + f * g->pyr_frame + lv.pyr_off;
        const int pitch = l == 0 ? img_pitch : lv.pitch;
        uint8_t *dst = blur + f * g->blur_frame + lv.blur_off;
        const bool interior = gx >= 4 && gx + 12 <= W && 4 * lane < BLUR2_TW;
#if ORBG_BLUR2_DPP
        // lane j loads the dword at column gx - 4 of the row's 4-byte-aligned start (columns
        // from a clamped offset at the row ends: those outputs are the edge tasks'); lanes
        // j+1 .. j+3 hold the next three dwords (DPP wave shifts), so one coalesced dword per
        // lane and row feeds the 12-byte window plus the row's uniform byte shift
        const int xs = min(max(gx - 4, 0), (W - 4) & ~3);
        uint32_t ring[PF], rsh[PF];
        auto issue = [&](int i) {
            const int y = b2_reflect101(min(y0 - 3 + i, H + 2), H);
            const uint8_t *rb = src + (int64_t)y * pitch;
            const uint32_t sh = __builtin_amdgcn_readfirstlane((uint32_t)((uintptr_t)rb & 3));
            ring[i % PF] = *(const uint32_t *)(rb - sh + xs);
            rsh[i % PF] = sh;
        };
#pragma unroll
        for (int i = 0; i < PF; i++) issue(i);
        blur2_column<SEG>(
            k,
            [&](int i, uint32_t &w0, uint32_t &w1, uint32_t &w2) {
                const uint32_t d0 = ring[i % PF], sh = rsh[i % PF];
                if (i + PF < SEG + 6) issue(i + PF);
                // wave_shl1 (DPP 0x130): lane j reads lane j + 1
                const uint32_t d1 = __builtin_amdgcn_mov_dpp(d0, 0x130, 0xF, 0xF, true);
                const uint32_t d2 = __builtin_amdgcn_mov_dpp(d1, 0x130, 0xF, 0xF, true);
                const uint32_t d3 = __builtin_amdgcn_mov_dpp(d2, 0x130, 0xF, 0xF, true);
                w0 = __builtin_amdgcn_alignbyte(d1, d0, sh);
                w1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
                w2 = __builtin_amdgcn_alignbyte(d3, d2, sh);
            },
            [&](int o, uint32_t word) {
                const int gy = y0 + o;
                if (gy < H && interior)  // gy: wave-uniform; interior lanes: gx + 4 <= W
                    *(uint32_t *)(dst + (int64_t)gy * lv.pitch + gx) = word;
            });
#else
        // every lane loads a dwordx4 inside the row from a multiple-of-4 column (row-end lanes
        // from a clamped start: their outputs are the edge tasks'), so the byte shift of a row
        // is wave-uniform (the row's own alignment: level 0 may have any pitch) and the load is
        // a uniform row base + a per-lane 32-bit offset
        const int xs = min(max(gx - 4, 0), (W - 16) & ~3);
        uint4 ring[PF];
        uint32_t rsh[PF];
        auto issue = [&](int i) {
            const int y = b2_reflect101(min(y0 - 3 + i, H + 2), H);
            const uint8_t *rb = src + (int64_t)y * pitch;
            const uint32_t sh = __builtin_amdgcn_readfirstlane((uint32_t)((uintptr_t)rb & 3));
            ring[i % PF] = *(const uint4 *)(rb - sh + xs);
            rsh[i % PF] = sh;
        };
#pragma unroll
        for (int i = 0; i < PF; i++) issue(i);
        blur2_column<SEG>(
            k,
            [&](int i, uint32_t &w0, uint32_t &w1, uint32_t &w2) {
                const uint4 q = ring[i % PF];
                const uint32_t sh = rsh[i % PF];
                if (i + PF < SEG + 6) issue(i + PF);
                w0 = __builtin_amdgcn_alignbyte(q.y, q.x, sh);
                w1 = __builtin_amdgcn_alignbyte(q.z, q.y, sh);
                w2 = __builtin_amdgcn_alignbyte(q.w, q.z, sh);
            },
            [&](int o, uint32_t word) {
                const int gy = y0 + o;
                if (gy < H && interior)  // gy: wave-uniform; interior lanes: gx + 4 <= W
                    *(uint32_t *)(dst + (int64_t)gy * lv.pitch + gx) = word;
            });
#endif
    }
}

int blur2_seg() { return ORBG_BLUR2_SEG; }
int blur2_tw() { return BLUR2_TW; }
int blur2_neg() { return BLUR2_NEG; }

// levels [l_begin, l_end): tiles [t_begin, t_begin + t_count) of every frame + their edge tasks
hipError_t launch_blur2(hipStream_t st, const OrbgGeom *g, const int32_t *task_base,
                        const int32_t *edge_base, int edges, const uint8_t *img0, int64_t img_fs,
                        int img_pitch, const uint8_t *pyr, uint8_t *blur, int t_begin,
                        int t_count, int l_begin, int l_end, int nframes)
{
    // edge lanes in whole workgroups (4 waves) ahead of the tile waves
#ifdef ORBG_BLUR2_NOEDGE  // developer what-if: no edge waves (wrong results)
    const int edge_waves = 0;
#else
    const int edge_waves = 4 * ((edges * nframes + 255) / 256);
#endif
    const int waves = edge_waves + 4 * ((t_count * nframes + 3) / 4);
    if (waves > 0)
        hipLaunchKernelGGL(k_blur2<ORBG_BLUR2_SEG>, dim3(waves / 4), dim3(256), 0, st, g,
                           task_base, img0, img_fs, img_pitch, pyr, blur, t_begin, t_count,
                           edge_base, l_begin, l_end, edge_waves, nframes);
    return hipGetLastError();
}

}  // namespace orbg
