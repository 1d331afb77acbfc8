// blur_device.h -- one k_blur2 wave tile (GaussianBlur 7x7, sigma 2, BORDER_REFLECT_101,
// cv::GaussianBlur 8U bit-exact fixed point; ORBextractor.cc:1375-1377), shared by k_blur2
// (blur_kernels.hip, a launch over the pyramid) and k_pyramid (pyramid_kernels.hip, which blurs
// each level's band while the level is still in L2).  See blur_kernels.hip for the scheme.
#pragma once

#include <hip/hip_runtime.h>

#include "orbg_internal.h"
#include "orbg_device.h"

#pragma clang fp contract(off)

namespace orbg {

#define BLUR2_TW 244  // output columns per wave (4 per lane; the last 3 lanes supply data)
#define BLUR2_TW_T 240  // the same for tiled output: 15 whole 16-px tiles (lanes 60..63 supply data)
// tiled output's LDS stage: 8 rows of 64 dwords, padded to 68 so the 16-byte reads of one
// tile's 8 rows (lanes 8t .. 8t+7) fall on distinct banks (64 dwords apart they conflict 8-way)
#ifndef BLUR2_LDS_ROW
#define BLUR2_LDS_ROW 68
#endif
#ifndef ORBG_BLUR2_SEG
#define ORBG_BLUR2_SEG 32  // output rows per wave
#endif
#ifndef ORBG_BLUR2_ROWPF
#define ORBG_BLUR2_ROWPF 4  // source rows in flight per lane (vs 8: 4 -2.5%, 6 -1.7%, 12 +2% serial)
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
        // row pass weight words: output x = gx + i needs window bytes 1+i .. 7+i
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

template <int SEG, bool NORM256, typename Loader, typename Store>
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
            if constexpr (NORM256) {
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

// One wave: output columns tx * 244 + 4 * lane .. + 3 (lanes 61..63 only supply data) of rows
// [y0, y0 + SEG) of a W x H level at `src` (row pitch `pitch`) into `dst` (row pitch `dpitch`).
// Rows at or past `yend` are not stored (the store range ends there: k_pyramid's bands store
// only their own rows; their source rows past yend + 3 may be another band's and are never used
// by a stored output).
// TILED (k_blur2 with G.blur_tiled): `dst` is stored as 16 x 8-px tiles of 128 bytes, tile
// (tx, ty) at ty * 8 * dpitch + tx * 128, pixel (x, y) at byte (y & 7) * 16 + (x & 15) of it --
// the level's row-major footprint with its rows rounded up to 8 (k_orient_desc's rBRIEF
// neighbourhood then touches one cache line per tile row of a tile instead of one or two per
// image row).  The wave is BLUR2_TW_T = 15 tiles wide; its output rows go through `wlds` (8 x
// BLUR2_LDS_ROW dwords of this wave's LDS) and every 8 rows leave as two dwordx4 stores of whole tile rows
// (each instruction writes 8 whole 128-byte lines; dword stores into the tiles cost k_blur2
// +79%, profiles/r06r_blur_tiled_ab.txt).  y0 is a multiple of 8; rows in [yend, yend rounded
// up to 8) land in the last tile row's padding.
template <int SEG, bool TILED = false>
__device__ __forceinline__ void blur2_tile(const Blur2Weights &k, const uint8_t *src, int pitch,
                                           int W, int H, uint8_t *dst, int dpitch, int tx, int y0,
                                           int yend, int lane, uint32_t *wlds = nullptr)
{
    constexpr int PF = ORBG_BLUR2_ROWPF;
    constexpr int TW = TILED ? BLUR2_TW_T : BLUR2_TW;
    static_assert(!TILED || SEG % 8 == 0, "tiled output: whole tile rows per wave");
    const int gx = tx * TW + 4 * lane;
    const bool owner = 4 * lane < TW && gx < W;
    // row ends (REFLECT_101 at x = -1 and x = W): window byte b is column gx - 4 + b
    const bool left_wave = tx == 0, right_wave = (tx + 1) * TW + 8 > W;
    const bool is_left = gx == 0;
    const int m = W - gx;  // right lanes: m in 1..7 need reflected bytes inside the window
    uint32_t sel1 = 0x07060504u, sel2 = 0x07060504u;  // identity: w1, w2
    bool pair_lo = false;                             // w2' from (w1, w0) instead of (w2, w1)
    if (m >= 1 && m <= 7) {
        pair_lo = m <= 3;
        sel1 = sel2 = 0;
#pragma unroll
        for (int b = 4; b < 12; b++) {
            int sb = b < m + 4 ? b : 2 * m + 6 - b;  // bytes never used by a stored output: any
            if (b >= 8) sb = pair_lo ? max(sb, 0) : max(sb, 4) - 4;
            else sb = max(sb, 0);
            if (b < 8) sel1 |= (uint32_t)sb << (8 * (b - 4));
            else sel2 |= (uint32_t)sb << (8 * (b - 8));
        }
    }
    // bounds-checked loads over the level of this frame: offsets past its last byte (the
    // caller's image may end there) read 0.  The range starts at the dword holding the
    // level's first byte (src - sh0: a batch frame of the caller's may start at any byte, and
    // the dword straddling that start holds pixels 0 .. 3 - sh0 of row 0; a range starting at
    // src would give it a negative offset and zeros).  Offsets below are src-relative; the
    // loads add sh0.
    const int nrec = (H - 1) * pitch + W;
    const int sh0 = (int)((uintptr_t)src & 3);
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(src - sh0), (short)0, nrec + sh0, 0x00020000);
    bool strad_wave;
    {
        const int ro = (H - 1) * pitch;
        const int ol = ro - ((ro + sh0) & 3) + gx - 4;
        strad_wave = __ballot(ol + 4 > nrec && ol < nrec) != 0;
    }
    // stores: buffer stores over the blurred level incl. its row padding; lanes that store
    // nothing (past the tile or the level width) and rows past the level get an offset past
    // the range, which the hardware drops -- no exec-mask branches per row.  A lane whose
    // 4 columns pass W writes the rest of its dword into the row padding (pitch >= W
    // rounded up to 64; the padding is never read).
    const __amdgpu_buffer_rsrc_t drsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void *)dst, (short)0, (TILED ? (yend + 7) & ~7 : yend) * dpitch, 0x00020000);
    const int lane_off = owner ? gx : (1 << 30);
    // interior tiles (every source row inside the level, the last one above the level's last
    // row) need no REFLECT_101 row index and no straddle test: the row offset is affine in i
    const bool interior = y0 >= 3 && y0 + SEG + 3 < H;
    auto run = [&](auto INTERIOR, auto NORM) {
        constexpr bool inner = decltype(INTERIOR)::value;
        uint32_t ring[PF], rsh[PF];
        auto issue = [&](int i) {
            const int y = inner ? y0 - 3 + i : b2_reflect101(min(y0 - 3 + i, H + 2), H);
            const int rowoff = y * pitch;
            const int sh = __builtin_amdgcn_readfirstlane((rowoff + sh0) & 3);
            const int o = rowoff - sh + gx - 4;
            uint32_t v;
            // only the level's last row can hold that dword (a tile row reads < 256 + 8
            // bytes, less than pitch + W), and only in waves where some lane's last-row dword
            // does (wave-uniform test): every other row is one load with no exec-mask branches
            v = __builtin_amdgcn_raw_buffer_load_b32(rsrc, o + sh0, 0, 0);
            if (!inner && strad_wave && y == H - 1) {  // wave-uniform
                if (o + 4 > nrec && o < nrec) {
                    // the dword holding the level's last byte: a dword load straddling the
                    // range end reads 0 as a whole, so this one lane reads its in-range bytes
                    // one by one
                    uint32_t vb = 0;
                    for (int b = 0; b < 4 && o + b < nrec; b++)
                        vb |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rsrc, o + b + sh0, 0, 0) << (8 * b);
                    v = vb;
                }
            }
            ring[i % PF] = v;
            rsh[i % PF] = (uint32_t)sh;
        };
#pragma unroll
        for (int i = 0; i < PF; i++) issue(i);
        blur2_column<SEG, decltype(NORM)::value>(
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
                if (left_wave) {  // x = -4 .. -1 -> 4, 3, 2, 1
                    const uint32_t r = __builtin_amdgcn_perm(w2, w1, 0x01020304u);
                    w0 = is_left ? r : w0;
                }
                if (right_wave) {
                    const uint32_t v1 = __builtin_amdgcn_perm(w1, w0, sel1);
                    const uint32_t v2 = pair_lo ? __builtin_amdgcn_perm(w1, w0, sel2)
                                                : __builtin_amdgcn_perm(w2, w1, sel2);
                    w1 = v1;
                    w2 = v2;
                }
            },
            [&](int o, uint32_t word) {
                if (!TILED) {
                    __builtin_amdgcn_raw_buffer_store_b32(word, drsrc, lane_off + (y0 + o) * dpitch,
                                                          0, 0);
                    return;
                }
                wlds[(o & 7) * BLUR2_LDS_ROW + lane] = word;
                if ((o & 7) != 7) return;
                wave_sync_lds();
                const int tyoff = ((y0 + (o & ~7)) >> 3) * (8 * dpitch);
#pragma unroll
                for (int h = 0; h < 2; h++) {  // lane -> (tile t, tile row r)
                    const int idx = lane + 64 * h, t = idx >> 3, r = idx & 7;
                    typedef uint32_t b2_v4u __attribute__((ext_vector_type(4)));
                    const b2_v4u v = *(const b2_v4u *)(wlds + r * BLUR2_LDS_ROW + 4 * t);
                    const int x = tx * TW + 16 * t;
                    const int off = (t < TW / 16 && x < W) ? tyoff + (x >> 4) * 128 + r * 16 : (1 << 30);
                    __builtin_amdgcn_raw_buffer_store_b128(v, drsrc, off, 0, 0);
                }
                wave_sync_lds();  // the rows' reads before the next 8 rows overwrite them
            });
    };
    // (and the weight sum: legacy 257-sum tables saturate instead of taking byte 2)
    if (k.norm256) {
        if (interior)
            run(std::true_type{}, std::true_type{});
        else
            run(std::false_type{}, std::true_type{});
    } else {
        if (interior)
            run(std::true_type{}, std::false_type{});
        else
            run(std::false_type{}, std::false_type{});
    }
}

}  // namespace orbg
