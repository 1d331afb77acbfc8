// extract_kernels.hip -- ORBextractor::operator() as batched HIP kernels for gfx950.
//
// One launch per stage for a whole batch of frames (grid.y / grid.z = frame):
//   k_resize        ComputePyramid (ORBextractor.cc:1400-1443), cv::resize INTER_LINEAR 8U
//   k_fast_cells    ComputeKeyPointsOctTree FAST part (:970-1094): one workgroup per 30-px
//                   cell: LDS window, FAST-9 score, threshold fallback, cell-local NMS,
//                   raster-order compaction
//   k_blur          GaussianBlur 7x7 sigma 2 REFLECT_101 per level (:1375-1377)
//   k_octree        DistributeOctTree (:668-951) as a data-parallel quadtree: one workgroup
//                   per (frame, level); list order, split order and tie-breaks reproduced
//   k_orient_desc   IC_Angle (:83-111) + computeOrbDescriptor (:117-157) + output assembly
//                   (:1381-1395), one wave per keypoint
// Bit-exactness pins: no FMA contraction (-ffp-contract=off + pragma),
// cvRound = round-half-even, fastAtan2 polynomial, pinned double sincos.
#include <hip/hip_runtime.h>

#include "orbg_internal.h"
#include "orbg_device.h"
#include "fast_device.h"

#pragma clang fp contract(off)

namespace orbg {

// ---------------------------------------------------------------------------
// block-wide helpers (blockDim.x == 256)
// ---------------------------------------------------------------------------
// exclusive scan of one value per thread over the 256-thread block; *total = block sum.
// `sh` is an 8-int LDS scratch.  Contains two barriers.
__device__ int block_excl_scan(int v, int *total, int *sh)
{
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int nw = blockDim.x >> 6;
    int x = wave_incl_scan(v);
    if (lane == 63) sh[wid] = x;
    __syncthreads();
    int before = 0, tot = 0;
    for (int i = 0; i < nw; i++) {
        const int s = sh[i];
        before += (i < wid) ? s : 0;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return before + x - v;
}

__device__ int block_sum(int v, int *sh)
{
    int t;
    block_excl_scan(v, &t, sh);
    return t;
}

// ---------------------------------------------------------------------------
// k_resize: level l from level l-1 (cv::resize INTER_LINEAR, 8UC1, fixed point)
// xtab[dx] = {sx, a0 | a1 << 16}; ytab[dy] = {sy0 | sy1 << 16, b0 | b1 << 16}
// columns dx < bulk_end use the SIMD vertical pass (mulhi of S>>4), the rest the
// scalar FixedPtCast<int,uchar,22>.
// A workgroup walks RZ_NT vertical RZ_TW x RZ_TH output tiles.  The source rows/columns a
// tile touches are staged in LDS from 16-byte chunks (each row keeps its source address
// alignment, so a caller image with an odd pitch works); the next tile's chunks are in
// flight while the current one is computed.  Each thread owns 4 output columns (their
// coefficients stay in registers) and wave w walks the tile's rows 4w .. 4w+3 in order, so
// a source row's horizontal sums are computed once and reused by the next output row
// (1.2 source rows per output row instead of 2).  One dword store per output row.
// ---------------------------------------------------------------------------
#define RZ_TW 256
#define RZ_TH 16
#define RZ_NT ORBG_RZ_NT      // tiles per workgroup
#define RZ_FILL ORBG_RZ_FILL  // staged chunks per thread (host: rows x chunks <= 256 x RZ_FILL)
#ifndef RZ_WPE
#define RZ_WPE 1  // min waves per SIMD (no cap: the prefetch chunks need ~90 VGPRs)
#endif

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RZ_WPE, 8))) void k_resize(const uint8_t *__restrict__ src, int64_t sfs,
                                                int spitch, int sw, uint8_t *__restrict__ dst,
                                                int64_t dfs, int dpitch, int dw, int dh,
                                                const int2 *__restrict__ xtab,
                                                const int2 *__restrict__ ytab, int bulk_end,
                                                int lds_pitch)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t rz_lds[];
    uint8_t *lds = (uint8_t *)rz_lds;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int c0 = blockIdx.x * RZ_TW, rb0 = blockIdx.y * (RZ_TH * RZ_NT), f = blockIdx.z;
    const int ntile = min(RZ_NT, (dh - rb0 + RZ_TH - 1) / RZ_TH);  // >= 1
    const int c1 = min(c0 + RZ_TW, dw) - 1;
    const int sx_lo = xtab[c0].x;
    const int sx_hi = min(xtab[c1].x + 1, sw - 1);
    const uint8_t *fb = src + f * sfs;
    const int nch = (3 + sx_hi - sx_lo + 1 + 15) >> 4;  // chunks per row (upper bound)
    // ---- staging: chunk i = (row r, chunk c) of the tile's source rows, 16 bytes from the
    // row's 4-byte-aligned start; a chunk reaching outside [row, row + sw) (image edges) is
    // assembled byte-wise at store time ----
    uint4 q[RZ_FILL];
    int dsto[RZ_FILL];  // LDS offset, bit 30 = edge chunk, -1 = none
    auto load_tile = [&](int r0) {
        const int r1 = min(r0 + RZ_TH, dh) - 1;
        const int sy_lo = ytab[r0].x & 0xFFFF, sy_hi = ytab[r1].x >> 16;
        const int total = (sy_hi - sy_lo + 1) * nch;
#pragma unroll
        for (int k = 0; k < RZ_FILL; k++) {
            const int i = 256 * k + tid;
            q[k] = make_uint4(0, 0, 0, 0);
            dsto[k] = -1;
            if (i < total) {
                const int r = i / nch, c = i - r * nch;
                const uint8_t *row = fb + (int64_t)(sy_lo + r) * spitch;
                const uint8_t *start = row + sx_lo;
                const uint8_t *cp = start - ((uintptr_t)start & 3) + 16 * c;
                const bool in_row = cp >= row && cp + 16 <= row + sw;
                if (in_row) q[k] = *(const uint4 *)cp;
                dsto[k] = (r * lds_pitch + 16 * c) | (in_row ? 0 : 1 << 30);
            }
        }
        return sy_lo;
    };
    auto store_tile = [&](int sy_lo) {
#pragma unroll
        for (int k = 0; k < RZ_FILL; k++) {
            if (dsto[k] < 0) continue;
            int o = dsto[k];
            if (o & (1 << 30)) {
                o &= ~(1 << 30);
                int r = o / lds_pitch;
                // opaque: keeps the edge path's address math out of the tile loop
                asm volatile("" : "+v"(r));
                const int c = (o - r * lds_pitch) >> 4;
                const uint8_t *row = fb + (int64_t)(sy_lo + r) * spitch;
                const uint8_t *start = row + sx_lo;
                const uint8_t *cp = start - ((uintptr_t)start & 3) + 16 * c;
                uint32_t w4[4] = {0, 0, 0, 0};
                for (int b = 0; b < 16; b++)
                    if (cp + b >= row && cp + b < row + sw)
                        w4[b >> 2] |= (uint32_t)cp[b] << (8 * (b & 3));
                q[k] = make_uint4(w4[0], w4[1], w4[2], w4[3]);
            }
            *(uint4 *)(lds + o) = q[k];
        }
    };
    // ---- per-thread column coefficients ----
    const int dx0 = c0 + 4 * lane;
    int ox0[4], ox1[4], ca0[4], ca1[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int dx = min(dx0 + i, c1);
        const int2 xt = xtab[dx];
        ox0[i] = xt.x - sx_lo;
        ox1[i] = min(xt.x + 1, sw - 1) - sx_lo;
        ca0[i] = (int)(short)(xt.y & 0xFFFF);
        ca1[i] = (int)(short)(xt.y >> 16);
    }
    const int nvalid = min(4, c1 - dx0 + 1);  // <= 0: this thread has no columns
    int sy_lo = load_tile(rb0);
#pragma unroll 1
    for (int t = 0; t < ntile; t++) {  // workgroup-uniform trip count
        const int r0 = rb0 + t * RZ_TH, r1 = min(r0 + RZ_TH, dh) - 1;
        __syncthreads();  // the previous tile's LDS reads are done
        store_tile(sy_lo);
        __syncthreads();
        const int cur_lo = sy_lo;
        if (t + 1 < ntile) sy_lo = load_tile(r0 + RZ_TH);
        if (nvalid <= 0) continue;
        // horizontal sums of source row sy for this thread's 4 columns
        auto hrow = [&](int sy, int h[4]) {
            const int sh = (int)((uintptr_t)(fb + (int64_t)sy * spitch + sx_lo) & 3);
            const uint8_t *lr = lds + (sy - cur_lo) * lds_pitch + sh;
#pragma unroll
            for (int i = 0; i < 4; i++)
                h[i] = __mul24((int)lr[ox0[i]], ca0[i]) + __mul24((int)lr[ox1[i]], ca1[i]);
        };
        int psy = -1, ph[4] = {0, 0, 0, 0};
#pragma unroll 1
        for (int k = 0; k < RZ_TH / 4; k++) {
            const int dy = r0 + 4 * wv + k;  // wave-uniform
            if (dy > r1) break;
            const int2 yt = ytab[dy];
            const int sy0 = yt.x & 0xFFFF, sy1 = yt.x >> 16;
            const int b0 = (int)(short)(yt.y & 0xFFFF), b1 = (int)(short)(yt.y >> 16);
            int h0[4], h1[4];
            if (sy0 == psy) {
#pragma unroll
                for (int i = 0; i < 4; i++) h0[i] = ph[i];
            } else {
                hrow(sy0, h0);
            }
            if (sy1 == sy0) {
#pragma unroll
                for (int i = 0; i < 4; i++) h1[i] = h0[i];
            } else {
                hrow(sy1, h1);
            }
            psy = sy1;
#pragma unroll
            for (int i = 0; i < 4; i++) ph[i] = h1[i];
            uint32_t word = 0;
#pragma unroll
            for (int i = 0; i < 4; i++) {
                int v;
                // 24-bit multiplies (full rate): |h| <= 255 * 2 * 2048 < 2^23, |b| <= 2048
                if (dx0 + i < bulk_end) {
                    const int a = __mul24(h0[i] >> 4, b0) >> 16;
                    const int b = __mul24(h1[i] >> 4, b1) >> 16;
                    v = (a + b + 2) >> 2;
                } else {
                    v = (__mul24(h0[i], b0) + __mul24(h1[i], b1) + (1 << 21)) >> 22;
                }
                word |= (uint32_t)min(max(v, 0), 255) << (8 * i);
            }
            uint8_t *d = dst + f * dfs + (int64_t)dy * dpitch + dx0;
            if (nvalid == 4) {
                *(uint32_t *)d = word;  // dpitch % 64 == 0 and dx0 % 4 == 0
            } else {
                for (int i = 0; i < nvalid; i++) d[i] = (uint8_t)(word >> (8 * i));
            }
        }
    }
}

// ---------------------------------------------------------------------------
// k_fast_cells: one wave per (cell, frame), four cells per 256-thread workgroup; the
// 1-D grid of ceil(ncells * B / 4) workgroups is frame-major after the XCD remap, so a
// workgroup's cells are neighbours sharing halo rows in L1/L2.  Everything inside a cell
// is wave-synchronous (no workgroup barrier).
// LDS per wave: tile (window) + sc (scores), both fc_pitch bytes per row.  Window row r at
// tile[r][1 + x] (x window-local) so that a group of 4 detection pixels (window
// x = 3+4g .. 6+4g) and its +-3 neighbours are the 12 bytes of dwords g..g+2; the window
// is copied with aligned dword loads + v_alignbyte.  Scores: sc[ry+1][rx+4] with a zero
// border (NMS neighbours outside the cell's detection region count as 0 -- cv::FAST runs
// on the cell ROI alone).  Unit = (region row ry, 4-pixel group g), u = ry*RG + g, walked in
// raster order so the compaction preserves FAST's row-major output order.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6, 8))) void k_fast_cells(const OrbgGeom *__restrict__ g,
                                                    const OrbgCell *__restrict__ cells,
                                                    const uint8_t *__restrict__ img0,
                                                    int64_t img_fs, int img_pitch,
                                                    const uint8_t *__restrict__ pyr,
                                                    const uint32_t *__restrict__ ctab,
                                                    int32_t *__restrict__ cell_cnt,
                                                    uint2 *__restrict__ cell_kp, int nframes,
                                                    int c_begin, int c_count)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t fc_lds[];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int P = g->fc_pitch;
    uint8_t *tile = (uint8_t *)fc_lds + wv * g->fc_wave_bytes;
    uint8_t *sc = tile + g->fc_tile_rows * P;
    // wave-uniform: the cell record and level parameters come through the scalar cache
    const int cid = __builtin_amdgcn_readfirstlane(xcd_remap(blockIdx.x, gridDim.x) * 4 + wv);
    // cells [c_begin, c_begin + c_count) of every frame (level 0 alone or levels 1.. alone
    // when the level-0 cells run beside the pyramid)
    if (cid >= c_count * nframes) return;  // wave-uniform; no workgroup barrier below
    const int f = cid / c_count, c = c_begin + cid - f * c_count;
    // one dwordx4 (scalar load: sub-dword loads would go through the vector path)
    const uint4 cw4 = ((const uint4 *)cells)[c];
    const uint32_t cw0 = __builtin_amdgcn_readfirstlane(cw4.x);  // level | pad
    const uint32_t cw1 = __builtin_amdgcn_readfirstlane(cw4.y);  // x0 | y0
    const uint32_t cw2 = __builtin_amdgcn_readfirstlane(cw4.z);  // w | h
    struct {
        int x0, y0;
    } cl = {(int)(int16_t)(cw1 & 0xFFFF), (int)(int16_t)(cw1 >> 16)};
    const int l = (int)(int16_t)(cw0 & 0xFFFF);
    const int W = (int)(int16_t)(cw2 & 0xFFFF), H = (int)(int16_t)(cw2 >> 16);
    const uint8_t *base;
    int pitch;
    if (l == 0) {
        base = img0 + f * img_fs;
        pitch = img_pitch;
    } else {
        base = pyr + f * g->pyr_frame + g->lv[l].pyr_off;
        pitch = g->lv[l].pitch;
    }
    base += (int64_t)cl.y0 * pitch + cl.x0;
    const int RW = W - 6, RH = H - 6;
    const int RG = RW > 0 ? (RW + 3) >> 2 : 0;
    const int nunits = RH > 0 ? RH * RG : 0;
    // quadtree path codes of this cell's columns / rows (RW, RH <= 60 < 64), one per lane,
    // issued now so their latency hides behind the window loads
    const int xo = cl.x0 - ORBG_MIN_BORDER + 3, yo = cl.y0 - ORBG_MIN_BORDER + 3;
    const uint32_t xs_l = lane < RW ? ctab[g->lv[l].xs_off + xo + lane] : 0u;
    const uint32_t ys_l = lane < RH ? ctab[g->lv[l].ys_off + yo + lane] : 0u;
    {
        // dword j of tile row r = window bytes 4j-1 .. 4j+2 (the window sits >= 13 px inside
        // the level on every side, so the aligned over-read stays in the image)
        // all loads of a 512-word chunk are issued before the first LDS store (one memory
        // latency per chunk instead of one per 64 words)
        const int NWR = RG + 2;
        const int nw = H * NWR;
        // word i = lane + 64 k of the window as (row r, word j), advanced by (64 / NWR,
        // 64 % NWR) per k (no division in the loop); its byte offset r * pitch + 4 j - 1
        // and tile offset r * P + 4 j advance with it
        const int dr = 64 / NWR, dj = 64 - dr * NWR;
        int r = lane / NWR, j = lane - r * NWR;
        int goff = r * pitch + 4 * j - 1, toff = r * P + 4 * j;
        const int gstep_r = dr * pitch + 4 * dj, tstep_r = dr * P + 4 * dj;
        const int gwrap = pitch - 4 * NWR, twrap = P - 4 * NWR;
        for (int i0 = 0; i0 < nw; i0 += 8 * 64) {
            uint32_t lo[8], hi[8], sh[8];
            int dst[8];
#pragma unroll
            for (int k = 0; k < 8; k++) {
                // unconditional loads (a lane past the window reads word 0 again): no
                // branch, so all 16 loads are in flight before the first wait
                const bool ok = i0 + 64 * k + lane < nw;
                const int go = ok ? goff : -1;
                const int mis = (int)(((uint32_t)(uintptr_t)base + (uint32_t)go) & 3u);
                const uint32_t *aw = (const uint32_t *)(base + (go - mis));
                lo[k] = aw[0];
                hi[k] = aw[1];
                sh[k] = (uint32_t)mis;
                dst[k] = ok ? toff : -1;
                goff += gstep_r;
                toff += tstep_r;
                j += dj;
                if (j >= NWR) {
                    j -= NWR;
                    goff += gwrap;
                    toff += twrap;
                }
            }
#pragma unroll
            for (int k = 0; k < 8; k++)
                if (dst[k] >= 0)
                    *(uint32_t *)(tile + dst[k]) = __builtin_amdgcn_alignbyte(hi[k], lo[k], sh[k]);
        }
        uint32_t *z = (uint32_t *)sc;
        const int nz = (RH + 2) * (P >> 2);
        for (int i = lane; i < nz; i += 64) z[i] = 0;
    }
    wave_sync_lds();
    if (g->dbg == 11) return;

    // unit u = ry * RG + gg walked as u = lane + 64 k: (ry, gg) advance by (64 / RG, 64 % RG)
    const int rstep = RG > 0 ? 64 / RG : 0, gstep = RG > 0 ? 64 - rstep * RG : 0;
    const int ry0 = RG > 0 ? lane / RG : 0, gg0 = lane - ry0 * RG;
    // unit (ry, gg): its 7 window rows x 3 dwords, both pixel pairs scored, word -> sc
    auto score_unit = [&](int ry, int gg) {
        Rows7 R;
#pragma unroll
        for (int r = 0; r < 7; r++) {
            const uint32_t *p = (const uint32_t *)(tile + (ry + r) * P + 4 * gg);
            R.w[r][0] = p[0];
            R.w[r][1] = p[1];
            R.w[r][2] = p[2];
        }
        const v2s sa = fast_score_pair<0>(R);
        const v2s sb = fast_score_pair<2>(R);
        uint32_t word = (uint32_t)(uint16_t)sa.x | ((uint32_t)(uint16_t)sa.y << 8) |
                        ((uint32_t)(uint16_t)sb.x << 16) | ((uint32_t)(uint16_t)sb.y << 24);
        const int valid = min(RW - 4 * gg, 4);
        if (valid < 4) word &= (1u << (8 * valid)) - 1u;
        *(uint32_t *)(sc + (ry + 1) * P + 4 * gg + 4) = word;
    };
    const int thi = g->ini_th, tlo = g->min_th;
    // ---- compass pretest at iniThFAST + compaction ----
    // A corner at th has 9 contiguous circle pixels all brighter than v + th or all darker
    // than v - th; any 9-arc holds two adjacent compass points (circle 0/4, 4/8, 8/12,
    // 12/0), so "both brighter" or "both darker" for some adjacent pair is necessary.  Only
    // units with a pixel passing it are scored; the others keep score 0, which the NMS at
    // iniThFAST treats exactly like any score below th (a neighbour < th never blocks).
    // Pixel pairs in packed i16 lanes.  "Some adjacent pair both brighter" is
    // (b0 & b4) | (b4 & b8) | (b8 & b12) | (b12 & b0) = (b0 | b8) & (b4 | b12), i.e.
    // mb = min(max(c0, c8), max(c4, c12)) > v + th; darker: md = max(min(c0, c8),
    // min(c4, c12)) < v - th.
    // Two survivor lists (u16 row << 8 | group, raster order) of the pixel pairs A (pixels
    // 0,1) and B (2,3) with a pixel passing; the scores are computed per pair: 31% of the
    // pairs pass where 46% of the units do.
    const int lcap = (g->fc_wave_bytes - g->fc_list_off) / 4;
    uint16_t *alist = (uint16_t *)(tile + g->fc_list_off), *blist = alist + lcap;
    // the corner-unit list of the NMS is built after the scoring, over the pair lists
    uint16_t *plist = alist;
    int npass = 0, na = 0, nb = 0;
    {
        const v2s vth1 = (v2s){(short)(thi + 1), (short)(thi + 1)};
        // uniform trip count: the scan below is wave-wide
        for (int u0 = 0, ry = ry0, gg = gg0; u0 < nunits; u0 += 64) {
            const int u = u0 + lane;
            uint32_t pm = 0;
            if (u < nunits) {
                uint32_t r0[3], r3[3], r6[3];
                const uint32_t *p0 = (const uint32_t *)(tile + ry * P + 4 * gg);
                const uint32_t *p3 = (const uint32_t *)(tile + (ry + 3) * P + 4 * gg);
                const uint32_t *p6 = (const uint32_t *)(tile + (ry + 6) * P + 4 * gg);
#pragma unroll
                for (int k = 0; k < 3; k++) {
                    r0[k] = p0[k];
                    r3[k] = p3[k];
                    r6[k] = p6[k];
                }
                auto pretest = [&](auto I) -> uint32_t {
                    constexpr int i = decltype(I)::value;
                    const v2s v = gather2<4 + i>(r3[0], r3[1], r3[2]);
                    const v2s c0 = gather2<4 + i>(r6[0], r6[1], r6[2]);
                    const v2s c4 = gather2<7 + i>(r3[0], r3[1], r3[2]);
                    const v2s c8 = gather2<4 + i>(r0[0], r0[1], r0[2]);
                    const v2s c12 = gather2<1 + i>(r3[0], r3[1], r3[2]);
                    // "some adjacent compass pair both brighter" = (b0|b8) & (b4|b12)
                    const v2s mb = pmin(pmax(c0, c8), pmax(c4, c12));
                    const v2s md = pmax(pmin(c0, c8), pmin(c4, c12));
                    const v2s k = pmax(mb - v, v - md) - vth1;  // >= 0 <=> pass
                    const uint32_t w = __builtin_bit_cast(uint32_t, k);
                    return (~w >> 15 & 1u) | (~w >> 30 & 2u);
                };
                pm = pretest(std::integral_constant<int, 0>{}) |
                     pretest(std::integral_constant<int, 2>{}) << 2;
                const int valid = min(RW - 4 * gg, 4);
                if (valid < 4) pm &= (1u << valid) - 1u;
            }
            // ballot + mbcnt compaction of the three lists
            const uint16_t e = (uint16_t)(ry << 8 | gg);
            auto append = [&](bool flag, uint16_t *list, int &n) {
                const unsigned long long m = __ballot(flag);
                const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
                if (flag) list[n + below] = e;
                n += __popcll(m);
            };
            append((pm & 3u) != 0, alist, na);
            append((pm & 12u) != 0, blist, nb);
            ry += rstep;
            gg += gstep;
            if (gg >= RG) {
                gg -= RG;
                ry++;
            }
        }
    }
    wave_sync_lds();
    if (g->dbg == 14) return;
    // ---- scores of the pretest survivors, per pixel pair (dense over lanes) ----
    // a pair's two scores go to bytes 0,1 (A) or 2,3 (B) of the unit's score word; the
    // pair not listed keeps the zeros of the cleared score tile
    auto score_pair = [&](auto I, int e) {
        constexpr int i = decltype(I)::value;
        const int ry = e >> 8, gg = e & 0xFF;
        Rows7 R;
#pragma unroll
        for (int r = 0; r < 7; r++) {
            const uint32_t *p = (const uint32_t *)(tile + (ry + r) * P + 4 * gg);
            R.w[r][0] = p[0];
            R.w[r][1] = p[1];
            R.w[r][2] = p[2];
        }
        const v2s s = fast_score_pair<i>(R);
        // a score below iniThFAST is stored as 0: the NMS treats both alike (a neighbour
        // < th never blocks), and a unit with no corner then has a zero score word
        const uint32_t s0 = (uint16_t)s.x >= (uint32_t)thi ? (uint16_t)s.x : 0u;
        const uint32_t s1 = (uint16_t)s.y >= (uint32_t)thi ? (uint16_t)s.y : 0u;
        uint32_t h = s0 | (s1 << 8);
        if (RW - 4 * gg < i + 2) h &= 0xFFu;  // pixel i + 1 past the region
        *(uint16_t *)(sc + (ry + 1) * P + 4 * gg + 4 + i) = (uint16_t)h;
    };
    for (int j = lane; j < na; j += 64) score_pair(std::integral_constant<int, 0>{}, alist[j]);
    for (int j = lane; j < nb; j += 64) score_pair(std::integral_constant<int, 2>{}, blist[j]);
    wave_sync_lds();
    if (g->dbg == 12) return;

    // ---- NMS (cell-local) ----
    // cv::FAST keeps p iff s_p > every neighbour's score, a neighbour that is not a corner
    // at the cell threshold th counting as 0.  With s_p >= max(th, 1) that is exactly
    //   max(raw 8-neighbour scores) < max(th, s_p)
    // (a neighbour q < th is always below max(th, s_p); one with q >= th must be < s_p).
    // Pixel pairs in packed u16 lanes; keep bits (4 per unit) of unit (ry, gg).
    const v2s one = (v2s){1, 1};
    auto keep_bits = [&](int ry, int gg, int th) -> uint32_t {
        const v2s t1v = (v2s){(short)max(th, 1), (short)max(th, 1)};
        const v2s thv = (v2s){(short)th, (short)th};
        const uint32_t *mu = (const uint32_t *)(sc + ry * P + 4 * gg);
        const uint32_t *m0 = (const uint32_t *)(sc + (ry + 1) * P + 4 * gg);
        const uint32_t *md = (const uint32_t *)(sc + (ry + 2) * P + 4 * gg);
        const uint32_t c1 = m0[1];
        if (c1 == 0) return 0u;  // a unit with no scored pixel keeps nothing
        const uint32_t u0 = mu[0], u1 = mu[1], u2 = mu[2];
        const uint32_t c0 = m0[0], c2 = m0[2];
        const uint32_t d0 = md[0], d1 = md[1], d2 = md[2];
        // pixels 0,1 (bytes 4,5): neighbours at bytes 3..6
        v2s mA = pmax(pmax(gather2<3>(u0, u1, u2), gather2<4>(u0, u1, u2)), gather2<5>(u0, u1, u2));
        mA = pmax(mA, pmax(pmax(gather2<3>(d0, d1, d2), gather2<4>(d0, d1, d2)),
                           gather2<5>(d0, d1, d2)));
        mA = pmax(mA, pmax(gather2<3>(c0, c1, c2), gather2<5>(c0, c1, c2)));
        // pixels 2,3 (bytes 6,7): neighbours at bytes 5..8
        v2s mB = pmax(pmax(gather2<5>(u0, u1, u2), gather2<6>(u0, u1, u2)), gather2<7>(u0, u1, u2));
        mB = pmax(mB, pmax(pmax(gather2<5>(d0, d1, d2), gather2<6>(d0, d1, d2)),
                           gather2<7>(d0, d1, d2)));
        mB = pmax(mB, pmax(gather2<5>(c0, c1, c2), gather2<7>(c0, c1, c2)));
        const v2s sA = gather2<4>(c0, c1, c2), sB = gather2<6>(c0, c1, c2);
        // keep <=> min(s - t1, max(th, s) - M - 1) >= 0: sign bit of each u16 lane
        auto keep = [&](v2s sv, v2s m) -> uint32_t {
            const v2s k = pmin(sv - t1v, pmax(thv, sv) - m - one);
            const uint32_t w = __builtin_bit_cast(uint32_t, k);
            return (~w >> 15 & 1u) | (~w >> 30 & 2u);
        };
        uint32_t kb = keep(sA, mA) | keep(sB, mB) << 2;
        const int valid = min(RW - 4 * gg, 4);
        if (valid < 4) kb &= (1u << valid) - 1u;
        return kb;
    };
    // ---- raster-order compaction of one 64-unit chunk: lane's unit (ry, gg) keeps kb ----
    const int64_t slot = (int64_t)f * g->ncells + c;
    uint2 *out = cell_kp + slot * g->cell_cap;
    int run = 0;
    auto emit = [&](uint32_t kb, int ry, int gg) {
        const int n = __popc(kb);
        int tot;
        const int incl = wave_incl_scan_small(n, &tot);
        if (tot == 0) return;  // wave-uniform
        // path codes by shuffle, all lanes active (a lane past the region reads lane 0)
        const uint32_t cy = (uint32_t)__shfl((int)ys_l, ry & 63, 64);
        uint32_t cx[4];
#pragma unroll
        for (int i = 0; i < 4; i++) cx[i] = (uint32_t)__shfl((int)xs_l, (4 * gg + i) & 63, 64);
        if (kb) {
            int off = run + incl - n;
            const uint32_t c1 = *(const uint32_t *)(sc + (ry + 1) * P + 4 * gg + 4);
            const int x0 = xo + 4 * gg, y = yo + ry;
#pragma unroll
            for (int i = 0; i < 4; i++)
                if (kb & (1u << i))
                    out[off++] = make_uint2(orbg_pack(x0 + i, y, (c1 >> (8 * i)) & 0xFF),
                                            cx[i] | cy);
        }
        run += tot;
    };
    // FAST at iniThFAST: only units with a corner (nonzero score word) can keep a pixel;
    // they are listed in raster order (over the dead pair lists), then NMS + compaction walk
    // the list densely
    {
        int nc = 0;
        for (int u0 = 0, ry = ry0, gg = gg0; u0 < nunits; u0 += 64) {
            const bool corner =
                u0 + lane < nunits && *(const uint32_t *)(sc + (ry + 1) * P + 4 * gg + 4) != 0;
            const unsigned long long m = __ballot(corner);
            const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                        __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
            if (corner) plist[nc + below] = (uint16_t)(ry << 8 | gg);
            nc += __popcll(m);
            ry += rstep;
            gg += gstep;
            if (gg >= RG) {
                gg -= RG;
                ry++;
            }
        }
        npass = nc;
    }
    wave_sync_lds();
    for (int j0 = 0; j0 < npass; j0 += 64) {
        const int j = j0 + lane;
        int ry = 0, gg = 0;
        uint32_t kb = 0;
        if (j < npass) {
            const int e = plist[j];
            ry = e >> 8;
            gg = e & 0xFF;
            kb = keep_bits(ry, gg, thi);
        }
        emit(kb, ry, gg);
    }
    if (g->dbg == 13) return;
    if (run == 0) {
        // an empty cell retries at minThFAST (ORBextractor.cc:1069-1075) with every unit
        // scored (the window tile is still intact)
        wave_sync_lds();
        for (int u = lane, ry = ry0, gg = gg0; u < nunits; u += 64) {
            score_unit(ry, gg);
            ry += rstep;
            gg += gstep;
            if (gg >= RG) {
                gg -= RG;
                ry++;
            }
        }
        wave_sync_lds();
        for (int u0 = 0, ry = ry0, gg = gg0; u0 < nunits; u0 += 64) {
            const uint32_t kb = u0 + lane < nunits ? keep_bits(ry, gg, tlo) : 0u;
            emit(kb, ry, gg);
            ry += rstep;
            gg += gstep;
            if (gg >= RG) {
                gg -= RG;
                ry++;
            }
        }
    }
    if (lane == 0) cell_cnt[slot] = run;
}

// ---------------------------------------------------------------------------
// k_blur: GaussianBlur(7x7, sigma 2, BORDER_REFLECT_101), bit-exact fixed point
// out = sat((sum_v k_v * sum_h k_h * p + 2^15) >> 16).
// A 256-thread workgroup walks BLUR_NB vertical 128x32 output bands; the loads of band b+1
// are in flight while band b is computed.  The (128+8)x38 input tile (x origin at
// tile_x0 - 4) is filled with aligned dword pairs + v_alignbyte (REFLECT_101 bytes at the
// image edges), all loads issued before the LDS stores; the row pass keeps u16 sums
// (<= 256*255) in LDS; the column pass reads 4 sums per ds_read_b64 and stores 4 output
// pixels per dword.  The 1-D grid enumerates (frame, tile of any level), XCD-remapped.
// ---------------------------------------------------------------------------
#define BLUR_TW 128
#define BLUR_TH 32
#define BLUR_IW (BLUR_TW + 16)  // 9 x 16-byte chunks from x = tile_x0 - 4 (135 bytes read)
#define BLUR_IH (BLUR_TH + 6)
#define BLUR_NB ORBG_BLUR_NB  // bands per workgroup

// v_dot2_u32_u16 on u16 pairs held in u32 words
__device__ __forceinline__ uint32_t udot2_u32(uint32_t a, uint32_t b, uint32_t c)
{
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    return __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b), c,
                                  false);
}

__device__ __forceinline__ int reflect101(int i, int n)
{
    // single reflection suffices for the 3-pixel halo (n >= 4 for every level)
    i = i < 0 ? -i : i;
    return i >= n ? 2 * n - 2 - i : i;
}

__global__ __launch_bounds__(256) void k_blur(const OrbgGeom *__restrict__ g,
                                              const int32_t *__restrict__ tile_base,
                                              const uint8_t *__restrict__ img0, int64_t img_fs,
                                              int img_pitch, const uint8_t *__restrict__ pyr,
                                              uint8_t *__restrict__ blur, int tb_begin,
                                              int tb_count)
{
    __shared__ __attribute__((aligned(16))) uint8_t in[BLUR_IH][BLUR_IW];
    __shared__ __attribute__((aligned(16))) uint32_t rows[BLUR_IH / 2][BLUR_TW];  // row-pair sums
    // tiles [tb_begin, tb_begin + tb_count) of every frame (level 0 alone or levels 1..
    // alone when level 0 runs on the quadtree stream)
    const int id = xcd_remap(blockIdx.x, gridDim.x);
    const int f = id / tb_count, bt = tb_begin + id - f * tb_count, tid = threadIdx.x;
    int l = 0;
    while (l + 1 < g->L && bt >= tile_base[l + 1]) l++;
    const int t = bt - tile_base[l];
    const OrbgLevel &lv = g->lv[l];
    const int W = lv.w, H = lv.h;
    const int ntx = (W + BLUR_TW - 1) / BLUR_TW;
    const int ty = t / ntx;
    const int tx0 = (t - ty * ntx) * BLUR_TW, yr0 = ty * (BLUR_TH * BLUR_NB);
    const int nband = min(BLUR_NB, (H - yr0 + BLUR_TH - 1) / BLUR_TH);  // >= 1
    const uint8_t *src;
    int pitch;
    if (l == 0) {
        src = img0 + f * img_fs;
        pitch = img_pitch;
    } else {
        src = pyr + f * g->pyr_frame + lv.pyr_off;
        pitch = lv.pitch;
    }
    // fill of the band starting at output row ty0: column c of the tile is image
    // x = tx0 - 4 + c, row r is y = ty0 - 3 + r.  16-byte chunk c of a row = x0 .. x0+15
    // (x0 = tx0 - 4 + 16c): one dwordx4 from the aligned address + one dword for the
    // v_alignbyte shift when x0 .. x0+19 lies inside the row, else bytes with REFLECT_101
    // (image edges only).  The loads of band b+1 are issued before band b is computed.
    constexpr int NCH = BLUR_IW / 16;                      // chunks per row
    constexpr int NFILL = (BLUR_IH * NCH + 255) / 256;     // chunks per thread
    uint4 q[NFILL];
    uint32_t q4[NFILL], sh[NFILL];
    auto load_band = [&](int ty0) {
#pragma unroll
        for (int k = 0; k < NFILL; k++) {
            const int i = tid + 256 * k;
            q[k] = make_uint4(0, 0, 0, 0);
            q4[k] = sh[k] = 0;
            if (i < BLUR_IH * NCH) {
                const int r = i / NCH, c = i - r * NCH;
                const int y = reflect101(min(ty0 - 3 + r, H + 2), H);
                const uint8_t *row = src + (int64_t)y * pitch;
                const int x0 = tx0 - 4 + 16 * c;
                if (x0 >= 0 && x0 + 20 <= W) {
                    // pointer arithmetic (not an integer round trip): global_, not flat_, loads
                    const uint8_t *pa = row + x0;
                    sh[k] = (uint32_t)((uintptr_t)pa & 3);
                    const uint32_t *aw = (const uint32_t *)(pa - sh[k]);
                    q[k] = *(const uint4 *)aw;
                    if (sh[k]) q4[k] = aw[4];
                } else {
                    sh[k] = 4u;  // image-edge chunk: gathered byte-wise in store_band
                }
            }
        }
    };
    auto store_band = [&](int ty0) {
#pragma unroll
        for (int k = 0; k < NFILL; k++) {
            const int i = tid + 256 * k;
            if (i < BLUR_IH * NCH) {
                const int r = i / NCH, c = i - r * NCH;
                const uint32_t s = sh[k];
                uint4 o;
                if (s < 4u) {
                    o.x = __builtin_amdgcn_alignbyte(q[k].y, q[k].x, s);
                    o.y = __builtin_amdgcn_alignbyte(q[k].z, q[k].y, s);
                    o.z = __builtin_amdgcn_alignbyte(q[k].w, q[k].z, s);
                    o.w = __builtin_amdgcn_alignbyte(q4[k], q[k].w, s);
                } else {
                    const int y = reflect101(min(ty0 - 3 + r, H + 2), H);
                    const uint8_t *row = src + (int64_t)y * pitch;
                    int x0 = tx0 - 4 + 16 * c;
                    // opaque: keeps the 16 reflected column indices from being hoisted out
                    // of the band loop (32 VGPRs held across it)
                    asm volatile("" : "+v"(x0));
                    uint32_t w4[4] = {0, 0, 0, 0};
#pragma unroll
                    for (int bb = 0; bb < 16; bb++)
                        w4[bb >> 2] |= (uint32_t)row[reflect101(min(x0 + bb, W + 2), W)]
                                       << (8 * (bb & 3));
                    o = make_uint4(w4[0], w4[1], w4[2], w4[3]);
                }
                *(uint4 *)&in[r][16 * c] = o;
            }
        }
    };
    const uint32_t k0 = g->gk[0], k1 = g->gk[1], k2 = g->gk[2], k3 = g->gk[3], k4 = g->gk[4],
                   k5 = g->gk[5], k6 = g->gk[6];
    const uint32_t ksum = k0 + k1 + k2 + k3 + k4 + k5 + k6;
    // row pass weights: output x = 4j+i of a row needs tile bytes 4j+1+i .. 4j+7+i, i.e. the
    // aligned dwords W0..W2 = bytes 4j .. 4j+11 against the 7 weights placed at byte 1+i
    const uint32_t K00 = k0 << 8 | k1 << 16 | k2 << 24, K01 = k3 | k4 << 8 | k5 << 16 | k6 << 24;
    const uint32_t K10 = k0 << 16 | k1 << 24, K11 = k2 | k3 << 8 | k4 << 16 | k5 << 24, K12 = k6;
    const uint32_t K20 = k0 << 24, K21 = k1 | k2 << 8 | k3 << 16 | k4 << 24, K22 = k5 | k6 << 8;
    const uint32_t K31 = k0 | k1 << 8 | k2 << 16 | k3 << 24, K32 = k4 | k5 << 8 | k6 << 16;
    // column pass weights aligned to the output's parity (even o: (k0,k1)(k2,k3)(k4,k5)(k6,0);
    // odd o: (0,k0)(k1,k2)(k3,k4)(k5,k6))
    const uint32_t E0 = k0 | k1 << 16, E1 = k2 | k3 << 16, E2 = k4 | k5 << 16, E3 = k6;
    const uint32_t O0 = k0 << 16, O1 = k1 | k2 << 16, O2 = k3 | k4 << 16, O3 = k5 | k6 << 16;
    uint8_t *dst = blur + f * g->blur_frame + lv.blur_off;
    const int j = tid & 31, rg = tid >> 5;  // column pass: 4-column group j, 4-row group rg
    const int gx = tx0 + 4 * j;
    load_band(yr0);
#pragma unroll 1
    for (int b = 0; b < nband; b++) {  // workgroup-uniform trip count
        const int ty0 = yr0 + b * BLUR_TH;
        // every thread is past the previous band's row pass (barrier below), so in[] is free
        store_band(ty0);
        __syncthreads();  // in[] complete; every thread's previous column pass is done
        if (b + 1 < nband) load_band(ty0 + BLUR_TH);
        // row pass: unit = (row pair rp, 4-column group jj): ten v_dot4_u32_u8 per 4 outputs
        // (row sums <= 257 * 255, exact); the two rows' sums of a column are stored as one
        // u16 pair, rows[rp][x] = sum(2rp, x) | sum(2rp+1, x) << 16, for the column pass
        for (int u = tid; u < (BLUR_IH / 2) * (BLUR_TW / 4); u += 256) {
            const int rp = u >> 5, jj = u & 31;
            uint32_t sm[2][4];
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const uint32_t *w = (const uint32_t *)&in[2 * rp + h][4 * jj];
                const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
                sm[h][0] = __builtin_amdgcn_udot4(w1, K01, __builtin_amdgcn_udot4(w0, K00, 0u, false), false);
                sm[h][1] = __builtin_amdgcn_udot4(w2, K12, __builtin_amdgcn_udot4(w1, K11, __builtin_amdgcn_udot4(w0, K10, 0u, false), false), false);
                sm[h][2] = __builtin_amdgcn_udot4(w2, K22, __builtin_amdgcn_udot4(w1, K21, __builtin_amdgcn_udot4(w0, K20, 0u, false), false), false);
                sm[h][3] = __builtin_amdgcn_udot4(w2, K32, __builtin_amdgcn_udot4(w1, K31, 0u, false), false);
            }
            uint4 pk;
            pk.x = sm[0][0] | sm[1][0] << 16;
            pk.y = sm[0][1] | sm[1][1] << 16;
            pk.z = sm[0][2] | sm[1][2] << 16;
            pk.w = sm[0][3] | sm[1][3] << 16;
            *(uint4 *)&rows[rp][4 * jj] = pk;
        }
        __syncthreads();
        // column pass: outputs o = 4rg .. 4rg+3 from tile rows o .. o+6, i.e. row pairs
        // 2rg .. 2rg+4; four v_dot2_u32_u16 per output (sums <= 257 * 65535 fit 32 bits)
        // weights summing to 256 (the >= 3.4.9 table): S + 2^15 < 2^24, so the output byte is
        // byte 2 of the sum with the rounding term as the dot2 chain's initial value -- no
        // saturation, four outputs packed by two v_perm; the legacy table (sum 257) keeps
        // the saturating path
        const bool norm256 = ksum == 256u;
        const uint32_t c0 = norm256 ? (1u << 15) : 0u;
        uint32_t acc[4][4];
        {
            uint4 P[5];
#pragma unroll
            for (int qq = 0; qq < 5; qq++) P[qq] = *(const uint4 *)&rows[2 * rg + qq][4 * j];
#pragma unroll
            for (int bc = 0; bc < 4; bc++) {
                auto col = [&](int qq) -> uint32_t {
                    return bc == 0 ? P[qq].x : bc == 1 ? P[qq].y : bc == 2 ? P[qq].z : P[qq].w;
                };
#pragma unroll
                for (int o = 0; o < 4; o++) {
                    const int m = o >> 1;  // first pair of output 4rg+o: 2rg + m
                    uint32_t a2;
                    if ((o & 1) == 0) {
                        a2 = udot2_u32(col(m), E0, c0);
                        a2 = udot2_u32(col(m + 1), E1, a2);
                        a2 = udot2_u32(col(m + 2), E2, a2);
                        a2 = udot2_u32(col(m + 3), E3, a2);
                    } else {
                        a2 = udot2_u32(col(m), O0, c0);
                        a2 = udot2_u32(col(m + 1), O1, a2);
                        a2 = udot2_u32(col(m + 2), O2, a2);
                        a2 = udot2_u32(col(m + 3), O3, a2);
                    }
                    acc[o][bc] = a2;
                }
            }
        }
#pragma unroll
        for (int o = 0; o < 4; o++) {
            const int gy = ty0 + 4 * rg + o;
            if (gy >= H || gx >= W) continue;
            uint32_t word;
            if (norm256) {
                // bytes 2 of acc[o][0..3]: perm(b, a) picks byte 2 of a (sel 2) and of b (sel 6)
                const uint32_t lo = __builtin_amdgcn_perm(acc[o][1], acc[o][0], 0x0c0c0602u);
                const uint32_t hi = __builtin_amdgcn_perm(acc[o][3], acc[o][2], 0x06020c0cu);
                word = lo | hi;
            } else {
                word = 0;
#pragma unroll
                for (int bc = 0; bc < 4; bc++) word |= min((acc[o][bc] + (1u << 15)) >> 16, 255u) << (8 * bc);
            }
            uint8_t *d = dst + (int64_t)gy * lv.pitch + gx;
            if (gx + 4 <= W) {
                *(uint32_t *)d = word;  // pitch is a multiple of 64, gx of 4: aligned
            } else {
                for (int bc = 0; bc < 4 && gx + bc < W; bc++) d[bc] = (uint8_t)(word >> (8 * bc));
            }
        }
    }
}

// ---------------------------------------------------------------------------
// k_octree: DistributeOctTree for one (level, frame) per 256-thread workgroup.
//
// Node records (global, per frame/level region): int4 {x0 | y0<<16, x1 | y1<<16, cnt, tag}.
// Node ids are bump-allocated in the reference's creation order (parents in processing
// order, children n1..n4), so "id order" == "creation order" == the pinned pointer
// tie-break of the sort at ORBextractor.cc:869.  The std::list is an array of node ids
// in list order (LDS); each pass rebuilds it with the exact push_front / erase order:
//   [children of the last split parent (n4..n1), ..., children of the first], then the
//   untouched nodes in their previous order.
// Keys carry their node id (knode); only keys of multi-key nodes ("active") are touched.
// ---------------------------------------------------------------------------

struct OctShared {
    uint16_t ord[2][ORBG_OCT_ALIVE];
    uint16_t aux[ORBG_OCT_ALIVE];          // split-before counts / processing list
    uint16_t childid[4 * ORBG_OCT_ALIVE];
    union {
        uint32_t ccnt[4 * ORBG_OCT_ALIVE];
        unsigned long long sortk[2 * ORBG_OCT_ALIVE];
        uint32_t best[4 * ORBG_OCT_ALIVE];
    } u;
    int rootcnt[64];
    int red[8];
    int s_alive, s_cur, s_nact, s_newact, s_nalloc, s_finish, s_phase2, s_err;
    int s_nsplit, s_tote, s_nexp, s_nproc, s_vbase, s_vend, s_prev;
};

__device__ __forceinline__ int node_x0(int4 n) { return n.x & 0xFFFF; }
__device__ __forceinline__ int node_y0(int4 n) { return n.x >> 16; }
__device__ __forceinline__ int node_x1(int4 n) { return n.y & 0xFFFF; }
__device__ __forceinline__ int node_y1(int4 n) { return n.y >> 16; }

// DivideNode quadrant of a key (ORBextractor.cc:539-594)
__device__ __forceinline__ int quadrant(int4 n, uint32_t key)
{
    const int x0 = node_x0(n), y0 = node_y0(n), x1 = node_x1(n), y1 = node_y1(n);
    const int halfX = (int)ceilf((float)(x1 - x0) / 2);
    const int halfY = (int)ceilf((float)(y1 - y0) / 2);
    const float kx = (float)orbg_px(key), ky = (float)orbg_py(key);
    const bool left = kx < (float)(x0 + halfX);
    const bool top = ky < (float)(y0 + halfY);
    return left ? (top ? 0 : 2) : (top ? 1 : 3);
}

__device__ __forceinline__ int4 child_rect(int4 n, int q, int cnt)
{
    const int x0 = node_x0(n), y0 = node_y0(n), x1 = node_x1(n), y1 = node_y1(n);
    const int halfX = (int)ceilf((float)(x1 - x0) / 2);
    const int halfY = (int)ceilf((float)(y1 - y0) / 2);
    const int xm = x0 + halfX, ym = y0 + halfY;
    int cx0, cy0, cx1, cy1;
    switch (q) {
    case 0: cx0 = x0; cy0 = y0; cx1 = xm; cy1 = ym; break;
    case 1: cx0 = xm; cy0 = y0; cx1 = x1; cy1 = ym; break;
    case 2: cx0 = x0; cy0 = ym; cx1 = xm; cy1 = y1; break;
    default: cx0 = xm; cy0 = ym; cx1 = x1; cy1 = y1; break;
    }
    return make_int4((cx0 & 0xFFFF) | (cy0 << 16), (cx1 & 0xFFFF) | (cy1 << 16), cnt, -1);
}

__global__ __launch_bounds__(ORBG_OCT_THREADS) void k_octree(
    const OrbgGeom *__restrict__ g, const int32_t *__restrict__ cell_cnt,
    const uint2 *__restrict__ cell_kp, uint32_t *__restrict__ keys_all,
    uint32_t *__restrict__ knode_all, uint32_t *__restrict__ act_all,
    uint8_t *__restrict__ qk_all, int4 *__restrict__ nodes_all, uint32_t *__restrict__ lvl_kp,
    int32_t *__restrict__ lvl_cnt, int32_t *__restrict__ err_flag)
{
    __shared__ OctShared S;
    const int l = blockIdx.x, f = blockIdx.y, tid = threadIdx.x;
    const int nthr = blockDim.x;
    const OrbgLevel &lv = g->lv[l];
    const int64_t kbase = (int64_t)f * g->keys_frame + lv.key_off;
    uint32_t *keys = keys_all + kbase;
    uint32_t *knode = knode_all + kbase;
    uint32_t *actA = act_all + 2 * kbase;
    uint32_t *actB = actA + lv.key_cap;
    uint8_t *qk = qk_all + kbase;
    int4 *nodes = nodes_all + (int64_t)f * g->nodes_frame + lv.node_off;
    const int N = lv.nfeat;
    const int nIni = lv.nini;
    const float hX = lv.hx;
    const int rootH = lv.max_by - ORBG_MIN_BORDER;

    // ---- gather candidates of this level's cells in cell order (vToDistributeKeys) ----
    const int32_t *ccount = cell_cnt + (int64_t)f * g->ncells + lv.cell_base;
    const uint2 *ckp = cell_kp + ((int64_t)f * g->ncells + lv.cell_base) * g->cell_cap;
    int n = 0;
    {
        int run = 0;
        for (int c0 = 0; c0 < lv.ncells; c0 += nthr) {
            const int c = c0 + tid;
            int tot;
            block_excl_scan(c < lv.ncells ? ccount[c] : 0, &tot, S.red);
            run += tot;
        }
        if (run <= lv.oct_kcap && lv.ncells + 1 <= lv.oct_acap2) return;  // k_octree_lds
        if (g->dbg == 91) {
            // fault injection (ORBG_DBG=91, tests only): this fallback disabled, so a level
            // past k_octree_lds' capacity is an overflow -- the error path the host must surface
            if (tid == 0) {
                atomicOr(err_flag, 1 << 9);
                atomicMin(err_flag + 1, f);
                lvl_cnt[(int64_t)f * g->L + l] = 0;
            }
            return;
        }
        run = 0;
        for (int c0 = 0; c0 < lv.ncells; c0 += nthr) {
            const int c = c0 + tid;
            const int cn = c < lv.ncells ? ccount[c] : 0;
            int tot;
            const int off = block_excl_scan(cn, &tot, S.red) + run;
            for (int i = 0; i < cn; i++) keys[off + i] = ckp[(int64_t)c * g->cell_cap + i].x;
            run += tot;
        }
        n = run;
    }
    if (tid < 64) S.rootcnt[tid] = 0;
    if (tid == 0) {
        S.s_err = 0;
        S.s_finish = 0;
    }
    __syncthreads();

    // ---- roots (:674-739) ----
    for (int k = tid; k < n; k += nthr) {
        const int r = min((int)((float)orbg_px(keys[k]) / hX), nIni - 1);
        knode[k] = (uint32_t)r;
        atomicAdd(&S.rootcnt[r], 1);
    }
    __syncthreads();
    if (tid == 0) {
        int a = 0;
        for (int i = 0; i < nIni; i++) {
            const int x0 = (int)(hX * (float)i), x1 = (int)(hX * (float)(i + 1));
            nodes[i] = make_int4((x0 & 0xFFFF), (x1 & 0xFFFF) | (rootH << 16), S.rootcnt[i], -1);
            if (S.rootcnt[i] > 0) S.ord[0][a++] = (uint16_t)i;
        }
        S.s_alive = a;
        S.s_cur = 0;
        S.s_nalloc = nIni;
        S.s_nact = 0;
        S.s_phase2 = 0;
    }
    __syncthreads();
    for (int k = tid; k < n; k += nthr) {
        if (S.rootcnt[knode[k]] > 1) {
            const int j = atomicAdd(&S.s_nact, 1);
            actA[j] = (uint32_t)k;
        }
    }
    __syncthreads();

    uint32_t *act = actA, *act2 = actB;
    // ================= phase 1 passes (:751-852) =================
    while (true) {
        const int alive = S.s_alive, cur = S.s_cur, nact = S.s_nact;
        // (a) rank the nodes to split (cnt > 1) in list order
        int run = 0;
        for (int i0 = 0; i0 < alive; i0 += nthr) {
            const int i = i0 + tid;
            int fl = 0, nd = 0;
            if (i < alive) {
                nd = S.ord[cur][i];
                fl = nodes[nd].z > 1;
            }
            int tot;
            const int r = block_excl_scan(fl, &tot, S.red) + run;
            if (i < alive) {
                nodes[nd].w = fl ? r : -1;
                S.aux[i] = (uint16_t)r;  // # split nodes before position i
            }
            run += tot;
        }
        const int nsplit = run;
        for (int i = tid; i < 4 * nsplit; i += nthr) S.u.ccnt[i] = 0;
        __syncthreads();
        // (c) count keys per child
        for (int j = tid; j < nact; j += nthr) {
            const uint32_t k = act[j];
            const int4 nd = nodes[knode[k]];
            const int q = quadrant(nd, keys[k]);
            qk[j] = (uint8_t)q;
            atomicAdd(&S.u.ccnt[4 * nd.w + q], 1u);
        }
        __syncthreads();
        // (d) allocate children in creation order (parents in list order, n1..n4) and place
        //     them in the new list
        const int nalloc = S.s_nalloc;
        const int nxt = cur ^ 1;
        int tot_e = 0, nexp = 0;
        for (int r0 = 0; r0 < nsplit; r0 += nthr) {
            const int r = r0 + tid;
            int e = 0, m = 0;
            if (r < nsplit) {
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const uint32_t c = S.u.ccnt[4 * r + q];
                    e += c > 0;
                    m += c > 1;
                }
            }
            tot_e += block_sum(e, S.red);
            nexp += block_sum(m, S.red);
        }
        // second sweep (parents must be located by rank): iterate list positions
        __syncthreads();
        {
            int prefix_e = 0;
            for (int i0 = 0; i0 < alive; i0 += nthr) {
                const int i = i0 + tid;
                int nd = 0, r = -1, e = 0;
                uint32_t cc[4] = {0, 0, 0, 0};
                if (i < alive) {
                    nd = S.ord[cur][i];
                    r = nodes[nd].w;
                    if (r >= 0) {
#pragma unroll
                        for (int q = 0; q < 4; q++) {
                            cc[q] = S.u.ccnt[4 * r + q];
                            e += cc[q] > 0;
                        }
                    }
                }
                int tote;
                const int E = block_excl_scan(e, &tote, S.red) + prefix_e;
                if (i < alive) {
                    if (r >= 0) {
                        const int4 par = nodes[nd];
                        const int blk = tot_e - E - e;  // children of later parents come first
                        int k = 0;
#pragma unroll
                        for (int q = 0; q < 4; q++) {
                            if (cc[q] == 0) continue;
                            const int id = nalloc + E + k;
                            nodes[id] = child_rect(par, q, (int)cc[q]);
                            S.childid[4 * r + q] = (uint16_t)id;
                            S.ord[nxt][blk + (e - 1 - k)] = (uint16_t)id;
                            k++;
                        }
                    } else {
                        S.ord[nxt][tot_e + i - S.aux[i]] = (uint16_t)nd;
                    }
                }
                prefix_e += tote;
            }
        }
        if (tid == 0) {
            const int na = tot_e + alive - nsplit;
            S.s_alive = na;
            S.s_cur = nxt;
            S.s_nalloc = nalloc + tot_e;
            S.s_nexp = nexp;
            S.s_newact = 0;
            if (na > ORBG_OCT_ALIVE || nalloc + tot_e > lv.node_cap) S.s_err = 1;
        }
        __syncthreads();
        if (S.s_err) break;
        // (e) move keys to their children; keep keys of multi-key children active
        for (int j = tid; j < nact; j += nthr) {
            const uint32_t k = act[j];
            const int r = nodes[knode[k]].w;
            const int id = S.childid[4 * r + qk[j]];
            knode[k] = (uint32_t)id;
            if (nodes[id].z > 1) {
                const int t = atomicAdd(&S.s_newact, 1);
                act2[t] = k;
            }
        }
        __syncthreads();
        if (tid == 0) {
            S.s_nact = S.s_newact;
            S.s_vbase = nalloc;
            S.s_vend = nalloc + tot_e;
        }
        {
            uint32_t *t = act;
            act = act2;
            act2 = t;
        }
        __syncthreads();
        const int na = S.s_alive;
        if (na >= N || na == alive) break;                    // :849-852
        if (na + S.s_nexp * 3 > N) {                          // :856
            if (tid == 0) S.s_phase2 = 1;
            __syncthreads();
            break;
        }
    }

    // ================= phase 2 rounds (:859-924) =================
    if (S.s_phase2 && !S.s_err) {
        while (true) {
            const int alive = S.s_alive, cur = S.s_cur, nact = S.s_nact;
            const int vbase = S.s_vbase, vend = S.s_vend;
            const int prevSize = alive;
            // gather vPrevSizeAndPointerToNode = multi-key nodes created last round (id order)
            int runv = 0;
            for (int i0 = vbase; i0 < vend; i0 += nthr) {
                const int id = i0 + tid;
                int fl = 0, cnt = 0;
                if (id < vend) {
                    cnt = nodes[id].z;
                    fl = cnt > 1;
                }
                int tot;
                const int r = block_excl_scan(fl, &tot, S.red) + runv;
                if (fl) S.u.sortk[r] = ((unsigned long long)cnt << 32) | (unsigned)id;
                runv += tot;
            }
            const int np = runv;
            if (np > ORBG_OCT_ALIVE) {
                if (tid == 0) S.s_err = 2;
                __syncthreads();
                break;
            }
            int pw = 1;
            while (pw < np) pw <<= 1;
            for (int i = np + tid; i < pw; i += nthr) S.u.sortk[i] = ~0ull;
            __syncthreads();
            // bitonic sort ascending by (size, id)
            for (int k = 2; k <= pw; k <<= 1)
                for (int j = k >> 1; j > 0; j >>= 1) {
                    for (int i = tid; i < pw; i += nthr) {
                        const int ixj = i ^ j;
                        if (ixj > i) {
                            const unsigned long long a = S.u.sortk[i], b = S.u.sortk[ixj];
                            const bool up = (i & k) == 0;
                            if ((a > b) == up) {
                                S.u.sortk[i] = b;
                                S.u.sortk[ixj] = a;
                            }
                        }
                    }
                    __syncthreads();
                }
            // processing order p: largest first (:872); tag parents with p
            for (int p = tid; p < np; p += nthr) {
                const int id = (int)(S.u.sortk[np - 1 - p] & 0xFFFFFFFFu);
                S.aux[p] = (uint16_t)id;
            }
            __syncthreads();
            for (int p = tid; p < np; p += nthr) nodes[S.aux[p]].w = p;
            for (int i = tid; i < 4 * np; i += nthr) S.u.ccnt[i] = 0;
            __syncthreads();
            for (int j = tid; j < nact; j += nthr) {
                const uint32_t k = act[j];
                const int4 nd = nodes[knode[k]];
                if (nd.w >= 0) {
                    const int q = quadrant(nd, keys[k]);
                    qk[j] = (uint8_t)q;
                    atomicAdd(&S.u.ccnt[4 * nd.w + q], 1u);
                }
            }
            __syncthreads();
            // cut: first p with alive + sum_{p' <= p} (e_p' - 1) >= N  (break at :917-918)
            if (tid == 0) S.s_nproc = np;
            __syncthreads();
            {
                int runs = 0;
                for (int p0 = 0; p0 < np; p0 += nthr) {
                    const int p = p0 + tid;
                    int dlt = 0;
                    if (p < np) {
                        int e = 0;
#pragma unroll
                        for (int q = 0; q < 4; q++) e += S.u.ccnt[4 * p + q] > 0;
                        dlt = e - 1;
                    }
                    int tot;
                    const int incl = block_excl_scan(dlt, &tot, S.red) + runs + dlt;
                    if (p < np && alive + incl >= N) atomicMin(&S.s_nproc, p + 1);
                    runs += tot;
                }
            }
            __syncthreads();
            const int nproc = S.s_nproc;
            const int nalloc = S.s_nalloc;
            const int nxt = cur ^ 1;
            // children of processed parents, creation order = processing order
            int tot_e = 0;
            {
                int rune = 0;
                for (int p0 = 0; p0 < nproc; p0 += nthr) {
                    const int p = p0 + tid;
                    int e = 0;
                    uint32_t cc[4] = {0, 0, 0, 0};
                    if (p < nproc) {
#pragma unroll
                        for (int q = 0; q < 4; q++) {
                            cc[q] = S.u.ccnt[4 * p + q];
                            e += cc[q] > 0;
                        }
                    }
                    int tote;
                    const int E = block_excl_scan(e, &tote, S.red) + rune;
                    if (p < nproc) {
                        const int4 par = nodes[S.aux[p]];
                        int k = 0;
#pragma unroll
                        for (int q = 0; q < 4; q++) {
                            if (cc[q] == 0) continue;
                            const int id = nalloc + E + k;
                            nodes[id] = child_rect(par, q, (int)cc[q]);
                            S.childid[4 * p + q] = (uint16_t)id;
                            k++;
                        }
                    }
                    rune += tote;
                }
                tot_e = rune;
            }
            __syncthreads();
            // new list: children blocks in reverse processing order (n4..n1 inside), then
            // the old list minus the processed parents.  Block of p starts at tot_e - E_p - e_p.
            {
                int rune = 0;
                for (int p0 = 0; p0 < nproc; p0 += nthr) {
                    const int p = p0 + tid;
                    int e = 0;
                    if (p < nproc) {
#pragma unroll
                        for (int q = 0; q < 4; q++) e += S.u.ccnt[4 * p + q] > 0;
                    }
                    int tote;
                    const int E = block_excl_scan(e, &tote, S.red) + rune;
                    if (p < nproc) {
                        const int blk = tot_e - E - e;
                        int k = 0;
#pragma unroll
                        for (int q = 0; q < 4; q++) {
                            if (S.u.ccnt[4 * p + q] == 0) continue;
                            S.ord[nxt][blk + (e - 1 - k)] = S.childid[4 * p + q];
                            k++;
                        }
                    }
                    rune += tote;
                }
                int runp = 0;
                for (int i0 = 0; i0 < alive; i0 += nthr) {
                    const int i = i0 + tid;
                    int fl = 0, nd = 0;
                    if (i < alive) {
                        nd = S.ord[cur][i];
                        const int w = nodes[nd].w;
                        fl = (w >= 0 && w < nproc);
                    }
                    int tot;
                    const int before = block_excl_scan(fl, &tot, S.red) + runp;
                    if (i < alive && !fl) S.ord[nxt][tot_e + i - before] = (uint16_t)nd;
                    runp += tot;
                }
            }
            if (tid == 0) {
                S.s_newact = 0;
                const int na = tot_e + alive - nproc;
                S.s_alive = na;
                if (na > ORBG_OCT_ALIVE || nalloc + tot_e > lv.node_cap) S.s_err = 3;
            }
            __syncthreads();
            if (S.s_err) break;
            for (int j = tid; j < nact; j += nthr) {
                const uint32_t k = act[j];
                const int nid0 = knode[k];
                const int p = nodes[nid0].w;
                int id = nid0;
                if (p >= 0 && p < nproc) {
                    id = S.childid[4 * p + qk[j]];
                    knode[k] = (uint32_t)id;
                }
                if (nodes[id].z > 1) {
                    const int t = atomicAdd(&S.s_newact, 1);
                    act2[t] = k;
                }
            }
            __syncthreads();
            for (int p = tid; p < np; p += nthr) nodes[S.aux[p]].w = -1;
            if (tid == 0) {
                S.s_nact = S.s_newact;
                S.s_cur = nxt;
                S.s_nalloc = nalloc + tot_e;
                S.s_vbase = nalloc;
                S.s_vend = nalloc + tot_e;
            }
            {
                uint32_t *t = act;
                act = act2;
                act2 = t;
            }
            __syncthreads();
            const int na = S.s_alive;
            if (na >= N || na == prevSize) break;  // :921-922
        }
    }

    // ================= keep the best key of each node (:932-948) =================
    const int alive = S.s_alive, cur = S.s_cur;
    if (S.s_err) {
        if (tid == 0) {
            atomicOr(err_flag, 1 << S.s_err);
            atomicMin(err_flag + 1, f);
            lvl_cnt[(int64_t)f * g->L + l] = 0;
        }
        return;
    }
    for (int i = tid; i < alive; i += nthr) {
        nodes[S.ord[cur][i]].w = i;
        S.u.best[i] = 0;
    }
    __syncthreads();
    for (int k = tid; k < n; k += nthr) {
        const uint32_t key = keys[k];
        const int pos = nodes[knode[k]].w;
        atomicMax(&S.u.best[pos], ((uint32_t)orbg_ps(key) << 24) | (0xFFFFFFu - (uint32_t)k));
    }
    __syncthreads();
    uint32_t *out = lvl_kp + (int64_t)f * g->out_frame + lv.out_off;
    const int nout = min(alive, lv.out_cap);
    for (int i = tid; i < nout; i += nthr) {
        const uint32_t k = 0xFFFFFFu - (S.u.best[i] & 0xFFFFFFu);
        out[i] = keys[k];
    }
    if (tid == 0) {
        lvl_cnt[(int64_t)f * g->L + l] = nout;
        if (alive > lv.out_cap) {
            atomicOr(err_flag, 1 << 8);
            atomicMin(err_flag + 1, f);
        }
    }
}

}  // namespace orbg
