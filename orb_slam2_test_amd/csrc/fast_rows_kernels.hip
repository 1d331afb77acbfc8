// fast_rows_kernels.hip -- k_fast_rows: the FAST part of ComputeKeyPointsOctTree
// (ORBextractor.cc:966-1094: 30-px cells, cv::FAST(window, iniThFAST, NMS), the minThFAST
// retry of empty cells, kp.pt += (j * wCell, i * hCell)) for gfx950, streamed row by row over
// a strip of up to 8 cells of one cell row.
//
// k_fast2 gives a wave one 30-px cell: it stages the cell's window into LDS, pretests its 4-pixel
// units, scores the survivors from a task list and runs FAST's NMS per unit -- a cell's task list
// rarely fills the wave's last scoring iteration, and every phase waits on its own loads.  Here a
// wave owns a strip of consecutive cells of one cell row (<= 256 px: lane l owns the strip's pixels
// 4l .. 4l+3, a unit may straddle two cells) and walks the strip's window rows top to bottom:
//   row      one 16-byte global load per lane and row, issued FR_PF rows ahead (coalesced: the
//            strip's row is one contiguous segment), v_alignbyte to the window's byte 0, one LDS
//            store into a ring of window rows (slots 0..5 mirrored after the ring, so the seven
//            rows of a pixel are always consecutive slots);
//   pretest  region row y as soon as window row y + 6 is in: FAST's compass test at the
//            threshold, bright and dark apart, survivors (pixel pair, side) ballot-compacted
//            into one list for FR_G rows of the whole strip (all cells pooled);
//   score    every FR_G rows: one side of one pixel pair per lane task, cornerScore's arc
//            extremes (fast_device.h), scores below the threshold stored as 0, into a ring of
//            score rows;
//   NMS      the rows whose neighbours are all scored: units with a score listed, the 8-neighbour
//            maxima with the columns of another cell masked out (cv::FAST runs per cell window:
//            a neighbour outside the cell's region counts 0), kept pixels into a row bitmap;
//   emit     lane (cell, row): the cell's bits of the row, a per-cell prefix over the rows, the
//            packed {x | y << 12 | score << 24, quadtree path code} records in raster order.
// A cell with no keypoint at iniThFAST is redone at minThFAST (ORBextractor.cc:1069-1075) by a
// second pass over the strip restricted to the empty cells' pixels.  Output: exactly k_fast2's
// (d_cell_cnt, d_cell_kp), bit for bit.
#include <hip/hip_runtime.h>

#include "orbg_internal.h"
#include "orbg_device.h"
#include "fast_device.h"

#pragma clang fp contract(off)

namespace orbg {

#define FR_G 4                 // region rows per scoring group
#define FR_RR (FR_G + 6)       // window ring rows (a group's rows and their +-3 halo)
#define FR_TR (FR_RR + 6)      // ring slots incl. the mirror of slots 0..5
#define FR_RS (FR_G + 3)       // score ring rows
#define FR_SB 272              // ring row bytes: 68 dwords, consecutive rows 4 banks apart
#define FR_SS (FR_SB / 4)
#define FR_LCAP (2 * 64 * FR_G)  // pretest list entries (at most 2 per unit and row)
#define FR_PF 4                // window rows in flight per lane (== FR_G: static ring slots)
#define FR_TR_OFF 0
#define FR_SR_OFF (FR_TR_OFF + FR_TR * FR_SB)
#define FR_LIST_OFF (FR_SR_OFF + FR_RS * FR_SB)
#define FR_BM_OFF (FR_LIST_OFF + ((2 * (FR_LCAP + 1) + 15) & ~15))
#define FR_RUN_OFF (FR_BM_OFF + 8 * 32)
#define FR_VM_OFF (FR_RUN_OFF + 32)
#define FR_WAVE_BYTES (FR_VM_OFF + 64)
static_assert(FR_PF == FR_G, "the unrolled group loop indexes the load ring statically");

int fast_rows_wave_bytes() { return FR_WAVE_BYTES; }

__global__ __launch_bounds__(256) void k_fast_rows(
    const OrbgGeom *__restrict__ g, const OrbgFastTile *__restrict__ tiles,
    const uint8_t *__restrict__ img0, int64_t img_fs, int img_pitch,
    const uint8_t *__restrict__ pyr, const uint32_t *__restrict__ ctab,
    int32_t *__restrict__ cell_cnt, uint2 *__restrict__ cell_kp, int nframes, int t_begin,
    int t_count)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t fr_lds[];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int wid = __builtin_amdgcn_readfirstlane(xcd_remap(blockIdx.x, gridDim.x) * 4 + wv);
    if (wid >= t_count * nframes) return;  // wave-uniform; no workgroup barrier below
    uint8_t *lds = (uint8_t *)fr_lds + wv * FR_WAVE_BYTES;
    uint8_t *TR = lds + FR_TR_OFF;
    uint8_t *SR = lds + FR_SR_OFF;
    uint16_t *list = (uint16_t *)(lds + FR_LIST_OFF);
    uint32_t *BM = (uint32_t *)(lds + FR_BM_OFF);
    int32_t *RUNS = (int32_t *)(lds + FR_RUN_OFF);
    uint8_t *VM = lds + FR_VM_OFF;

    // strip record + level geometry through the scalar cache
    const int f = wid / t_count, t = t_begin + wid - f * t_count;
    const uint4 tw4 = ((const uint4 *)tiles)[t];
    const uint32_t q0 = __builtin_amdgcn_readfirstlane(tw4.x);
    const int c0 = (int)__builtin_amdgcn_readfirstlane(tw4.y);
    const uint32_t q2 = __builtin_amdgcn_readfirstlane(tw4.z);
    const uint32_t q3 = __builtin_amdgcn_readfirstlane(tw4.w);
    const int l = (int)(int16_t)(q0 & 0xFFFF), ncell = (int)(int16_t)(q0 >> 16);
    const int x0 = (int)(int16_t)(q2 & 0xFFFF), y0 = (int)(int16_t)(q2 >> 16);
    const int H = (int)(int16_t)(q3 & 0xFFFF), tw = (int)(int16_t)(q3 >> 16);
    const int RH = H - 6;
    const OrbgLevel &lv = g->lv[l];
    const int wc = lv.wcell;
    const uint8_t *base;
    int pitch;
    if (l == 0) {
        base = img0 + f * img_fs;
        pitch = img_pitch;
    } else {
        base = pyr + f * g->pyr_frame + lv.pyr_off;
        pitch = lv.pitch;
    }
    const uint8_t *win = base + (int64_t)y0 * pitch + x0;
    const int thi = g->ini_th, tlo = g->min_th;
    // developer phase stops (ORBG_DBG, developer builds; 0 in the product library): 31 window
    // rows only, 32 + pretest, 33 + scoring, 34 + NMS -- wrong outputs by design
    const int dbg = g->dbg;
    const int ncells = g->ncells, cell_cap = g->cell_cap;
    const int xs = lv.xs_off + x0 + 3 - ORBG_MIN_BORDER;  // path code of strip pixel 0's column
    const int ys = lv.ys_off + y0 + 3 - ORBG_MIN_BORDER;  // ... of region row 0
    // window dwords the ring holds: 0 .. D-1 (lane l's own dword l, lane 63 also 64, 65)
    const int D = min((tw + 6 + 3) >> 2, 66);
    const int lane_c = min(lane, D - 1);  // lanes past the window re-read its last dword
    // the strip cell of each of the lane's pixels (pass 2 selects the empty cells' pixels)
    int pcell[4];
#pragma unroll
    for (int i = 0; i < 4; i++) pcell[i] = min((4 * lane + i) / wc, 7);
    // NMS cell-boundary masks of unit gl (u16 lane pairs of pixels 0-1 / 2-3): a pixel's left
    // (right) neighbour column is masked when the pixel starts (ends) a cell's region -- the
    // column is in another cell's FAST window region, which cv::FAST never scored
    const int wc_inv = (65536 + wc - 1) / wc;  // p / wc == (p * wc_inv) >> 16 for p < 256
    auto lane_masks = [&](int gl, uint32_t &ml01, uint32_t &mr01, uint32_t &ml23, uint32_t &mr23) {
        const int p0 = 4 * gl;
        const int rem = p0 - ((p0 * wc_inv) >> 16) * wc;
        const int bl = rem == 0 ? 0 : wc - rem;  // unit pixel starting a cell (>= 4: none)
        const int br = wc - rem - 1;             // unit pixel ending a cell (>= 4: none)
        auto m2 = [](int b, int i0) -> uint32_t {
            return (b == i0 ? 0u : 0xFFFFu) | (b == i0 + 1 ? 0u : 0xFFFF0000u);
        };
        ml01 = m2(bl, 0);
        ml23 = m2(bl, 2);
        mr01 = m2(br, 0);
        mr23 = m2(br, 2);
    };
    if (lane < 8) RUNS[lane] = 0;
    // quadtree path codes, loaded once: lane l holds those of its four columns and of region
    // row l (the emit loop fetches them with wave-wide shuffles, every lane active)
    uint32_t xcode[4];
#pragma unroll
    for (int i = 0; i < 4; i++) xcode[i] = 4 * lane + i < tw ? ctab[xs + 4 * lane + i] : 0u;
    const uint32_t ycode = lane < RH ? ctab[ys + lane] : 0u;

    // one pass over the strip at threshold th for the pixels in `vm` (4 bits per lane)
    auto run_pass = [&](int th, uint32_t vm) {
        VM[lane] = (uint8_t)vm;
        // score ring: every slot zero (rows -1 .. FR_G + 1 of the first group among them)
        for (int r = 0; r < FR_RS; r++)
            if (lane < FR_SS / 2) *(uint2 *)(SR + r * FR_SB + 8 * lane) = make_uint2(0, 0);
        const bool in = vm != 0;
        const v2s vth1 = (v2s){(short)(th + 1), (short)(th + 1)};
        uint4 ring[FR_PF];
        uint32_t rsh[FR_PF];
        auto issue = [&](int i, int k) {
            const uint8_t *rp = win + (int64_t)min(i, H - 1) * pitch;
            const uint32_t sh = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)rp & 3u);
            ring[k] = *(const uint4 *)(rp - sh + 4 * lane_c);
            rsh[k] = sh;
        };
        int ts = 0;  // ring slot of the next window row
        auto put = [&](int k) {
            const uint4 q = ring[k];
            const uint32_t sh = rsh[k];
            const uint32_t a0 = __builtin_amdgcn_alignbyte(q.y, q.x, sh);
            uint32_t *row = (uint32_t *)(TR + ts * FR_SB);
            if (lane < D) row[lane] = a0;
            if (ts < 6 && lane < D) row[FR_RR * FR_SS + lane] = a0;  // mirror
            if (lane == 63 && D > 64) {
                const uint32_t a1 = __builtin_amdgcn_alignbyte(q.z, q.y, sh);
                const uint32_t a2 = __builtin_amdgcn_alignbyte(q.w, q.z, sh);
                row[64] = a1;
                row[65] = a2;
                if (ts < 6) {
                    row[FR_RR * FR_SS + 64] = a1;
                    row[FR_RR * FR_SS + 65] = a2;
                }
            }
            ts = ts + 1 == FR_RR ? 0 : ts + 1;
        };
#pragma unroll
        for (int k = 0; k < FR_PF; k++) issue(k, k);
        // prologue: window rows 0 .. 5 (the first region row's upper halo and itself's - 3 ..)
#pragma unroll
        for (int i = 0; i < 6; i++) {
            put(i % FR_PF);
            issue(i + FR_PF, i % FR_PF);
        }
        int nms_next = 0;       // first region row not yet through NMS
        int ss_next = 1;        // score slot of the next region row (region row -1 -> slot 0)
        for (int y0g = 0; y0g < RH; y0g += FR_G) {
            int nlist = 0, nboth = 0;
            const int ss_g = ss_next;  // score slot of region row y0g
            // fully unrolled (the load ring's slots must be static: a dynamic index would cost
            // a register array in scratch, a rolled loop collapses the ring to one row in flight)
#pragma unroll
            for (int u = 0; u < FR_G; u++) {
                const int y = y0g + u;
                // window row y + 6 arrives (its load slot is static: (y + 6) % 4 == (u + 2) % 4);
                // past the last region row the loads are clamped re-reads and no row is tested
                const int k = (u + 2) % FR_PF;
                if (y >= RH) continue;  // wave-uniform
                put(k);
                issue(y + 6 + FR_PF, k);
                wave_sync_lds();
                if (dbg == 31) continue;
                // pretest region row y: window rows y, y + 3, y + 6 are ring slots
                // (y % RR) + 0, 3, 6 (mirrored past the ring)
                const int tb = y % FR_RR;
                const int sslot = ss_next;
                ss_next = ss_next + 1 == FR_RS ? 0 : ss_next + 1;
                uint32_t ab, ad, bb, bd;
                {
                    const uint32_t *p = (const uint32_t *)(TR + tb * FR_SB) + lane;
                    uint32_t r0[3], r3[3], r6[3];
#pragma unroll
                    for (int j = 0; j < 3; j++) {
                        r0[j] = p[j];
                        r3[j] = p[3 * FR_SS + j];
                        r6[j] = p[6 * FR_SS + j];
                    }
                    auto pretest = [&](auto I, uint32_t &pb_, uint32_t &pd_) {
                        constexpr int i = decltype(I)::value;
                        const v2s v = gather2<3 + i>(r3[0], r3[1], r3[2]);
                        const v2s c0_ = gather2<3 + i>(r6[0], r6[1], r6[2]);
                        const v2s c4 = gather2<6 + i>(r3[0], r3[1], r3[2]);
                        const v2s c8 = gather2<3 + i>(r0[0], r0[1], r0[2]);
                        const v2s c12 = gather2<0 + i>(r3[0], r3[1], r3[2]);
                        const v2s mb = pmin(pmax(c0_, c8), pmax(c4, c12));
                        const v2s md = pmax(pmin(c0_, c8), pmin(c4, c12));
                        const uint32_t wb = __builtin_bit_cast(uint32_t, (v2s)(mb - (v + vth1)));
                        const uint32_t wd = __builtin_bit_cast(uint32_t, (v2s)((v - vth1) - md));
                        pb_ = ~wb & 0x80008000u;
                        pd_ = ~wd & 0x80008000u;
                    };
                    pretest(std::integral_constant<int, 0>{}, ab, ad);
                    pretest(std::integral_constant<int, 2>{}, bb, bd);
                }
                const uint16_t e = (uint16_t)(tb << 11 | sslot << 8 | lane << 2);
                const bool bothA = in && ab && ad, bothB = in && bb && bd;
                {
                    const bool fA = in && (ab | ad) && !bothA, fB = in && (bb | bd) && !bothB;
                    const unsigned long long mA = __ballot(fA), mB = __ballot(fB);
                    const int below =
                        __builtin_amdgcn_mbcnt_hi((uint32_t)(mA >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mA, 0)) +
                        __builtin_amdgcn_mbcnt_hi((uint32_t)(mB >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mB, 0));
                    const int pa = nlist + below;
                    list[fA ? pa : FR_LCAP] = (uint16_t)(e | (ab ? 0 : 1));
                    list[fB ? pa + (int)fA : FR_LCAP] = (uint16_t)(e | (bb ? 2 : 3));
                    nlist += __popcll(mA) + __popcll(mB);
                }
                if (__ballot(bothA || bothB)) {
                    auto append = [&](bool flag, uint16_t tag) {
                        const unsigned long long m = __ballot(flag);
                        const int below = __builtin_amdgcn_mbcnt_hi(
                            (uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
                        if (flag) list[FR_LCAP - 1 - (nboth + below)] = (uint16_t)(e | tag);
                        nboth += __popcll(m);
                    };
                    append(bothA, 0);
                    append(bothB, 2);
                }
            }
            const int yend = min(y0g + FR_G, RH);  // region rows [y0g, yend) pretested
            if (dbg == 31 || dbg == 32) continue;
            wave_sync_lds();
            // ---- score: one side of one pixel pair per lane task ----
            for (int j = lane; j < nlist + 2 * nboth; j += 64) {
                const int tt = j - nlist;
                const bool top = tt >= 0;
                const int e = list[top ? FR_LCAP - 1 - (tt >> 1) : j] | (top ? (tt & 1) : 0);
                const int tb = e >> 11, sslot = (e >> 8) & 7, gg = (e >> 2) & 63, half = (e >> 1) & 1;
                const uint32_t flip = (e & 1) ? 0xFFFFFFFFu : 0u;  // dark: complemented bytes
                const uint32_t *p = (const uint32_t *)(TR + tb * FR_SB) + gg;
                Rows7 R;
#pragma unroll
                for (int r = 0; r < 7; r++) {
                    R.w[r][0] = p[r * FR_SS] ^ flip;
                    R.w[r][1] = p[r * FR_SS + 1] ^ flip;
                    R.w[r][2] = p[r * FR_SS + 2] ^ flip;
                }
                const v2s s = fast_score_side_rt(R, half ? 0x00020002u : 0u);
                const uint32_t vmg = (uint32_t)VM[gg] >> (2 * half);
                uint32_t s1 = (uint16_t)s.y >= (uint32_t)th && (vmg & 2) ? (uint16_t)s.y : 0u;
                uint32_t s0 = (uint16_t)s.x >= (uint32_t)th && (vmg & 1) ? (uint16_t)s.x : 0u;
                __hip_atomic_fetch_or((uint32_t *)(SR + sslot * FR_SB) + gg + 1,
                                      (s0 | s1 << 8) << (16 * half), __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_WAVEFRONT);
            }
            wave_sync_lds();
            if (dbg == 33) continue;
            // ---- NMS of the region rows whose neighbour rows are scored ----
            const int na = nms_next, nb = yend == RH ? RH : yend - 1;
            nms_next = nb;
            // bitmap rows 0 .. nb - na - 1 (<= FR_G + 1) cleared
            BM[lane] = 0u;
            int npass = 0;
            {
                int sl = ss_g;  // slot of region row na: ss_g - (y0g - na)
                for (int d = y0g - na; d > 0; d--) sl = sl == 0 ? FR_RS - 1 : sl - 1;
                for (int y = na; y < nb; y++) {
                    const uint32_t sw = ((const uint32_t *)(SR + sl * FR_SB))[lane + 1];
                    const bool corner = sw != 0;
                    const unsigned long long m = __ballot(corner);
                    const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
                    if (corner) list[npass + below] = (uint16_t)(sl << 9 | (y - na) << 6 | lane);
                    npass += __popcll(m);
                    sl = sl + 1 == FR_RS ? 0 : sl + 1;
                }
            }
            wave_sync_lds();
            {
                const v2s one = (v2s){1, 1};
                const v2s t1v = (v2s){(short)max(th, 1), (short)max(th, 1)};
                for (int j = lane; j < npass; j += 64) {
                    const int e = list[j];
                    const int sl = e >> 9, r = (e >> 6) & 7, gl = e & 63;
                    const int su = sl == 0 ? FR_RS - 1 : sl - 1, sd = sl == FR_RS - 1 ? 0 : sl + 1;
                    const uint32_t *mu = (const uint32_t *)(SR + su * FR_SB) + gl;
                    const uint32_t *mc = (const uint32_t *)(SR + sl * FR_SB) + gl;
                    const uint32_t *md = (const uint32_t *)(SR + sd * FR_SB) + gl;
                    const uint32_t u0 = mu[0], u1 = mu[1], u2 = mu[2];
                    const uint32_t cc0 = mc[0], cc1 = mc[1], cc2 = mc[2];
                    const uint32_t d0 = md[0], d1 = md[1], d2 = md[2];
                    uint32_t ml01, mr01, ml23, mr23;
                    lane_masks(gl, ml01, mr01, ml23, mr23);
                    auto colmax = [&](auto O) {
                        constexpr int o = decltype(O)::value;
                        return hmax3(as_h2(gather2<o>(u0, u1, u2)), as_h2(gather2<o>(cc0, cc1, cc2)),
                                     as_h2(gather2<o>(d0, d1, d2)));
                    };
                    const h2 cm34 = colmax(std::integral_constant<int, 3>{});
                    const h2 cm56 = colmax(std::integral_constant<int, 5>{});
                    const h2 cm78 = colmax(std::integral_constant<int, 7>{});
                    const h2 m45 = __builtin_elementwise_maximum(as_h2(gather2<4>(u0, u1, u2)),
                                                                 as_h2(gather2<4>(d0, d1, d2)));
                    const h2 m67 = __builtin_elementwise_maximum(as_h2(gather2<6>(u0, u1, u2)),
                                                                 as_h2(gather2<6>(d0, d1, d2)));
                    auto msk = [](h2 v, uint32_t m) {
                        return __builtin_bit_cast(h2, __builtin_bit_cast(uint32_t, v) & m);
                    };
                    const v2s n01 = as_v2s(hmax3(msk(cm34, ml01), m45, msk(cm56, mr01)));
                    const v2s n23 = as_v2s(hmax3(msk(cm56, ml23), m67, msk(cm78, mr23)));
                    const v2s s01 = gather2<4>(cc0, cc1, cc2), s23 = gather2<6>(cc0, cc1, cc2);
                    auto keep = [&](v2s sv, v2s mm) -> uint32_t {
                        const v2s k = pmin(sv - t1v, sv - mm - one);
                        const uint32_t w = __builtin_bit_cast(uint32_t, k);
                        return (~w >> 15 & 1u) | (~w >> 30 & 2u);
                    };
                    const uint32_t kb = keep(s01, n01) | keep(s23, n23) << 2;
                    if (kb)
                        __hip_atomic_fetch_or(BM + r * 8 + (gl >> 3), kb << (4 * (gl & 7)),
                                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                }
            }
            wave_sync_lds();
            if (dbg == 34) continue;
            // ---- emit: lane (cell k, row na + r), raster order within each cell ----
            {
                const int k = lane >> 3, r = lane & 7;
                const bool act = k < ncell && r < nb - na;
                const int s0 = k * wc;
                const int cw = k == ncell - 1 ? tw - s0 : wc;
                uint32_t bits = 0;
                if (act) {
                    const int dw = s0 >> 5, o = s0 & 31;
                    const uint32_t lo = BM[r * 8 + dw], hi = dw + 1 < 8 ? BM[r * 8 + dw + 1] : 0u;
                    bits = __builtin_amdgcn_alignbit(hi, lo, o) &
                           (cw >= 32 ? 0xFFFFFFFFu : ((1u << cw) - 1u));
                }
                const int n = __popc(bits);
                const int incl = wave_incl_scan_dpp(n);
                const int segb = __shfl(incl, max((lane & ~7) - 1, 0), 64);
                const int before = (lane & ~7) ? segb : 0;
                const int excl = incl - n - before;
                const int run = RUNS[k & 7];
                if (__ballot(bits != 0)) {
                    // score slot of region row na + r
                    int sl = ss_g;
                    for (int d = y0g - na; d > 0; d--) sl = sl == 0 ? FR_RS - 1 : sl - 1;
                    sl += r;
                    if (sl >= FR_RS) sl -= FR_RS;
                    const int yy = na + r;
                    const uint32_t cy = (uint32_t)__shfl((int)ycode, yy & 63, 64);
                    uint2 *out = cell_kp + ((int64_t)f * ncells + c0 + (k & 7)) * cell_cap;
                    int pos = run + excl;
                    // every lane runs every iteration (the shuffles read other lanes)
                    while (__ballot(bits != 0)) {
                        const bool has = bits != 0;
                        const int b = has ? __builtin_ctz(bits) : 0;
                        bits &= bits - 1u;
                        const int px = min(s0 + b, 255);
                        const int src = px >> 2, sel = px & 3;
                        const uint32_t x0c = (uint32_t)__shfl((int)xcode[0], src, 64);
                        const uint32_t x1c = (uint32_t)__shfl((int)xcode[1], src, 64);
                        const uint32_t x2c = (uint32_t)__shfl((int)xcode[2], src, 64);
                        const uint32_t x3c = (uint32_t)__shfl((int)xcode[3], src, 64);
                        const uint32_t cx = sel == 0 ? x0c : sel == 1 ? x1c : sel == 2 ? x2c : x3c;
                        if (has) {
                            const uint32_t sc = SR[sl * FR_SB + 4 + px];
                            if (pos < cell_cap)
                                out[pos] = make_uint2(orbg_pack(x0 + 3 - ORBG_MIN_BORDER + px,
                                                                y0 + 3 - ORBG_MIN_BORDER + yy, sc),
                                                      cx | cy);
                            pos++;
                        }
                    }
                }
                wave_sync_lds();
                if (r == 7 && k < ncell) RUNS[k] = run + (incl - before);
            }
            // score rows of the next group and the one past it cleared (their slots held rows
            // that are through NMS): region rows yend .. yend + FR_G
            wave_sync_lds();
            {
                int sl = ss_next;
                for (int d = 0; d <= FR_G; d++) {
                    if (lane < FR_SS / 2) *(uint2 *)(SR + sl * FR_SB + 8 * lane) = make_uint2(0, 0);
                    sl = sl + 1 == FR_RS ? 0 : sl + 1;
                }
            }
        }
        wave_sync_lds();
    };

    // pass 1: every pixel of the strip's region at iniThFAST
    uint32_t vm = 0;
#pragma unroll
    for (int i = 0; i < 4; i++)
        if (4 * lane + i < tw) vm |= 1u << i;
    run_pass(thi, vm);
    // pass 2: the cells left empty, at minThFAST (ORBextractor.cc:1069-1075)
    const int run_l = lane < 8 ? RUNS[lane] : 1;
    const unsigned long long empty = __ballot(lane < ncell && run_l == 0);
    if (empty && !dbg) {  // wave-uniform
        uint32_t vm2 = 0;
#pragma unroll
        for (int i = 0; i < 4; i++)
            if ((vm >> i & 1u) && (empty >> pcell[i] & 1ull)) vm2 |= 1u << i;
        run_pass(tlo, vm2);
    }
    if (lane < ncell) cell_cnt[(int64_t)f * ncells + c0 + lane] = RUNS[lane];
}

hipError_t launch_fast_rows(hipStream_t st, const OrbgGeom *g, const OrbgFastTile *tiles,
                            const uint8_t *img0, int64_t img_fs, int img_pitch,
                            const uint8_t *pyr, const uint32_t *ctab, int32_t *cell_cnt,
                            uint2 *cell_kp, int nframes, int t_begin, int t_count)
{
    const int waves = t_count * nframes;
    if (waves <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_fast_rows, dim3((waves + 3) / 4), dim3(256), 4 * FR_WAVE_BYTES, st, g,
                       tiles, img0, img_fs, img_pitch, pyr, ctab, cell_cnt, cell_kp, nframes,
                       t_begin, t_count);
    return hipGetLastError();
}

}  // namespace orbg
