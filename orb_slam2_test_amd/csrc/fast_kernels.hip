// fast_kernels.hip -- k_fast2: the FAST part of ComputeKeyPointsOctTree (ORBextractor.cc:
// 966-1094: 30-px cells, cv::FAST(window, iniThFAST, NMS), minThFAST retry of empty cells,
// kp.pt += (j * wCell, i * hCell)) for gfx950.  Every cell window of the reference's 30-px
// grid (< 66 x 66 px) fits one of the instantiated LDS pitches.
//
// The kernel is VALU-issue bound (round-2 counters: ~70% of SIMD cycles issue VALU), so this
// version cuts instructions:
//   - the LDS row pitch is a template parameter: every row offset of the 7-row circle reads
//     is an immediate of the ds_read, no address arithmetic per row;
//   - the window is staged once per 16-byte chunk with a fixed (row, chunk) per lane; both
//     pixel pairs of a 4-pixel unit are gathered from the unit's three row dwords, pair 2-3
//     by v_perm selectors shifted 2 bytes per lane (one code path for both);
//   - the compass pretest keeps the bright and dark verdicts apart, and each listed entry
//     scores ONE side of one pixel pair (a pixel is never a corner on both sides at one
//     threshold: 9 + 9 > 16 circle pixels): the dark side is the bright side of the
//     complemented bytes, so bright and dark entries share one list and one loop;
//   - the arc extremes pair the 16 starts (fast_score_side, 36 packed ops per side).
// Scores of a pixel below the cell threshold are stored as 0 (FAST's NMS treats any score
// below the threshold like an empty neighbour), and the two sides of a pair are merged with
// an LDS OR: at most one of them is non-zero per pixel.
#include <hip/hip_runtime.h>

#include "orbg_internal.h"
#include "orbg_device.h"
#include "fast_device.h"
#include "blur_device.h"

#pragma clang fp contract(off)

namespace orbg {

// LDS per wave (fc2_* offsets in OrbgGeom, host plan):
//   tA [H][2P]    window row r at byte r * 2P + x (x window-local), i.e. dword j holds
//                 window bytes 4j .. 4j+3; a unit (ry, gg) = detection pixels
//                 x = 3 + 4gg .. 6 + 4gg of row 3 + ry (bytes 3 .. 6 of dwords gg ..), and
//                 the circle of either pixel pair is within dwords gg .. gg+2 of rows
//                 ry .. ry+6 (21 dwords per scored pair side; the compass pretest reads 9
//                 per unit); the row stride 2P (24 dwords for P = 48) puts the 8 x 8 units
//                 of a pretest wave (and of the NMS scan) on 64 distinct banks
//   sc [RH+2][2P] u8 scores at sc[ry + 1][4 + 4gg + i], zero border, rows interleaved with
//                 the window rows (sc row r = bytes P .. 2P - 9 of tile row stride r; 4 RG + 8
//                 <= P - 8 bytes used)
//   list u16      pretest survivors: ry << 8 | gg << 2 | half << 1 | dark
#ifndef ORBG_FC2_IL
#define ORBG_FC2_IL 1  // score rows interleaved with the tile rows (row stride 2P; 0: apart, +0.6% per step)
#endif
#ifndef ORBG_FC2_DBG
#define ORBG_FC2_DBG 0  // 1: the phase-stop checks in a product build (round-4 register layout: 65 VGPRs, 7 waves/SIMD)
#endif
#ifndef ORBG_FC2_LATE_PC
#define ORBG_FC2_LATE_PC 1  // path codes loaded after the scoring: 64 VGPRs, 8 waves/SIMD (0: at the cell start)
#endif
#ifndef FC2_CPW
#define FC2_CPW 2  // consecutive cells per wave (shared halo lines in L1, fewer workgroups)
#endif
// small batches (B <= FC2_SMALL_B, the single-frame drop-in: an idle chip, the FAST launches on
// the critical chain) take one cell per wave: twice the waves, half the chain (1 at B = 1:
// extraction -6 us, profiles/r06ap_single_knobs.txt; at B = 1024 2 is as fast or faster)
#ifndef FC2_CPW_SMALL
#define FC2_CPW_SMALL 1
#endif
#define FC2_SMALL_B 8

// one cell, wave-uniform (scalar registers)
struct Fc2Cell {
    const uint8_t *base;  // window top-left
    int pitch, f, c, W, H, RW, RH, RG, nunits, xo, yo, NC, nch, xs, ys;
    // fused GaussianBlur (blur != nullptr): the region's level origin, its blurred plane
    uint8_t *bdst;
    int X0, Y0, bpitch, bplane;
};

#ifndef FC2_WPE
#define FC2_WPE 7  // min waves per SIMD the register allocation targets (72 VGPRs, 12 B spill; 6 -> 7 with the 7-WG LDS plan: -0.3% per step)
#endif
// FB: the fused GaussianBlur phase (opt-in, ORBG_FAST_BLUR=1) compiled in; the default
// instantiation (FB = false) keeps the 64-VGPR / 8-waves register budget
template <int P4, bool FB>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(FC2_WPE, 8))) void k_fast2(
    const OrbgGeom *__restrict__ g, const OrbgCell *__restrict__ cells,
    const uint8_t *__restrict__ img0, int64_t img_fs, int img_pitch,
    const uint8_t *__restrict__ pyr, const uint32_t *__restrict__ ctab,
    int32_t *__restrict__ cell_cnt, uint2 *__restrict__ cell_kp, uint8_t *__restrict__ blur,
    int nframes, int c_begin, int c_count, int cpw)
{
    constexpr int P = 4 * P4;
#if ORBG_FC2_IL
    constexpr int RS = 2 * P, RS4 = 2 * P4;  // tile row stride (bytes, dwords)
    constexpr int SP4 = RS4, SP = RS;         // score row stride: the tile's (interleaved)
#else
    constexpr int RS = P, RS4 = P4;           // tile row stride (bytes, dwords)
    constexpr int SP4 = P4 - 2, SP = 4 * SP4;  // score rows apart: RG + 2 dwords <= P4 - 2
#endif
    constexpr int ZR = (P - 8) / 8;           // score row bytes in use (RG + 2 dwords <= P4 - 2), as uint2
    extern __shared__ __attribute__((aligned(16))) uint32_t fc2_lds[];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint8_t *tA = (uint8_t *)fc2_lds + wv * g->fc2_wave_bytes;
    uint8_t *sc = tA + g->fc2_sc_off;
    uint16_t *list = (uint16_t *)(tA + g->fc2_list_off);
#if ORBG_FC2_BITMAP
    // units with a nonzero score, marked by the scoring; 32 units per word, raster order
    uint32_t *bmap = (uint32_t *)(tA + g->fc2_list_off + 2 * g->fc2_list_cap + 4);
#endif
    const int total = c_count * nframes;
    // cpw consecutive cells per wave (neighbours: shared halo lines in L1 / L2)
    const int cid0 =
        __builtin_amdgcn_readfirstlane((xcd_remap(blockIdx.x, gridDim.x) * 4 + wv) * cpw);
    if (cid0 >= total) return;  // wave-uniform; no workgroup barrier below

    // cell record + level geometry through the scalar cache
    auto decode = [&](int cid) {
        Fc2Cell k;
        k.f = cid / c_count;
        k.c = c_begin + cid - k.f * c_count;
        const uint4 cw4 = ((const uint4 *)cells)[k.c];
        const uint32_t cw0 = __builtin_amdgcn_readfirstlane(cw4.x);
        const uint32_t cw1 = __builtin_amdgcn_readfirstlane(cw4.y);
        const uint32_t cw2 = __builtin_amdgcn_readfirstlane(cw4.z);
        const int x0 = (int)(int16_t)(cw1 & 0xFFFF), y0 = (int)(int16_t)(cw1 >> 16);
        const int l = (int)(int16_t)(cw0 & 0xFFFF);
        k.W = (int)(int16_t)(cw2 & 0xFFFF);
        k.H = (int)(int16_t)(cw2 >> 16);
        if (l == 0) {
            k.base = img0 + k.f * img_fs;
            k.pitch = img_pitch;
        } else {
            k.base = pyr + k.f * g->pyr_frame + g->lv[l].pyr_off;
            k.pitch = g->lv[l].pitch;
        }
        k.base += (int64_t)y0 * k.pitch + x0;
        k.RW = k.W - 6;
        k.RH = k.H - 6;
        k.RG = k.RW > 0 ? (k.RW + 3) >> 2 : 0;
        k.nunits = k.RH > 0 ? k.RH * k.RG : 0;
        k.xo = x0 - ORBG_MIN_BORDER + 3;
        k.yo = y0 - ORBG_MIN_BORDER + 3;
        k.xs = g->lv[l].xs_off + k.xo;
        k.ys = g->lv[l].ys_off + k.yo;
        k.NC = (k.RG + 2 + 3) >> 2;  // tile dwords 0 .. RG+1
        k.X0 = x0 + 3;
        k.Y0 = y0 + 3;
        if (FB) {
            // the fused blur's last output dword starts below X0 + RW; its 7-tap sources reach
            // 3 bytes past it: window bytes up to 4 ceil((X0 + RW) / 4) + 2 - x0 (the plan
            // checked the pitch holds them)
            const int nb = 4 * ((k.X0 + k.RW + 3) >> 2) + 3 - x0;
            k.NC = max(k.NC, (nb + 15) >> 4);
            k.bdst = blur + k.f * g->blur_frame + g->lv[l].blur_off;
            k.bpitch = g->lv[l].pitch;
            k.bplane = g->lv[l].h * k.bpitch;
        }
        k.nch = k.H * k.NC;
        return k;
    };
    // Window chunk i = (row r, chunk cc): tile dwords 4cc .. 4cc+3 = window bytes 16cc ..
    // 16cc+15, from 6 aligned dwords + v_alignbyte.  The window sits >= 13 px inside the level
    // and every row has >= 16 rows below it, so the aligned over-read stays in the image.
    auto chunk_src = [&](const Fc2Cell &k, int i, uint32_t &sh) {
        const int mdiv = (65536 + k.NC - 1) / k.NC;  // i / NC == (i * mdiv) >> 16, i < 1024
        const int r = (i * mdiv) >> 16, cc = i - r * k.NC;
        // pointer arithmetic (no integer round trip): global_, not flat_, loads
        const uint8_t *src = k.base + (int64_t)r * k.pitch + 16 * cc;
        sh = (uint32_t)((uintptr_t)src & 3u);
        return (const uint32_t *)(src - sh);
    };
    auto put = [&](const Fc2Cell &k, int i, uint4 q, uint32_t q4, uint32_t sh) {
        const int mdiv = (65536 + k.NC - 1) / k.NC;
        const int r = (i * mdiv) >> 16, cc = i - r * k.NC;
        const int to = r * RS + 16 * cc;
        const uint32_t d[5] = {q.x, q.y, q.z, q.w, q4};
        uint32_t A[4];
#pragma unroll
        for (int j = 0; j < 4; j++) A[j] = __builtin_amdgcn_alignbyte(d[j + 1], d[j], sh);
        if constexpr (P % 16 == 0) {
            *(uint4 *)(tA + to) = make_uint4(A[0], A[1], A[2], A[3]);
        } else {  // rows 8-byte aligned
            *(uint2 *)(tA + to) = make_uint2(A[0], A[1]);
            *(uint2 *)(tA + to + 8) = make_uint2(A[2], A[3]);
        }
    };

    // launch constants read once (scalar loads after the LDS fences would wait on the LDS
    // queue too: both count in lgkmcnt)
#if defined(ORBG_DEV_KNOBS) || ORBG_FC2_DBG
    const int dbg = g->dbg;  // developer phase stops (tools/fast_phase.sh)
#else
    constexpr int dbg = 0;   // product build: no phase-stop checks (their masks cost registers)
#endif
    const int thi = g->ini_th, tlo = g->min_th;
    const int lcap = g->fc2_list_cap;  // pretest list entries (2 per unit of the largest cell)
    const int ncells = g->ncells, cell_cap = g->cell_cap;
#pragma unroll 1
    for (int kc = 0; kc < cpw; kc++) {
    const int cid = cid0 + kc;
    if (cid >= total) break;  // wave-uniform
    const Fc2Cell cur = decode(cid);
    const int f = cur.f, c = cur.c, RW = cur.RW, RH = cur.RH, RG = cur.RG, nunits = cur.nunits;
    const int xo = cur.xo, yo = cur.yo;
#if !ORBG_FC2_LATE_PC
    uint32_t xs_l = lane < RW ? ctab[cur.xs + lane] : 0u;
    uint32_t ys_l = lane < RH ? ctab[cur.ys + lane] : 0u;
#endif
    // ---- window -> tA: all of a lane's chunk loads in flight before the first store
    // (the previous cell's reads of the tiles are done: a wave's LDS ops complete in order) ----
    wave_sync_lds();
    {
        for (int i0 = 0; i0 < cur.nch; i0 += 2 * 64) {
            uint4 q[2];
            uint32_t q4[2];
            uint32_t sh[2];
#pragma unroll
            for (int u = 0; u < 2; u++) {
                // lanes past the last chunk redo it (the same bytes to the same place): the
                // stores below need no exec-mask branch
                const int i = min(i0 + 64 * u + lane, cur.nch - 1);
                const uint32_t *aw = chunk_src(cur, i, sh[u]);
                q[u] = *(const uint4 *)aw;  // unconditional: both in flight
                q4[u] = aw[4];
            }
#pragma unroll
            for (int u = 0; u < 2; u++) put(cur, min(i0 + 64 * u + lane, cur.nch - 1), q[u], q4[u], sh[u]);
        }
        const int nz = (RH + 2) * ZR;
        for (int i = lane; i < nz; i += 64) {
            const int r = i / ZR;
            *(uint2 *)(sc + r * SP + 8 * (i - r * ZR)) = make_uint2(0, 0);
        }
#if ORBG_FC2_BITMAP
        for (int i = lane; i < (nunits + 31) >> 5; i += 64) bmap[i] = 0u;
#endif
    }
    wave_sync_lds();
    if (dbg == 11) continue;


    // unit u = ry * RG + gg walked as u = lane + 64 k: (ry, gg) advance by (64 / RG, 64 % RG)
    const int rstep = RG > 0 ? 64 / RG : 0, gstep = RG > 0 ? 64 - rstep * RG : 0;
    const int ry0 = RG > 0 ? lane / RG : 0, gg0 = lane - ry0 * RG;

    // ---- compass pretest at iniThFAST (necessary for a 9-arc: some adjacent compass pair
    // (0,4), (4,8), (8,12), (12,0) is on the arc's side), bright and dark apart:
    //   bright: min(max(c0, c8), max(c4, c12)) > v + th,  dark: max(min(c0, c8), min(c4, c12)) < v - th
    // Survivors (pair, side) are ballot-compacted into one list; order is irrelevant (the
    // scores go to their place in sc) ----
    int nlist = 0, nboth = 0;
    {
        const v2s vth1 = (v2s){(short)(thi + 1), (short)(thi + 1)};
        // tile offset of unit (ry, gg) kept incrementally (no per-iteration multiply)
        int toff = ry0 * RS + 4 * gg0;
        const int tstep = rstep * RS + 4 * gstep, twrap = RS - 4 * RG;
        for (int u0 = 0, ry = ry0, gg = gg0; u0 < nunits; u0 += 64) {
            const int u = u0 + lane;
            // per pair: bright / dark survivors as the sign bits (15, 31) of a packed word,
            // 0 = none.  Every lane runs the test (lanes past the last unit read unit 0's
            // words; their entries are dropped below): no exec-mask branch per 64 units.
            // Pixels of the last unit column past the region are tested like the others (the
            // window tile holds bytes there): the scoring loop zeroes their scores
            uint32_t ab = 0, ad = 0, bb = 0, bd = 0;
            const bool in = u < nunits;
            {
                const uint32_t *p = (const uint32_t *)(tA + (in ? toff : 0));
                uint32_t r0[3], r3[3], r6[3];
#pragma unroll
                for (int k = 0; k < 3; k++) {
                    r0[k] = p[k];
                    r3[k] = p[3 * RS4 + k];
                    r6[k] = p[6 * RS4 + k];
                }
                auto pretest = [&](auto I, uint32_t &pb_, uint32_t &pd_) {
                    constexpr int i = decltype(I)::value;
                    const v2s v = gather2<3 + i>(r3[0], r3[1], r3[2]);
                    const v2s c0 = gather2<3 + i>(r6[0], r6[1], r6[2]);
                    const v2s c4 = gather2<6 + i>(r3[0], r3[1], r3[2]);
                    const v2s c8 = gather2<3 + i>(r0[0], r0[1], r0[2]);
                    const v2s c12 = gather2<0 + i>(r3[0], r3[1], r3[2]);
                    const v2s mb = pmin(pmax(c0, c8), pmax(c4, c12));
                    const v2s md = pmax(pmin(c0, c8), pmin(c4, c12));
                    // lane >= 0 <=> pass: mb - (v + th + 1) and (v - th - 1) - md
                    const uint32_t wb = __builtin_bit_cast(uint32_t, (v2s)(mb - (v + vth1)));
                    const uint32_t wd = __builtin_bit_cast(uint32_t, (v2s)((v - vth1) - md));
                    pb_ = ~wb & 0x80008000u;
                    pd_ = ~wd & 0x80008000u;
                };
                pretest(std::integral_constant<int, 0>{}, ab, ad);
                pretest(std::integral_constant<int, 2>{}, bb, bd);
            }
            const uint16_t e = (uint16_t)(ry << 8 | gg << 2);
            // one entry per pair with a survivor, from the bottom of the list (side: bright
            // unless only dark passed); pairs passing both sides (rare) from the top, expanded
            // into two lane tasks by the scoring loop -- 2 entries per unit at most
            auto append = [&](bool flag, bool top, uint16_t tag) {
                const unsigned long long m = __ballot(flag);
                const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
                if (flag) list[top ? lcap - 1 - (nboth + below) : nlist + below] = (uint16_t)(e | tag);
                (top ? nboth : nlist) += __popcll(m);
            };
            const bool bothA = in && ab && ad, bothB = in && bb && bd;
            // the common entries of pixels 0-1 and 2-3 in one append: a lane's entries follow
            // those of every lower lane, its pair-0-1 entry before its pair-2-3 entry; a lane
            // without an entry writes the spare slot past the list (lcap), so both stores are
            // unconditional (no exec-mask branches)
            {
                const bool fA = in && (ab | ad) && !bothA, fB = in && (bb | bd) && !bothB;
                const unsigned long long mA = __ballot(fA), mB = __ballot(fB);
                const int below =
                    __builtin_amdgcn_mbcnt_hi((uint32_t)(mA >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mA, 0)) +
                    __builtin_amdgcn_mbcnt_hi((uint32_t)(mB >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mB, 0));
                const int pa = nlist + below;
                list[fA ? pa : lcap] = (uint16_t)(e | (ab ? 0 : 1));
                list[fB ? pa + (int)fA : lcap] = (uint16_t)(e | (bb ? 2 : 3));
                nlist += __popcll(mA) + __popcll(mB);
            }
            if (__ballot(bothA || bothB)) {
                append(bothA, true, 0);
                append(bothB, true, 2);
            }
            ry += rstep;
            gg += gstep;
            toff += tstep;
            if (gg >= RG) {
                gg -= RG;
                ry++;
                toff += twrap;
            }
        }
    }
    wave_sync_lds();
    if (dbg == 14) continue;

    // ---- one side of one pixel pair per lane task: tasks [0, nlist) are the bottom entries,
    // then two per top entry (bright, dark) ----
    for (int j = lane; j < nlist + 2 * nboth; j += 64) {
        // branch-free (selects, one LDS read): no exec-mask juggling per task
        const int t = j - nlist;
        const bool top = t >= 0;
        const int e = list[top ? lcap - 1 - (t >> 1) : j] | (top ? (t & 1) : 0);
        const int ry = e >> 8, gg = (e >> 2) & 63, half = (e >> 1) & 1;
        const uint32_t flip = (e & 1) ? 0xFFFFFFFFu : 0u;  // dark: complemented bytes
        const uint32_t *p = (const uint32_t *)(tA + ry * RS + 4 * gg);
        Rows7 R;
#pragma unroll
        for (int r = 0; r < 7; r++) {
            R.w[r][0] = p[r * RS4] ^ flip;
            R.w[r][1] = p[r * RS4 + 1] ^ flip;
            R.w[r][2] = p[r * RS4 + 2] ^ flip;
        }
        const v2s s = fast_score_side_rt(R, half ? 0x00020002u : 0u);
        uint32_t s1 = (uint16_t)s.y >= (uint32_t)thi ? (uint16_t)s.y : 0u;
        uint32_t s0 = (uint16_t)s.x >= (uint32_t)thi ? (uint16_t)s.x : 0u;
        const int valid = RW - 4 * gg - 2 * half;  // pixels of the pair inside the region
        if (valid < 2) s1 = 0;
        if (valid < 1) s0 = 0;
        __hip_atomic_fetch_or((uint32_t *)(sc + (ry + 1) * SP + 4 * gg + 4),
                              (s0 | s1 << 8) << (16 * half), __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_WAVEFRONT);
#if ORBG_FC2_BITMAP
        {
            const int u = ry * RG + gg;  // unconditional: an empty task ORs 0
            __hip_atomic_fetch_or(bmap + (u >> 5), (s0 | s1) ? 1u << (u & 31) : 0u,
                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        }
#endif
    }
    wave_sync_lds();
    if (dbg == 12) continue;

    // ---- NMS (cell-local) + raster-order compaction ----
    // cv::FAST keeps p iff s_p > every neighbour's score, a neighbour that is not a corner
    // at the cell threshold th counting as 0; with s_p >= max(th, 1) that is exactly
    //   max(raw 8-neighbour scores) < max(th, s_p).
    const v2s one = (v2s){1, 1};
    auto keep_bits = [&](int ry, int gg, int th, bool may_be_empty) -> uint32_t {
        const v2s t1v = (v2s){(short)max(th, 1), (short)max(th, 1)};
        const v2s thv = (v2s){(short)th, (short)th};
        const uint32_t *m = (const uint32_t *)(sc + ry * SP + 4 * gg);
        const uint32_t c1 = m[SP4 + 1];
        if (may_be_empty && c1 == 0) return 0u;  // a unit with no scored pixel keeps nothing
        const uint32_t u0 = m[0], u1 = m[1], u2 = m[2];
        const uint32_t c0 = m[SP4], c2 = m[SP4 + 2];
        const uint32_t d0 = m[2 * SP4], d1 = m[2 * SP4 + 1], d2 = m[2 * SP4 + 2];
        v2s mA = pmax(pmax(gather2<3>(u0, u1, u2), gather2<4>(u0, u1, u2)), gather2<5>(u0, u1, u2));
        mA = pmax(mA, pmax(pmax(gather2<3>(d0, d1, d2), gather2<4>(d0, d1, d2)),
                           gather2<5>(d0, d1, d2)));
        mA = pmax(mA, pmax(gather2<3>(c0, c1, c2), gather2<5>(c0, c1, c2)));
        v2s mB = pmax(pmax(gather2<5>(u0, u1, u2), gather2<6>(u0, u1, u2)), gather2<7>(u0, u1, u2));
        mB = pmax(mB, pmax(pmax(gather2<5>(d0, d1, d2), gather2<6>(d0, d1, d2)),
                           gather2<7>(d0, d1, d2)));
        mB = pmax(mB, pmax(gather2<5>(c0, c1, c2), gather2<7>(c0, c1, c2)));
        const v2s sA = gather2<4>(c0, c1, c2), sB = gather2<6>(c0, c1, c2);
        auto keep = [&](v2s sv, v2s mm) -> uint32_t {
            const v2s k = pmin(sv - t1v, pmax(thv, sv) - mm - one);
            const uint32_t w = __builtin_bit_cast(uint32_t, k);
            return (~w >> 15 & 1u) | (~w >> 30 & 2u);
        };
        uint32_t kb = keep(sA, mA) | keep(sB, mB) << 2;
        const int valid = min(RW - 4 * gg, 4);
        if (valid < 4) kb &= (1u << valid) - 1u;
        return kb;
    };
    // quadtree path codes of the cell's columns / rows (one per lane): loaded after the
    // scoring (not live through its register peak), in flight during the corner-unit pass
#if ORBG_FC2_LATE_PC
    uint32_t xs_l = lane < RW ? ctab[cur.xs + lane] : 0u;
    uint32_t ys_l = lane < RH ? ctab[cur.ys + lane] : 0u;
#endif
    const int64_t slot = (int64_t)f * ncells + c;
    uint2 *out = cell_kp + slot * cell_cap;
    const __amdgpu_buffer_rsrc_t orsrc =
        __builtin_amdgcn_make_buffer_rsrc((void *)out, (short)0, cell_cap * 8, 0x00020000);
    int run = 0;
    auto emit = [&](uint32_t kb, int ry, int gg) {
        const int n = __popc(kb);
        int tot;
        const int incl = wave_incl_scan_small(n, &tot);
        if (tot == 0) return;  // wave-uniform
        const uint32_t cy = (uint32_t)__shfl((int)ys_l, ry & 63, 64);
        uint32_t cx[4];
#pragma unroll
        for (int i = 0; i < 4; i++) cx[i] = (uint32_t)__shfl((int)xs_l, (4 * gg + i) & 63, 64);
        // four unconditional buffer stores: a pixel that is not kept gets an offset past the
        // cell's range, which the hardware drops (no exec-mask branch per pixel)
        const int off = run + incl - n;
        const uint32_t c1 = *(const uint32_t *)(sc + (ry + 1) * SP + 4 * gg + 4);
        const int xx = xo + 4 * gg, y = yo + ry;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int pos = off + __popc(kb & ((1u << i) - 1u));
            typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
            const u32x2 rec = {orbg_pack(xx + i, y, (c1 >> (8 * i)) & 0xFF), cx[i] | cy};
            __builtin_amdgcn_raw_buffer_store_b64(rec, orsrc, (kb >> i & 1u) ? pos * 8 : (1 << 30),
                                                  0, 0);
        }
        run += tot;
    };
    // units with a corner (nonzero score word), raster order, over the dead pretest list
    uint16_t *plist = list;
    int npass = 0;
#if ORBG_FC2_BITMAP
    {
        // the scoring's bitmap, four units per lane: a 3-bit scan, no pass over every unit
        const int mdiv = (65536 + RG - 1) / max(RG, 1);  // u / RG == (u * mdiv) >> 16, u < 1024
        for (int b0 = 0; b0 < nunits; b0 += 256) {
            const int u4 = b0 + 4 * lane;
            const uint32_t w = u4 < nunits ? bmap[u4 >> 5] : 0u;
            const uint32_t nib = (w >> (u4 & 31)) & 15u;
            const int n = __popc(nib);
            int tot;
            const int incl = wave_incl_scan_small(n, &tot);
            int pos = npass + incl - n;
#pragma unroll
            for (int k = 0; k < 4; k++)
                if ((nib >> k) & 1u) {
                    const int u = u4 + k, ry = (u * mdiv) >> 16, gg = u - ry * RG;
                    plist[pos++] = (uint16_t)(ry << 8 | gg);
                }
            npass += tot;
        }
    }
#else
    for (int u0 = 0, ry = ry0, gg = gg0; u0 < nunits; u0 += 64) {
        const bool in = u0 + lane < nunits;  // the read is unconditional (no exec branch)
        const uint32_t sw = *(const uint32_t *)(sc + (in ? (ry + 1) * SP + 4 * gg + 4 : 0));
        const bool corner = in && sw != 0;
        const unsigned long long m = __ballot(corner);
        const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
        if (corner) plist[npass + below] = (uint16_t)(ry << 8 | gg);
        npass += __popcll(m);
        ry += rstep;
        gg += gstep;
        if (gg >= RG) {
            gg -= RG;
            ry++;
        }
    }
#endif
    wave_sync_lds();
    for (int j0 = 0; j0 < npass; j0 += 64) {
        const int j = j0 + lane;
        // branch-free: lanes past the list redo the last entry and keep nothing (every
        // listed unit has a scored pixel, so no empty-unit exit either)
        const int e = plist[min(j, npass - 1)];
        const int ry = e >> 8, gg = e & 0xFF;
        const uint32_t kb0 = keep_bits(ry, gg, thi, false);
        const uint32_t kb = j < npass ? kb0 : 0u;
        emit(kb, ry, gg);
    }
    if (dbg == 13) continue;
    if (run == 0) {
        // an empty cell retries at minThFAST (ORBextractor.cc:1069-1075): every unit scored
        // on both sides (the window tiles are intact), then NMS at minThFAST
        wave_sync_lds();
        for (int u = lane, ry = ry0, gg = gg0; u < nunits; u += 64) {
            // the four (pixel pair, side) scores of the unit one at a time, each from the
            // tile re-read (the dark side = the bright side of the complemented bytes): max
            // over sides of max(M_side - 1, 0) = cornerScore's max(M - 1, 0).  A rare path:
            // re-reading keeps its register use below the main loops'.
            v2s sp0 = (v2s){0, 0}, sp1 = (v2s){0, 0};
#pragma unroll 1
            for (int t = 0; t < 4; t++) {
                const uint32_t flip = (t & 1) ? 0xFFFFFFFFu : 0u;
                const uint32_t *p = (const uint32_t *)(tA + ry * RS + 4 * gg);
                Rows7 R;
#pragma unroll
                for (int r = 0; r < 7; r++) {
                    R.w[r][0] = p[r * RS4] ^ flip;
                    R.w[r][1] = p[r * RS4 + 1] ^ flip;
                    R.w[r][2] = p[r * RS4 + 2] ^ flip;
                }
                const v2s sc2 = fast_score_side_rt(R, (t & 2) ? 0x00020002u : 0u);
                if (t & 2)
                    sp1 = pmax(sp1, sc2);
                else
                    sp0 = pmax(sp0, sc2);
            }
            uint32_t word = (uint32_t)(uint16_t)sp0.x | ((uint32_t)(uint16_t)sp0.y << 8) |
                            ((uint32_t)(uint16_t)sp1.x << 16) | ((uint32_t)(uint16_t)sp1.y << 24);
            const int valid = min(RW - 4 * gg, 4);
            if (valid < 4) word &= (1u << (8 * valid)) - 1u;
            *(uint32_t *)(sc + (ry + 1) * SP + 4 * gg + 4) = word;
            ry += rstep;
            gg += gstep;
            if (gg >= RG) {
                gg -= RG;
                ry++;
            }
        }
        // the path codes again (re-read, not kept live through the scoring above)
        xs_l = lane < RW ? ctab[cur.xs + lane] : 0u;
        ys_l = lane < RH ? ctab[cur.ys + lane] : 0u;
        wave_sync_lds();
        for (int u0 = 0, ry = ry0, gg = gg0; u0 < nunits; u0 += 64) {
            const uint32_t kb = u0 + lane < nunits ? keep_bits(ry, gg, tlo, true) : 0u;
            emit(kb, ry, gg);
            ry += rstep;
            gg += gstep;
            if (gg >= RG) {
                gg -= RG;
                ry++;
            }
        }
    }
    // ---- fused GaussianBlur 7x7 (ORBextractor.cc:1375-1377; k_blur2's arithmetic,
    // blur2_column) of the cell's detection region from the window tile (intact: the
    // phases above write only the score rows and the lists): output dwords
    // (level x = 4q, q in [ceil(X0 / 4), ceil((X0 + RW) / 4))) x 4-row segments, a task per
    // lane; the region rows' 7-row sources are window rows, the columns' 7-tap sources window
    // bytes (the tile holds them, decode()).  Cells tile the level's rectangle [16, bx1) x
    // [16, by1) with disjoint dwords; k_blur_border does the rest ----
    if constexpr (FB) {
        const Blur2Weights bw(g);
        const int qa = (cur.X0 + 3) >> 2, nq = ((cur.X0 + RW + 3) >> 2) - qa;
        const int ntask = nq * ((RH + 3) >> 2);
        const int ob0 = 4 * qa - cur.X0 - 1;  // tile byte of column 4 qa - 4: -1 .. 2
        const uint32_t bsh = (uint32_t)(ob0 & 3);
        const int qdiv = (65536 + nq - 1) / max(nq, 1);  // t / nq == (t * qdiv) >> 16, t < 1024
        const __amdgpu_buffer_rsrc_t brs =
            __builtin_amdgcn_make_buffer_rsrc((void *)cur.bdst, (short)0, cur.bplane, 0x00020000);
        auto seg = [&](auto NORM) {
            for (int t = lane; t < ntask; t += 64) {
                const int sg = (t * qdiv) >> 16, q = t - sg * nq;
                const int ob = ob0 + 4 * q, di = (ob - (int)bsh) >> 2;  // di >= -1
                const uint32_t *rowp = (const uint32_t *)tA + 4 * sg * RS4 + max(di, 0);
                const int soff = (cur.Y0 + 4 * sg) * cur.bpitch + 4 * (qa + q);
                blur2_column<4, decltype(NORM)::value>(
                    bw,
                    [&](int i, uint32_t &w0, uint32_t &w1, uint32_t &w2) {
                        // one row's loads at a time (hoisting all ten rows' LDS reads took
                        // the kernel past 64 VGPRs, i.e. below 8 waves per SIMD)
                        __builtin_amdgcn_sched_barrier(0);
                        const uint32_t *pr = rowp + i * RS4;
                        // di = -1: dword -1 feeds only byte 0 of w0 (column gx - 4, weight 0)
                        const uint32_t d0 = di >= 0 ? pr[0] : 0u;
                        const uint32_t *pq = pr + (di >= 0 ? 1 : 0);
                        const uint32_t d1 = pq[0], d2 = pq[1], d3 = pq[2];
                        w0 = __builtin_amdgcn_alignbyte(d1, d0, bsh);
                        w1 = __builtin_amdgcn_alignbyte(d2, d1, bsh);
                        w2 = __builtin_amdgcn_alignbyte(d3, d2, bsh);
                    },
                    [&](int o, uint32_t word) {
                        __builtin_amdgcn_raw_buffer_store_b32(
                            word, brs, 4 * sg + o < RH ? soff + o * cur.bpitch : (1 << 30), 0, 0);
                    });
            }
        };
        if (bw.norm256)
            seg(std::true_type{});
        else
            seg(std::false_type{});
    }
    if (lane == 0) cell_cnt[slot] = run;
    }  // cells of this wave
}

// instantiated LDS pitches (dwords); the host plan picks one
#define ORBG_FAST2_PITCHES(X) X(12) X(14) X(16) X(18) X(20) X(22) X(24) X(26) X(28) X(32)

bool fast2_pitch_ok(int p4)
{
    switch (p4) {
#define X(n) case n:
        ORBG_FAST2_PITCHES(X)
#undef X
        return true;
    default:
        return false;
    }
}

template <int P4, bool FB>
static hipError_t launch_fast2_t(size_t lds, dim3 grid, hipStream_t st, const OrbgGeom *g,
                                 const OrbgCell *cells, const uint8_t *img0, int64_t img_fs,
                                 int img_pitch, const uint8_t *pyr, const uint32_t *ctab,
                                 int32_t *cell_cnt, uint2 *cell_kp, uint8_t *blur, int nframes,
                                 int c_begin, int c_count, int cpw)
{
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute((const void *)k_fast2<P4, FB>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL((k_fast2<P4, FB>), grid, dim3(256), lds, st, g, cells, img0, img_fs,
                       img_pitch, pyr, ctab, cell_cnt, cell_kp, blur, nframes, c_begin, c_count, cpw);
    return hipGetLastError();
}

hipError_t launch_fast2(int p4, size_t lds, hipStream_t st, const OrbgGeom *g,
                        const OrbgCell *cells, const uint8_t *img0, int64_t img_fs,
                        int img_pitch, const uint8_t *pyr, const uint32_t *ctab,
                        int32_t *cell_cnt, uint2 *cell_kp, uint8_t *blur, int nframes,
                        int c_begin, int c_count)
{
    const int cpw = nframes <= FC2_SMALL_B ? FC2_CPW_SMALL : FC2_CPW;
    const dim3 grid((c_count * nframes + 4 * cpw - 1) / (4 * cpw));
    switch (p4) {
#define X(n)                                                                                  \
    case n:                                                                                   \
        if (blur) return launch_fast2_t<n, true>(lds, grid, st, g, cells, img0, img_fs,       \
                                                 img_pitch, pyr, ctab, cell_cnt, cell_kp,     \
                                                 blur, nframes, c_begin, c_count, cpw);       \
        return launch_fast2_t<n, false>(lds, grid, st, g, cells, img0, img_fs, img_pitch, pyr, \
                                        ctab, cell_cnt, cell_kp, nullptr, nframes, c_begin,   \
                                        c_count, cpw);
        ORBG_FAST2_PITCHES(X)
#undef X
    default:
        return hipErrorInvalidValue;
    }
}

}  // namespace orbg
