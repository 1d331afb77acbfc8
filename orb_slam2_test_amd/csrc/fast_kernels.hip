// fast_kernels.hip -- k_fast2: the FAST part of ComputeKeyPointsOctTree (ORBextractor.cc:
// 966-1094: 30-px cells, cv::FAST(window, iniThFAST, NMS), minThFAST retry of empty cells,
// kp.pt += (j * wCell, i * hCell)) for gfx950.  Same outputs, bit for bit, as k_fast_cells
// (extract_kernels.hip), which stays as the fallback for LDS pitches not instantiated here.
//
// The kernel is VALU-issue bound (round-2 counters: ~70% of SIMD cycles issue VALU), so this
// version cuts instructions:
//   - the LDS row pitch is a template parameter: every row offset of the 7-row circle reads
//     is an immediate of the ds_read, no address arithmetic per row;
//   - the window is staged once per 16-byte chunk with a fixed (row, chunk) per lane, plus a
//     copy shifted by 2 bytes, so pixel pairs 2-3 of a 4-pixel unit are read exactly like
//     pairs 0-1 (one code path for both);
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

#pragma clang fp contract(off)

namespace orbg {

// LDS per wave (fc2_* offsets in OrbgGeom, host plan):
//   tA [H][P]     window row r at byte r * P + 1 + x (x window-local), i.e. dword j holds
//                 window bytes 4j-1 .. 4j+2; a unit (ry, gg) = detection pixels
//                 x = 3 + 4gg .. 6 + 4gg of row 3 + ry, and its circle is dwords gg .. gg+2
//                 of rows ry .. ry+6
//   tB [H][P]     tA shifted by 2 bytes (tB byte k = tA byte k + 2): pixels 2-3 of a unit
//                 sit where pixels 0-1 sit in tA
//   sc [RH+2][P]  u8 scores at sc[ry + 1][4 + 4gg + i], zero border
//   list u16      pretest survivors: ry << 8 | gg << 2 | half << 1 | dark
template <int P4>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8))) void k_fast2(
    const OrbgGeom *__restrict__ g, const OrbgCell *__restrict__ cells,
    const uint8_t *__restrict__ img0, int64_t img_fs, int img_pitch,
    const uint8_t *__restrict__ pyr, const uint32_t *__restrict__ ctab,
    int32_t *__restrict__ cell_cnt, uint2 *__restrict__ cell_kp, int nframes, int c_begin,
    int c_count)
{
    constexpr int P = 4 * P4;
    extern __shared__ __attribute__((aligned(16))) uint32_t fc2_lds[];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint8_t *tA = (uint8_t *)fc2_lds + wv * g->fc2_wave_bytes;
    uint8_t *tB = tA + g->fc2_tileb_off;
    uint8_t *sc = tA + g->fc2_sc_off;
    uint16_t *list = (uint16_t *)(tA + g->fc2_list_off);
    // wave-uniform cell record through the scalar cache (as k_fast_cells)
    const int cid = __builtin_amdgcn_readfirstlane(xcd_remap(blockIdx.x, gridDim.x) * 4 + wv);
    if (cid >= c_count * nframes) return;  // wave-uniform; no workgroup barrier below
    const int f = cid / c_count, c = c_begin + cid - f * c_count;
    const uint4 cw4 = ((const uint4 *)cells)[c];
    const uint32_t cw0 = __builtin_amdgcn_readfirstlane(cw4.x);
    const uint32_t cw1 = __builtin_amdgcn_readfirstlane(cw4.y);
    const uint32_t cw2 = __builtin_amdgcn_readfirstlane(cw4.z);
    const int x0 = (int)(int16_t)(cw1 & 0xFFFF), y0 = (int)(int16_t)(cw1 >> 16);
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
    base += (int64_t)y0 * pitch + x0;
    const int RW = W - 6, RH = H - 6;
    const int RG = RW > 0 ? (RW + 3) >> 2 : 0;
    const int nunits = RH > 0 ? RH * RG : 0;
    // quadtree path codes of this cell's columns / rows (one per lane), issued early
    const int xo = x0 - ORBG_MIN_BORDER + 3, yo = y0 - ORBG_MIN_BORDER + 3;
    const uint32_t xs_l = lane < RW ? ctab[g->lv[l].xs_off + xo + lane] : 0u;
    const uint32_t ys_l = lane < RH ? ctab[g->lv[l].ys_off + yo + lane] : 0u;

    // ---- window -> tA / tB: lane = (row, 16-byte chunk); chunk cc is tile dwords 4cc ..
    // 4cc+3, window bytes 16cc-1 .. 16cc+14, loaded as 6 aligned dwords + v_alignbyte (the
    // window sits >= 13 px inside the level, every row has >= 16 rows below it, so the
    // aligned over-read stays inside the image) ----
    {
        const int NC = (RG + 3 + 3) >> 2;     // tile dwords 0 .. RG+2 (tB needs tA dword RG+2)
        const int nch = H * NC;
        const int mdiv = (65536 + NC - 1) / NC;  // i / NC == (i * mdiv) >> 16 for i < 1024
        for (int i0 = 0; i0 < nch; i0 += 128) {
            uint4 q[2];
            uint2 q2[2];
            uint32_t sh[2];
            int to[2];
#pragma unroll
            for (int k = 0; k < 2; k++) {
                const int i = i0 + 64 * k + lane;
                const bool ok = i < nch;
                const int ii = ok ? i : 0;  // unconditional loads: all four in flight
                const int r = (ii * mdiv) >> 16, cc = ii - r * NC;
                const uintptr_t a = (uintptr_t)(base + (int64_t)r * pitch + 16 * cc - 1);
                sh[k] = (uint32_t)(a & 3u);
                const uint32_t *aw = (const uint32_t *)(a - sh[k]);
                q[k] = *(const uint4 *)aw;
                q2[k] = *(const uint2 *)(aw + 4);
                to[k] = ok ? r * P + 16 * cc : -1;
            }
#pragma unroll
            for (int k = 0; k < 2; k++) {
                if (to[k] < 0) continue;
                const uint32_t d[6] = {q[k].x, q[k].y, q[k].z, q[k].w, q2[k].x, q2[k].y};
                uint32_t A[5], Bw[4];
#pragma unroll
                for (int j = 0; j < 5; j++) A[j] = __builtin_amdgcn_alignbyte(d[j + 1], d[j], sh[k]);
#pragma unroll
                for (int j = 0; j < 4; j++) Bw[j] = __builtin_amdgcn_alignbyte(A[j + 1], A[j], 2);
                *(uint2 *)(tA + to[k]) = make_uint2(A[0], A[1]);
                *(uint2 *)(tA + to[k] + 8) = make_uint2(A[2], A[3]);
                *(uint2 *)(tB + to[k]) = make_uint2(Bw[0], Bw[1]);
                *(uint2 *)(tB + to[k] + 8) = make_uint2(Bw[2], Bw[3]);
            }
        }
        uint2 *z = (uint2 *)sc;
        const int nz = (RH + 2) * (P / 8);
        for (int i = lane; i < nz; i += 64) z[i] = make_uint2(0, 0);
    }
    wave_sync_lds();
    if (g->dbg == 11) return;

    // unit u = ry * RG + gg walked as u = lane + 64 k: (ry, gg) advance by (64 / RG, 64 % RG)
    const int rstep = RG > 0 ? 64 / RG : 0, gstep = RG > 0 ? 64 - rstep * RG : 0;
    const int ry0 = RG > 0 ? lane / RG : 0, gg0 = lane - ry0 * RG;
    const int thi = g->ini_th, tlo = g->min_th;

    // ---- compass pretest at iniThFAST (necessary for a 9-arc: some adjacent compass pair
    // (0,4), (4,8), (8,12), (12,0) is on the arc's side), bright and dark apart:
    //   bright: min(max(c0, c8), max(c4, c12)) > v + th,  dark: max(min(c0, c8), min(c4, c12)) < v - th
    // Survivors (pair, side) are ballot-compacted into one list; order is irrelevant (the
    // scores go to their place in sc) ----
    int nlist = 0;
    {
        const v2s vth1 = (v2s){(short)(thi + 1), (short)(thi + 1)};
        for (int u0 = 0, ry = ry0, gg = gg0; u0 < nunits; u0 += 64) {
            const int u = u0 + lane;
            uint32_t pa = 0, pb = 0;
            if (u < nunits) {
                const uint32_t *p = (const uint32_t *)(tA + ry * P + 4 * gg);
                uint32_t r0[3], r3[3], r6[3];
#pragma unroll
                for (int k = 0; k < 3; k++) {
                    r0[k] = p[k];
                    r3[k] = p[3 * P4 + k];
                    r6[k] = p[6 * P4 + k];
                }
                // bits: 0/1 bright pixel i/i+1, 2/3 dark pixel i/i+1
                auto pretest = [&](auto I) -> uint32_t {
                    constexpr int i = decltype(I)::value;
                    const v2s v = gather2<4 + i>(r3[0], r3[1], r3[2]);
                    const v2s c0 = gather2<4 + i>(r6[0], r6[1], r6[2]);
                    const v2s c4 = gather2<7 + i>(r3[0], r3[1], r3[2]);
                    const v2s c8 = gather2<4 + i>(r0[0], r0[1], r0[2]);
                    const v2s c12 = gather2<1 + i>(r3[0], r3[1], r3[2]);
                    const v2s mb = pmin(pmax(c0, c8), pmax(c4, c12));
                    const v2s md = pmax(pmin(c0, c8), pmin(c4, c12));
                    const uint32_t wb = __builtin_bit_cast(uint32_t, (v2s)(mb - v - vth1));
                    const uint32_t wd = __builtin_bit_cast(uint32_t, (v2s)(v - md - vth1));
                    return (~wb >> 15 & 1u) | (~wb >> 30 & 2u) | (~wd >> 13 & 4u) |
                           (~wd >> 28 & 8u);
                };
                pa = pretest(std::integral_constant<int, 0>{});
                pb = pretest(std::integral_constant<int, 2>{});
                const int valid = min(RW - 4 * gg, 4);  // pixels of the unit inside the region
                pa &= valid > 1 ? 15u : 5u;
                pb &= valid > 3 ? 15u : (valid > 2 ? 5u : 0u);
            }
            const uint16_t e = (uint16_t)(ry << 8 | gg << 2);
            auto append = [&](bool flag, uint16_t tag) {
                const unsigned long long m = __ballot(flag);
                const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
                if (flag) list[nlist + below] = (uint16_t)(e | tag);
                nlist += __popcll(m);
            };
            append((pa & 3u) != 0, 0);   // pixels 0-1, bright
            append((pa & 12u) != 0, 1);  // pixels 0-1, dark
            append((pb & 3u) != 0, 2);   // pixels 2-3, bright
            append((pb & 12u) != 0, 3);  // pixels 2-3, dark
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

    // ---- one side of one pixel pair per listed entry ----
    for (int j = lane; j < nlist; j += 64) {
        const int e = list[j];
        const int ry = e >> 8, gg = (e >> 2) & 63, half = (e >> 1) & 1;
        const uint32_t flip = (e & 1) ? 0xFFFFFFFFu : 0u;  // dark: complemented bytes
        const uint32_t *p = (const uint32_t *)((half ? tB : tA) + ry * P + 4 * gg);
        Rows7 R;
#pragma unroll
        for (int r = 0; r < 7; r++) {
            R.w[r][0] = p[r * P4] ^ flip;
            R.w[r][1] = p[r * P4 + 1] ^ flip;
            R.w[r][2] = p[r * P4 + 2] ^ flip;
        }
        const v2s s = fast_score_side<0>(R);
        const uint32_t s0 = (uint16_t)s.x >= (uint32_t)thi ? (uint16_t)s.x : 0u;
        uint32_t s1 = (uint16_t)s.y >= (uint32_t)thi ? (uint16_t)s.y : 0u;
        if (RW - 4 * gg < 2 * half + 2) s1 = 0;  // pixel i + 1 past the region
        __hip_atomic_fetch_or((uint32_t *)(sc + (ry + 1) * P + 4 * gg + 4),
                              (s0 | s1 << 8) << (16 * half), __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
    wave_sync_lds();
    if (g->dbg == 12) return;

    // ---- NMS (cell-local) + raster-order compaction, as k_fast_cells ----
    // cv::FAST keeps p iff s_p > every neighbour's score, a neighbour that is not a corner
    // at the cell threshold th counting as 0; with s_p >= max(th, 1) that is exactly
    //   max(raw 8-neighbour scores) < max(th, s_p).
    const v2s one = (v2s){1, 1};
    auto keep_bits = [&](int ry, int gg, int th) -> uint32_t {
        const v2s t1v = (v2s){(short)max(th, 1), (short)max(th, 1)};
        const v2s thv = (v2s){(short)th, (short)th};
        const uint32_t *m = (const uint32_t *)(sc + ry * P + 4 * gg);
        const uint32_t c1 = m[P4 + 1];
        if (c1 == 0) return 0u;  // a unit with no scored pixel keeps nothing
        const uint32_t u0 = m[0], u1 = m[1], u2 = m[2];
        const uint32_t c0 = m[P4], c2 = m[P4 + 2];
        const uint32_t d0 = m[2 * P4], d1 = m[2 * P4 + 1], d2 = m[2 * P4 + 2];
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
    const int64_t slot = (int64_t)f * g->ncells + c;
    uint2 *out = cell_kp + slot * g->cell_cap;
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
        if (kb) {
            int off = run + incl - n;
            const uint32_t c1 = *(const uint32_t *)(sc + (ry + 1) * P + 4 * gg + 4);
            const int xx = xo + 4 * gg, y = yo + ry;
#pragma unroll
            for (int i = 0; i < 4; i++)
                if (kb & (1u << i))
                    out[off++] = make_uint2(orbg_pack(xx + i, y, (c1 >> (8 * i)) & 0xFF), cx[i] | cy);
        }
        run += tot;
    };
    // units with a corner (nonzero score word), raster order, over the dead pretest list
    uint16_t *plist = list;
    int npass = 0;
    for (int u0 = 0, ry = ry0, gg = gg0; u0 < nunits; u0 += 64) {
        const bool corner =
            u0 + lane < nunits && *(const uint32_t *)(sc + (ry + 1) * P + 4 * gg + 4) != 0;
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
        // an empty cell retries at minThFAST (ORBextractor.cc:1069-1075): every unit scored
        // on both sides (the window tiles are intact), then NMS at minThFAST
        wave_sync_lds();
        for (int u = lane, ry = ry0, gg = gg0; u < nunits; u += 64) {
            Rows7 R;
            const uint32_t *p = (const uint32_t *)(tA + ry * P + 4 * gg);
#pragma unroll
            for (int r = 0; r < 7; r++) {
                R.w[r][0] = p[r * P4];
                R.w[r][1] = p[r * P4 + 1];
                R.w[r][2] = p[r * P4 + 2];
            }
            const v2s sa = fast_score_pair<0>(R);
            const v2s sb = fast_score_pair<2>(R);
            uint32_t word = (uint32_t)(uint16_t)sa.x | ((uint32_t)(uint16_t)sa.y << 8) |
                            ((uint32_t)(uint16_t)sb.x << 16) | ((uint32_t)(uint16_t)sb.y << 24);
            const int valid = min(RW - 4 * gg, 4);
            if (valid < 4) word &= (1u << (8 * valid)) - 1u;
            *(uint32_t *)(sc + (ry + 1) * P + 4 * gg + 4) = word;
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

// instantiated LDS pitches (dwords); the host plan picks one, else k_fast_cells
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

hipError_t launch_fast2(int p4, dim3 grid, size_t lds, hipStream_t st, const OrbgGeom *g,
                        const OrbgCell *cells, const uint8_t *img0, int64_t img_fs,
                        int img_pitch, const uint8_t *pyr, const uint32_t *ctab,
                        int32_t *cell_cnt, uint2 *cell_kp, int nframes, int c_begin,
                        int c_count)
{
    switch (p4) {
#define X(n)                                                                                  \
    case n:                                                                                   \
        if (lds > 64 * 1024) {                                                                \
            hipError_t e = hipFuncSetAttribute((const void *)k_fast2<n>,                      \
                                               hipFuncAttributeMaxDynamicSharedMemorySize,    \
                                               (int)lds);                                     \
            if (e != hipSuccess) return e;                                                    \
        }                                                                                     \
        hipLaunchKernelGGL(k_fast2<n>, grid, dim3(256), lds, st, g, cells, img0, img_fs,      \
                           img_pitch, pyr, ctab, cell_cnt, cell_kp, nframes, c_begin, c_count); \
        return hipGetLastError();
        ORBG_FAST2_PITCHES(X)
#undef X
    default:
        return hipErrorInvalidValue;
    }
}

}  // namespace orbg
