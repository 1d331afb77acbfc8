// pyramid_kernels.hip -- k_pyramid: ComputePyramid (ORBextractor.cc:1400-1443, cv::resize
// INTER_LINEAR 8UC1, fixed point) for every level of a frame in ONE launch, for gfx950.
//
// k_resize (extract_kernels.hip) builds one level per launch: seven dependent launches,
// each latency-bound at its tail, and ~35 VALU ops per output pixel spent on byte gathers
// from LDS.  Here a workgroup owns (frame, band of rows) and walks the levels in order with
// a workgroup barrier between them, reading the previous level back from L2 (its own
// writes, same CU):
//   - bands: the host gives every band, per level, the rows it computes -- its own rows plus
//     the rows its higher levels read (the closure), so bands never wait on each other.  Rows
//     in two bands' closures are written twice with the same bytes;
//   - a lane owns an 8 x 8 output block: per source row one 16-byte load, three
//     v_alignbyte to the 12 bytes starting at the block's first source column, then per
//     output column one v_perm (the two source bytes as u16 lanes, selectors precomputed
//     per octet) and one v_dot2_u32_u16 against {a0, a1} << 4, i.e. h << 4;
//   - the vertical pass of cv::resize's SIMD bulk, ((h0 >> 4) * b0 >> 16) + ((h1 >> 4) * b1
//     >> 16) + 2 >> 2, is v_mul_hi_u32_u24((h << 4) & ~0xFF, b << 8) twice plus one add3 and
//     one shift; columns past the SIMD bulk (the last few of a row) take the scalar
//     FixedPtCast<int, uchar, 22> (h0 * b0 + h1 * b1 + 2^21) >> 22 in a wave-uniform branch.
// ~10 VALU ops per output pixel.  Bit-exact with k_resize and the oracle's resize modes.
#include <hip/hip_runtime.h>

#include "orbg_device.h"
#include "blur_device.h"
#include "pyramid_args.h"

#pragma clang fp contract(off)

namespace orbg {

__device__ __forceinline__ uint32_t pyr_dot2(uint32_t a, uint32_t b)
{
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    return __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b), 0u,
                                  false);
}

// (x * y) >> 16 for x = (h >> 4) << 8 < 2^24 and y = b << 8 < 2^20: v_mul_hi_u32_u24
__device__ __forceinline__ uint32_t pyr_mulhi(uint32_t h16, uint32_t b8)
{
    const uint32_t x = h16 & 0x00FFFF00u, y = b8 & 0x000FFFFFu;
    return (uint32_t)(((unsigned long long)x * y) >> 32);
}

struct PyrOct {
    uint32_t sel[PYR_COLS], cf[PYR_COLS];
};

// h << 4 of the octet's 8 output columns from one source row's 16 raw bytes (o = byte
// offset of source column sx0 in the first dword)
__device__ __forceinline__ void pyr_hrow(uint4 raw, uint32_t o, const PyrOct &t,
                                         uint32_t h[PYR_COLS])
{
    const uint32_t w0 = __builtin_amdgcn_alignbyte(raw.y, raw.x, o);
    const uint32_t w1 = __builtin_amdgcn_alignbyte(raw.z, raw.y, o);
    const uint32_t w2 = __builtin_amdgcn_alignbyte(raw.w, raw.z, o);
#pragma unroll
    for (int i = 0; i < 4; i++) h[i] = pyr_dot2(__builtin_amdgcn_perm(w1, w0, t.sel[i]), t.cf[i]);
#pragma unroll
    for (int i = 4; i < 8; i++) h[i] = pyr_dot2(__builtin_amdgcn_perm(w2, w1, t.sel[i]), t.cf[i]);
}

// 16 bytes at the 4-aligned address at or below p (o = p & 3); with `guard`, bytes at or
// past `end` (the caller's last image byte + 1) are not read
__device__ __forceinline__ uint4 pyr_load(const uint8_t *p, const uint8_t *end, bool guard,
                                          uint32_t &o)
{
    o = (uint32_t)(uintptr_t)p & 3u;
    // pointer arithmetic, not an integer round trip: the compiler keeps the global address
    // space (global_load, not flat_load: a flat load also counts in lgkmcnt, so every scalar
    // ytab load's wait would drain the prefetched rows)
    const uint8_t *a = p - o;
    if (guard && a + 16 > end) {
        uint32_t w[4] = {0, 0, 0, 0};
        for (int b = 0; b < 16; b++)
            if (a + b < end) w[b >> 2] |= (uint32_t)a[b] << (8 * (b & 3));
        return make_uint4(w[0], w[1], w[2], w[3]);
    }
    return *(const uint4 *)a;
}

__device__ __forceinline__ void pyr_oct(const uint4 *__restrict__ oct, PyrOct &t)
{
    const uint4 s0 = oct[1], s1 = oct[2], c0 = oct[3], c1 = oct[4];
    t.sel[0] = s0.x; t.sel[1] = s0.y; t.sel[2] = s0.z; t.sel[3] = s0.w;
    t.sel[4] = s1.x; t.sel[5] = s1.y; t.sel[6] = s1.z; t.sel[7] = s1.w;
    t.cf[0] = c0.x; t.cf[1] = c0.y; t.cf[2] = c0.z; t.cf[3] = c0.w;
    t.cf[4] = c1.x; t.cf[5] = c1.y; t.cf[6] = c1.z; t.cf[7] = c1.w;
}

// Fast path, one wave: output rows [y0, y0 + n) (wave-uniform: SGPRs, scalar ytab loads)
// x 64 column octets (lane = octet).  Source rows are walked in order, fully unrolled,
// PYR_PF loads ahead; no branch but the uniform "row k completes here".  Stores only
// `store` lanes (octets without FixedPtCast columns) and rows with sy0 != sy1: the rest is
// pyr_fix's.  The loads never pass the caller's buffer (the host routes the wave items
// that could to pyr_fix as well).
__device__ __forceinline__ void pyr_wave_item(const uint8_t *__restrict__ src, int spitch,
                                              uint8_t *__restrict__ dst, int dpitch,
                                              const int4 *__restrict__ ytab,
                                              const uint4 *__restrict__ oct, int dx0, bool store,
                                              int y0, int n)
{
    PyrOct t;
    pyr_oct(oct, t);
    const int sx0 = (int)oct[0].x;
    int4 yt = ytab[y0];
    const int first = yt.x & 0xFFFF;
    const int nsrc = (ytab[y0 + n - 1].x >> 16) - first + 1;  // <= PYR_NS (host plan)
    const uint8_t *rp = src + (int64_t)first * spitch + sx0;
    uint4 ring[PYR_PF];
    uint32_t oring[PYR_PF];
#pragma unroll
    for (int p = 0; p < PYR_PF; p++)
        ring[p] = pyr_load(rp + (int64_t)min(p, nsrc - 1) * spitch, nullptr, false, oring[p]);
    uint32_t h[2][PYR_COLS];
#pragma unroll
    for (int i = 0; i < PYR_COLS; i++) h[1][i] = 0;
    int k = 0, nexty = (yt.x >> 16) - first;  // source row (relative) completing row k
    uint8_t *drow = dst + (int64_t)y0 * dpitch + dx0;
#pragma unroll
    for (int j = 0; j < PYR_NS; j++) {
        // rows past nsrc re-sum the last row (clamped loads) and complete no output row
        uint32_t *hc = h[j & 1], *hp = h[(j & 1) ^ 1];
        const uint4 raw = ring[j % PYR_PF];
        const uint32_t o = oring[j % PYR_PF];
        if (j + PYR_PF < PYR_NS)
            ring[j % PYR_PF] = pyr_load(rp + (int64_t)min(j + PYR_PF, nsrc - 1) * spitch,
                                        nullptr, false, oring[j % PYR_PF]);
        pyr_hrow(raw, o, t, hc);
#pragma unroll
        for (int i = 0; i < PYR_COLS; i++) hc[i] &= 0x00FFFF00u;  // (h >> 4) << 8
        // output row k completes at its sy1 (at most one per source row: scale > 1)
        if (j == nexty) {
            const uint32_t y8 = (uint32_t)yt.y & 0x000FFFFFu, z8 = (uint32_t)yt.z & 0x000FFFFFu;
            uint32_t v[PYR_COLS];
#pragma unroll
            for (int i = 0; i < PYR_COLS; i++) {
                const uint32_t a = (uint32_t)(((unsigned long long)hp[i] * y8) >> 32);
                const uint32_t b = (uint32_t)(((unsigned long long)hc[i] * z8) >> 32);
                v[i] = (a + b + 2) >> 2;
            }
            const uint32_t lo = v[0] | v[1] << 8 | v[2] << 16 | v[3] << 24;
            const uint32_t hi = v[4] | v[5] << 8 | v[6] << 16 | v[7] << 24;
            if ((yt.x & 0xFFFF) - first != j && store)  // sy0 == sy1 rows: pyr_fix
                *(uint2 *)drow = make_uint2(lo, hi);    // dpitch % 64 == 0, dx0 % 8 == 0
            drow += dpitch;
            k++;
            yt = ytab[y0 + min(k, n - 1)];
            nexty = k < n ? (yt.x >> 16) - first : 1 << 30;
        }
    }
}

// One output row of one octet, every column by its own rule (SIMD bulk or FixedPtCast,
// sy0 == sy1 rows, a partial last octet), loads guarded: the octets and rows the fast path
// leaves out.
__device__ __forceinline__ void pyr_fix(const uint8_t *src, int spitch, uint8_t *dst,
                                        int dpitch, int dw, const int4 *ytab, const uint4 *oct,
                                        int dx0, int dy, const uint8_t *end, bool guard)
{
    PyrOct t;
    pyr_oct(oct, t);
    const uint4 o0 = oct[0];
    const int4 yt = ytab[dy];
    uint32_t h0[PYR_COLS], h1[PYR_COLS];
    {
        uint32_t o;
        uint4 raw = pyr_load(src + (int64_t)(yt.x & 0xFFFF) * spitch + (int)o0.x, end, guard, o);
        pyr_hrow(raw, o, t, h0);
        raw = pyr_load(src + (int64_t)(yt.x >> 16) * spitch + (int)o0.x, end, guard, o);
        pyr_hrow(raw, o, t, h1);
    }
    const uint32_t b0 = (uint32_t)yt.w & 0xFFFFu, b1 = (uint32_t)yt.w >> 16;
    uint8_t *d = dst + (int64_t)dy * dpitch + dx0;
    const int nc = min(PYR_COLS, dw - dx0);
#pragma unroll
    for (int i = 0; i < PYR_COLS; i++) {
        uint32_t v;
        if (o0.y >> i & 1u) {
            v = ((h0[i] >> 4) * b0 + (h1[i] >> 4) * b1 + (1u << 21)) >> 22;
        } else {
            const uint32_t a = (uint32_t)(((unsigned long long)(h0[i] & 0x00FFFF00u) *
                                           ((uint32_t)yt.y & 0x000FFFFFu)) >> 32);
            const uint32_t b = (uint32_t)(((unsigned long long)(h1[i] & 0x00FFFF00u) *
                                           ((uint32_t)yt.z & 0x000FFFFFu)) >> 32);
            v = (a + b + 2) >> 2;
        }
        if (i < nc) d[i] = (uint8_t)v;
    }
}

// grid: nband * nframes workgroups (XCD-remapped: a frame's bands share an L2); levels
// [1, L) in order, one phase per level with a workgroup barrier after it.  Phase p computes
// level p + 1's rows of the band: fast wave items (row group of PYR_ROWS rows x chunk of 64
// octets), then the fix-up rows (one lane per (row, octet)): the octets from P.fix_oct on
// (FixedPtCast columns, a partial last octet) for every row, every octet of the sy0 == sy1 rows
// from P.clamp_row on, and for the caller image every octet of the rows whose fast loads could
// pass the buffer (from P.guard_row on, last frame only).  With A.fuse_blur the same phase also
// blurs level p's own rows (k_blur2's wave tiles, blur_device.h): level p is complete in this
// workgroup (level 0 is the caller's image), still in L2, and no second kernel re-reads the
// pyramid from HBM to blur it (ORBextractor.cc:1375-1377 after :1400-1443).
__global__ __launch_bounds__(1024) void k_pyramid(PyrArgs A, const OrbgGeom *__restrict__ g,
                                                 const uint4 *__restrict__ ptab,
                                                 const int4 *__restrict__ ytab_all,
                                                 const int4 *__restrict__ bands,
                                                 const uint8_t *__restrict__ img0,
                                                 int64_t img_fs, int img_pitch,
                                                 const uint8_t *img_end, uint8_t *pyr,
                                                 uint8_t *blur, int nframes)
{
    const int id = xcd_remap(blockIdx.x, gridDim.x);
    const int f = id / A.nband, band = id - f * A.nband;
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nw = blockDim.x >> 6;
    uint8_t *fpyr = pyr + (int64_t)f * A.pyr_frame;
    for (int ph = 0; ph < A.L; ph++) {
        const int l = ph + 1;
        if (l < A.L) {
            const PyrLevelArgs &P = A.lv[l];
            const bool lvl1 = l == 1;
            const uint8_t *src = lvl1 ? img0 + (int64_t)f * img_fs : fpyr + P.src_off;
            const int spitch = lvl1 ? img_pitch : P.spitch;
            uint8_t *dst = fpyr + P.dst_off;
            const int4 cr = bands[band * A.L + l];
            const int4 *ytab = ytab_all + P.ytab_off;
            const uint4 *ptab_l = ptab + P.ptab_off;
            // rows [cr.x, fast_end) go through the fast path (the caller image's last frame
            // stops before its guarded rows)
            const int fast_end = (lvl1 && f == nframes - 1) ? min(cr.y, P.guard_row) : cr.y;
            const int ngroups = max(fast_end - cr.x, 0) / PYR_ROWS + ((max(fast_end - cr.x, 0) % PYR_ROWS) != 0);
            const int nchunk = (P.fix_oct + 63) >> 6;
            const int items = ngroups * nchunk;
            for (int it = wv; it < items; it += nw) {
                const int gi = it / nchunk, cc = it - gi * nchunk;
                const int q = 64 * cc + lane;
                const int y0 = cr.x + gi * PYR_ROWS, n = min(PYR_ROWS, fast_end - y0);
                pyr_wave_item(src, spitch, dst, P.dpitch, ytab, ptab_l + 5 * min(q, P.fix_oct - 1),
                              q * PYR_COLS, q < P.fix_oct, y0, n);
            }
            // fix-up: (row, octet) pairs
            {
                const int nrow = cr.y - cr.x, nfo = P.noct - P.fix_oct;
                const int clamp0 = max(P.clamp_row, cr.x), guard0 = max(fast_end, cr.x);
                const int nclamp = max(cr.y - clamp0, 0), nguard = max(cr.y - guard0, 0);
                const int n1 = nrow * nfo;                       // FixedPtCast / partial octets
                const int n2 = n1 + nclamp * P.fix_oct;          // sy0 == sy1 rows
                const int n3 = n2 + (guard0 < clamp0 ? min(nguard, clamp0 - guard0) : 0) * P.fix_oct;
                for (int i = threadIdx.x; i < n3; i += blockDim.x) {
                    int dy, q;
                    if (i < n1) {
                        dy = cr.x + i / nfo;
                        q = P.fix_oct + i % nfo;
                    } else if (i < n2) {
                        dy = clamp0 + (i - n1) / P.fix_oct;
                        q = (i - n1) % P.fix_oct;
                    } else {
                        dy = guard0 + (i - n2) / P.fix_oct;
                        q = (i - n2) % P.fix_oct;
                    }
                    pyr_fix(src, spitch, dst, P.dpitch, P.dw, ytab, ptab_l + 5 * q, q * PYR_COLS,
                            dy, img_end, lvl1);
                }
            }
        }
        if (A.fuse_blur == 1 || (A.fuse_blur == 2 && ph > 0)) {
            // GaussianBlur of level ph's own rows of this band (every source row it reads is
            // the band's: computed in the phase before, the barrier orders it)
            const int4 bo = bands[band * A.L + ph];
            const bool l0 = ph == 0;
            const int W = l0 ? A.w0 : A.lv[ph].dw, H = l0 ? A.h0 : A.lv[ph].dh;
            const uint8_t *bsrc = l0 ? img0 + (int64_t)f * img_fs : fpyr + A.lv[ph].dst_off;
            const int bp = l0 ? img_pitch : A.lv[ph].dpitch;
            const int dp = l0 ? A.bpitch0 : A.lv[ph].dpitch;
            uint8_t *bdst = blur + (int64_t)f * A.blur_frame + (l0 ? A.blur_off0 : A.lv[ph].blur_off);
            const int ntx = (W + BLUR2_TW - 1) / BLUR2_TW;
            const int nseg = (max(bo.w - bo.z, 0) + PYR_BLUR_SEG - 1) / PYR_BLUR_SEG;
            if (nseg > 0) {
                const Blur2Weights kw(g);
                for (int it = wv; it < ntx * nseg; it += nw) {
                    const int sg = it / ntx, tx = it - sg * ntx;
                    blur2_tile<PYR_BLUR_SEG>(kw, bsrc, bp, W, H, bdst, dp, tx,
                                             bo.z + sg * PYR_BLUR_SEG, bo.w, lane);
                }
            }
        }
        // level l is complete in this workgroup before level l + 1 reads it (same CU: the
        // barrier's workgroup-scope release/acquire orders the global stores and loads)
        __syncthreads();
    }
}

}  // namespace orbg
