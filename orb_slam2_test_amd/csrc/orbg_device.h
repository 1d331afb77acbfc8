// orbg_device.h -- small wave64 helpers shared by the kernel translation units.
#pragma once

#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

namespace orbg {

// inclusive wave64 prefix sum by DPP (row_shr 1..3 from the inputs, row_shr 4 / 8 with bank
// masks, row_bcast 15 / 31 with row masks): seven adds, no LDS round trips (a __shfl_up
// ladder is six ds_bpermute round trips, on the critical path of every block scan: the
// quadtree's chains of scans and barriers, the matchers' compactions).  Integer adds, exact.
__device__ __forceinline__ int wave_incl_scan(int x)
{
    int y = x;
    y += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true);  // row_shr:1
    y += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true);  // row_shr:2
    y += __builtin_amdgcn_update_dpp(0, x, 0x113, 0xf, 0xf, true);  // row_shr:3
    y += __builtin_amdgcn_update_dpp(0, y, 0x114, 0xf, 0xe, true);  // row_shr:4, banks 1-3
    y += __builtin_amdgcn_update_dpp(0, y, 0x118, 0xf, 0xc, true);  // row_shr:8, banks 2-3
    y += __builtin_amdgcn_update_dpp(0, y, 0x142, 0xa, 0xf, false); // row_bcast:15, rows 1, 3
    y += __builtin_amdgcn_update_dpp(0, y, 0x143, 0xc, 0xf, false); // row_bcast:31, rows 2, 3
    return y;
}
__device__ __forceinline__ int wave_incl_scan_dpp(int x) { return wave_incl_scan(x); }

// the round-5 form (a __shfl_up ladder), kept for A/B builds (-DORBG_SCAN_SHFL)
__device__ __forceinline__ int wave_incl_scan_shfl(int x)
{
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    return x;
}
#ifdef ORBG_SCAN_SHFL
#define wave_incl_scan wave_incl_scan_shfl
#endif

// inclusive wave prefix of small counts 0 <= x < 8 from three ballots (no shuffles);
// *total = wave total
__device__ __forceinline__ int wave_incl_scan_small(int x, int *total)
{
    int incl = 0, tot = 0;
#pragma unroll
    for (int b = 0; b < 3; b++) {
        const unsigned long long m = __ballot((x >> b) & 1);
        const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
        incl += (below + ((x >> b) & 1)) << b;
        tot += __popcll(m) << b;
    }
    *total = tot;
    return incl;
}

// wave64 sum, uniform result: every lane gets its 16-lane row's sum by DPP quad_perm /
// row_ror adds, row_bcast:15 / row_bcast:31 fold the four rows into lane 63 (gfx9 DPP: no
// LDS round trips, unlike __shfl_xor's ds_bpermute).  Integer adds, exact in any order.
__device__ __forceinline__ int wave_sum(int x)
{
    x += __builtin_amdgcn_update_dpp(0, x, 0xb1, 0xf, 0xf, false);   // quad_perm [1,0,3,2]
    x += __builtin_amdgcn_update_dpp(0, x, 0x4e, 0xf, 0xf, false);   // quad_perm [2,3,0,1]
    x += __builtin_amdgcn_update_dpp(0, x, 0x124, 0xf, 0xf, false);  // row_ror:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x128, 0xf, 0xf, false);  // row_ror:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xf, 0xf, false);  // row_bcast:15 (row r += r-1)
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xf, 0xf, false);  // row_bcast:31 (rows 2, 3)
    return __builtin_amdgcn_readlane(x, 63);
}

// LDS written by some lanes of a wave, then read by others: keep the compiler from
// reordering (the hardware keeps one wave's LDS ops in order).
__device__ __forceinline__ void wave_sync_lds()
{
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// XCD-aware block remap (cdna_hip_programming.md T1, bijective for nwg % 8 != 0).
// The dispatcher deals workgroups round-robin over the 8 XCDs (orig % 8 shares an L2);
// the remap hands each XCD a contiguous run of logical blocks, so neighbouring cells /
// tiles / keypoints of one frame (which share halo lines and pyramid levels) hit in the
// same 4 MiB L2 instead of being fetched once per XCD.  Speed only, never correctness.
__device__ __forceinline__ int xcd_remap(int orig, int nwg)
{
    const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

// double sin/cos pinned to one polynomial so the oracle (orb_oracle.c) matches bit for bit
__device__ __forceinline__ void pinned_sincos(double x, double *s, double *c)
{
    const double two_over_pi = 6.36619772367581382433e-01;
    const double pio2_1 = 1.57079632673412561417e+00;
    const double pio2_1t = 6.07710050650619224932e-11;
    const double kd = rint(x * two_over_pi);
    const int k = (int)kd;
    const double r = (x - kd * pio2_1) - kd * pio2_1t;
    const double r2 = r * r;
    const double sp =
        r + r * r2 *
                (-1.0 / 6.0 +
                 r2 * (1.0 / 120.0 +
                       r2 * (-1.0 / 5040.0 +
                             r2 * (1.0 / 362880.0 +
                                   r2 * (-1.0 / 39916800.0 +
                                         r2 * (1.0 / 6227020800.0 +
                                               r2 * (-1.0 / 1307674368000.0 +
                                                     r2 * (1.0 / 355687428096000.0 +
                                                           r2 * (-1.0 / 121645100408832000.0)))))))));
    const double cp =
        1.0 + r2 * (-0.5 +
                    r2 * (1.0 / 24.0 +
                          r2 * (-1.0 / 720.0 +
                                r2 * (1.0 / 40320.0 +
                                      r2 * (-1.0 / 3628800.0 +
                                            r2 * (1.0 / 479001600.0 +
                                                  r2 * (-1.0 / 87178291200.0 +
                                                        r2 * (1.0 / 20922789888000.0 +
                                                              r2 * (-1.0 / 6402373705728000.0)))))))));
    switch (k & 3) {
    case 0: *s = sp; *c = cp; break;
    case 1: *s = cp; *c = -sp; break;
    case 2: *s = -sp; *c = -cp; break;
    default: *s = -cp; *c = sp; break;
    }
}

// glibc 2.35 sinf / cosf (sysdeps/ieee754/flt-32/s_sinf.c, s_cosf.c, sincosf.h and its
// __sincosf_table) for |y| < 120 -- the rBRIEF rotation's (float)cos(angle) /
// (float)sin(angle) (ORBextractor.cc:122) resolve to these.  Same restatement as
// oracle/orb_oracle.c orc_glibc_sinf/cosf; both equal the host libm for every float in
// [0, 7) (tools/sincosf_sweep.c).  Double arithmetic, unfused (-ffp-contract=off; the
// fused x86_64 build rounds to the same floats on that range), one rounding to float.
static __constant__ const double orbg_sincosf_tab[2][14] = {
    {1.0, -1.0, -1.0, 1.0, 0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0, 1.0,
     -0x1.ffffffd0c621cp-2, -0x1.555545995a603p-3, 0x1.55553e1068f19p-5, 0x1.1107605230bc4p-7,
     -0x1.6c087e89a359dp-10, -0x1.994eb3774cf24p-13, 0x1.99343027bf8c3p-16},
    {1.0, -1.0, -1.0, 1.0, 0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0, -1.0,
     0x1.ffffffd0c621cp-2, -0x1.555545995a603p-3, -0x1.55553e1068f19p-5, 0x1.1107605230bc4p-7,
     0x1.6c087e89a359dp-10, -0x1.994eb3774cf24p-13, -0x1.99343027bf8c3p-16}};

// sinf_poly: sine polynomial for even n, cosine for odd n
__device__ __forceinline__ float glibc_sincosf_poly(double x, double x2, const double *p, int n)
{
    if ((n & 1) == 0) {
        const double x3 = x * x2;
        const double s1 = p[10] + x2 * p[12];  // s2 + x2 * s3
        const double x7 = x3 * x2;
        const double s = x + x3 * p[8];        // x + x3 * s1
        return (float)(s + x7 * s1);
    }
    const double x4 = x2 * x2;
    const double c2 = p[11] + x2 * p[13];      // c3 + x2 * c4
    const double c1 = p[6] + x2 * p[7];        // c0 + x2 * c1
    const double x6 = x4 * x2;
    const double c = c1 + x4 * p[9];           // c1 + x4 * c2
    return (float)(c + x6 * c2);
}

// *c = cosf(y), *s = sinf(y) as glibc computes them (quadrant reduction shared)
__device__ __forceinline__ void glibc_sincosf(float y, float *s, float *c)
{
    const uint32_t top = (__float_as_uint(y) >> 20) & 0x7ff;
    double x = y;
    if (top < 0x3f4) {            // abstop12(y) < abstop12(pio4)
        if (top < 0x398) {        // < abstop12(0x1p-12f)
            *s = y;
            *c = 1.0f;
            return;
        }
        const double x2 = x * x;
        *s = glibc_sincosf_poly(x, x2, orbg_sincosf_tab[0], 0);
        *c = glibc_sincosf_poly(x, x2, orbg_sincosf_tab[0], 1);
        return;
    }
    // reduce_fast without TOINT_INTRINSICS: quadrant from the 2^24-scaled product
    const double r = x * orbg_sincosf_tab[0][4];
    const int n = ((int32_t)r + 0x800000) >> 24;
    x = x - n * orbg_sincosf_tab[0][5];
    const double sg = orbg_sincosf_tab[0][n & 3];
    const double *p = orbg_sincosf_tab[(n & 2) ? 1 : 0];
    const double xs = x * sg, x2 = x * x;
    *s = glibc_sincosf_poly(xs, x2, p, n);
    *c = glibc_sincosf_poly(xs, x2, p, n ^ 1);
}

}  // namespace orbg
