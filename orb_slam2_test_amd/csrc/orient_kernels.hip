// orient_kernels.hip -- IC_Angle (ORBextractor.cc:83-111, computeOrientation :523-530),
// computeOrbDescriptor (:117-157) and the output assembly of ORBextractor::operator()
// (:1381-1395) as one batched HIP kernel for gfx950.
// Bit-exactness pins: no FMA contraction (-ffp-contract=off + pragma),
// cvRound = round-half-even, fastAtan2 polynomial, glibc cosf/sinf restated (orbg_device.h).
#include <hip/hip_runtime.h>

#include "orbg_internal.h"
#include "orbg_device.h"

#pragma clang fp contract(off)

namespace orbg {

// bit_pattern_31_ (ORBextractor.cc:160-418): test t = bytes 4t .. 4t+3 = (x0, y0, x1, y1)
__device__ __attribute__((aligned(16))) int8_t od_pattern_i8[1024] = {
#define ORBG_PAIR(a, b, c, d) a, b, c, d,
#include "orb_pattern.inc"
#undef ORBG_PAIR
};


// cv::fastAtan2 (OpenCV 3.4 atan_f32), degrees in [0, 360]
__device__ __forceinline__ float fast_atan2(float y, float x)
{
    const float r2d = (float)(180 / 3.14159265358979323846);
    const float p1 = 0.9997878412794807f * r2d;
    const float p3 = -0.3258083974640975f * r2d;
    const float p5 = 0.1555786518463281f * r2d;
    const float p7 = -0.04432655554792128f * r2d;
    const float eps = (float)2.2204460492503131e-16;
    const float ax = fabsf(x), ay = fabsf(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + eps);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + eps);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

// ---------------------------------------------------------------------------
// k_orient_desc: each wave owns OD_KPW consecutive quadtree output slots of one frame
// (frame, level, list position); the keypoint of a filled slot is written at
// i = (keypoints of lower levels) + position, the level-major order of ORBextractor.cc:1381.
// Lane j < OD_KPW locates slot j once; the wave then runs three phases, so the wave-uniform
// scalar math (fastAtan2, the double sincos, the keypoint record) runs once per wave with
// one slot per lane instead of once per slot on all 64 lanes:
//   A  per slot: the 31x31 unblurred patch as 93 aligned 16-byte row chunks; circle-masked
//      moments are v_dot4_u32_u8 products with per-(alignment, lane) byte tables staged in
//      LDS (weights u+15 and ones, 0 outside the circle), so per 16 patch bytes
//      m_10 += dot(w) - 15 dot(1) and m_01 += v dot(1); DPP wave sums; lane j keeps slot j's;
//   B  all lanes at once: angle, cos, sin; lanes j write their keypoint records;
//   C  per slot: the 37x37 blurred neighbourhood (every rotated rBRIEF sample lies within
//      +-18 px) staged in LDS; lane L runs tests L, L+64, L+128, L+192, so ballot t is
//      descriptor bits 64t .. 64t+63 and lanes 0..7 store the 32 bytes as dwords.
// ---------------------------------------------------------------------------
struct OrbgKeypointDev {
    float x, y, size, angle, response;
    int32_t octave, class_id;
};

#define OD_R 18                 // rBRIEF sample radius bound: 13 * sqrt(2) rounded
#define OD_SPAN (2 * OD_R + 1)  // 37 rows
#define OD_ROWB 48              // staged row: 3 x 16 bytes (37 bytes + up to 3 of alignment)
// tiled blurred levels (G.blur_tiled, TB): the staged row starts at the window's tile column
// (16-px aligned) and holds bytes d .. d + 36 of it, d = window left & 15 <= 15: 52 bytes
#define OD_ROWB_T 52
#define OD_BPW ((OD_SPAN * OD_ROWB_T + 15) / 16)  // staged neighbourhood per wave (uint4)
#define OD_KPW ORBG_OD_KPW      // slots per wave
#ifndef ORBG_OD_LDSTAB
#define ORBG_OD_LDSTAB 1
#endif
#ifndef ORBG_OD_WPE
#define ORBG_OD_WPE 8  // min waves per SIMD (VGPR budget)
#endif
#define OD_TABW ORBG_OD_TABW    // IC_Angle lanes: 31 patch rows x 3 16-byte chunks
#ifndef ORBG_OD_PRIO
#define ORBG_OD_PRIO 1  // wave priority (s_setprio) of k_orient_desc (with k_octree_lds at 2: -1% per step)
#endif
#ifndef ORBG_OD_PFD
#define ORBG_OD_PFD 2  // slots whose loads are in flight ahead of the one being summed / sampled (1: -0.4% per step)
#endif
#define OD_PFD ORBG_OD_PFD
#ifndef ORBG_OD_PK
#define ORBG_OD_PK 1  // rBRIEF sample rotation on packed f32 pairs (0: scalar ops)
#endif
typedef float od_f2 __attribute__((ext_vector_type(2)));
#ifndef ORBG_OD_EARLYC
#define ORBG_OD_EARLYC 0  // phase C's first neighbourhood loads (<= OD_PFD) issued during phase A's last slots (1: orient +1.3%, 2: +16%, spills; r05k A/B)
#endif
static_assert(OD_KPW >= 1 && OD_KPW <= 32, "one slot per lane, okmask is 32 bits");

// IC_Angle byte tables (host-built, orbg_api.hip make_od_tab): entry (sh, w) for the patch
// row r = w / 3, chunk c = w % 3 loaded from the 4-byte-aligned address sh bytes before the
// row start: byte b is column u = 16c + b - sh - 15, weight u + 15 and one when
// |u| <= umax[|r - 15|], else 0.  [sh][0][w] = weights, [sh][1][w] = ones.
// BFMA: the rBRIEF rotation x*b + y*a with one FMA (brief_fma pin) or two roundings (default)
// HC (the single-frame drop-in, B = 1): every output is also stored into the packed host
// block orbg_download_frame reads (k_pack_frame's layout: [0..4) the sticky error word and
// the count, keypoints at byte hc.okp, descriptors at hc.ods), so no packing kernel and no
// copy follow the extraction
struct OdHostCopy {
    uint8_t *base;
    const int32_t *err;
    int32_t okp, ods;
    int32_t tag;  // != 0: the quadtree's fallback flag is err[4] == tag (else err[2])
};

template <bool BFMA, bool HC, bool TB>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(ORBG_OD_WPE, 8))) void k_orient_desc(
    const OrbgGeom *__restrict__ g, const uint8_t *__restrict__ img0, int64_t img_fs,
    int img_pitch, const uint8_t *__restrict__ pyr, const uint8_t *__restrict__ blur,
    const uint4 *__restrict__ odtab, const uint32_t *__restrict__ lvl_kp,
    const uint16_t *__restrict__ lvl_idx, const int32_t *__restrict__ lvl_cnt,
    OrbgKeypointDev *__restrict__ kps,
    uint8_t *__restrict__ desc, int32_t *__restrict__ counts, OdHostCopy hc)
{
#if ORBG_OD_PRIO
    __builtin_amdgcn_s_setprio(ORBG_OD_PRIO);  // on the pipelined step's critical path (A/B)
#endif
    __shared__ uint4 bpatch[4][OD_BPW];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#if ORBG_OD_LDSTAB
    __shared__ uint4 tab[4 * OD_TABW * 2];
    for (int i = threadIdx.x; i < 4 * OD_TABW * 2; i += 256) tab[i] = odtab[i];
    __syncthreads();
#else
    const uint4 *tab = odtab;  // 11.9 KB, L1/L2-resident
#endif
    const int nb = (g->out_frame + 4 * OD_KPW - 1) / (4 * OD_KPW);  // blocks per frame
    const int id = xcd_remap(blockIdx.x, gridDim.x);
    const int f = id / nb, bx = id - f * nb;
    const int s0 = __builtin_amdgcn_readfirstlane((bx * 4 + wv) * OD_KPW);  // wave-uniform
    const int L = g->L, OF = g->out_frame;
    if (s0 >= OF) return;
    const int32_t *lc = lvl_cnt + (int64_t)f * L;
    if (s0 == 0 && lane == 0) {
        int total = 0;
        for (int l = 0; l < L; l++) total += lc[l];
        counts[f] = total;
        if (HC) {  // header: the error word (final: its writers ran before), the count
            int32_t *hdr = (int32_t *)hc.base;
            hdr[0] = hc.err[0];
            hdr[1] = hc.err[1];
            hdr[2] = total;
            // a level left to k_octree (orbg_extract reruns the frame)
            hdr[3] = hc.tag ? (int32_t)(hc.err[4] == hc.tag) : hc.err[2];
        }
    }
    // lane j < OD_KPW: slot s0 + j -> quadtree key, level, output row (the winner's list
    // position lvl_idx: the octree put the slots in image-tile order); okmask bit j
    // (wave-uniform) = the slot holds a keypoint
    uint32_t kl = 0u;
    int my_lev = 0, my_i = 0, my_ok = 0;
    {
        const int slot = s0 + lane;
        if (lane < OD_KPW && slot < OF) {
            int level = 0;
            while (level + 1 < L && slot >= g->lv[level + 1].out_off) level++;
            int before = 0;
            for (int l = 0; l < level; l++) before += lc[l];
            const int pos = slot - g->lv[level].out_off;
            if (pos < lc[level]) {
                kl = lvl_kp[(int64_t)f * OF + slot];
                my_ok = 1;
                my_lev = level;
                my_i = before + lvl_idx[(int64_t)f * OF + slot];
            }
        }
    }
    const uint32_t okmask = (uint32_t)__ballot(my_ok);
    // lane-constant (row, 16-byte chunk) of the patch / neighbourhood words this lane loads
    // (the loads of lanes past the last word re-read the last word: unconditional loads keep
    // the pipelined loops below free of exec branches, so their vmcnt waits stay partial)
    int pr[2], pc[2], par[2], pac[2];
#pragma unroll
    for (int k = 0; k < 2; k++) {
        const int w = min(lane + 64 * k, OD_SPAN * 3 - 1);
        pr[k] = w / 3;
        pc[k] = w - pr[k] * 3;
        const int wa = min(lane + 64 * k, OD_TABW - 1);
        par[k] = wa / 3;
        pac[k] = wa - par[k] * 3;
    }

    if (!okmask) return;  // wave-uniform: no keypoint in this wave's slots
    // Empty slots borrow the first filled slot's key (their results are dropped), so every
    // slot's loads below are unconditional and the unrolled slot loops have no branches
    // around them: each vmcnt wait then covers exactly the current slot's loads.
    const int jfirst = __builtin_ctz(okmask);
    const uint32_t kl_l = my_ok ? kl : (uint32_t)__builtin_amdgcn_readlane((int)kl, jfirst);
    const int lev_l = my_ok ? my_lev : __builtin_amdgcn_readlane(my_lev, jfirst);
    // per-slot addresses, lane j = slot j, computed once: the slot loops take them by
    // v_readlane instead of scalar loads of the level records (which, after the LDS fences,
    // would be reissued per slot and wait on the LDS queue: both count in lgkmcnt)
    int ppitch_l, bpitch_l, bxy_l = 0;
    // patch centre (from img0 / pyr); neighbourhood top-left in the blurred level (TB: the
    // level's first byte, and bxy_l = window top << 16 | window left)
    int64_t poff_l, boff_l;
    {
        const OrbgLevel &lv = g->lv[lev_l];
        const int x = orbg_px(kl_l) + ORBG_MIN_BORDER, y = orbg_py(kl_l) + ORBG_MIN_BORDER;
        bpitch_l = lv.pitch;
        ppitch_l = lev_l == 0 ? img_pitch : bpitch_l;
        poff_l = (lev_l == 0 ? (int64_t)f * img_fs : (int64_t)f * g->pyr_frame + lv.pyr_off) +
                 (int64_t)y * ppitch_l + x;
        if (TB) {
            boff_l = (int64_t)f * g->blur_frame + lv.blur_off;
            bxy_l = (y - OD_R) << 16 | (x - OD_R);
        } else {
            boff_l = (int64_t)f * g->blur_frame + lv.blur_off + (int64_t)(y - OD_R) * bpitch_l +
                     (x - OD_R);
        }
    }
    const int64_t drow0 = (int64_t)f * g->frame_cap;  // this frame's first output row
    auto readlane64 = [](int64_t v, int j) -> int64_t {
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, j);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), j);
        return (int64_t)((uint64_t)hi << 32 | lo);
    };

    // phase C's neighbourhood loads (defined here: the first OD_PFD are issued at the end of
    // phase A, so their latency overlaps A's last slots and phase B)
    // Row-major blurred levels: lane (row pr, chunk pc) loads 16 bytes of the window row from
    // its 4-byte-aligned start (sh = that alignment).  Tiled levels (TB, blur2_tile's layout:
    // 16 x 8-px tiles of 128 bytes, tile rows 8 * pitch apart): lane (pr, pc) loads row pr of
    // the window's tile column pc -- 16 bytes of one tile -- so the 37 rows touch about 19
    // cache lines instead of about 50 (the loads' cost follows the lines an instruction
    // touches, hit or miss: profiles/r06p_orient_load_exp.txt, r06q_orient_a2_ab.txt); sh = the
    // window's column inside its first tile, and when sh >= 12 the window's last bytes lie in
    // a fourth tile column: one more dword per row (d3, lanes < 37).
    struct Nbhd {
        uint4 v0, v1;
        uint32_t d3;
        int sh;
    };
    auto tile_row = [](const uint8_t *lvb, int pitch, int y, int tcol) -> const uint8_t * {
        return lvb + (int64_t)(y >> 3) * (8 * pitch) + tcol * 128 + (y & 7) * 16;
    };
    auto load_nbhd = [&](int j) -> Nbhd {
        const int bpitch = __builtin_amdgcn_readlane(bpitch_l, j);
        const uint8_t *bl0 = blur + readlane64(boff_l, j);
        Nbhd n;
        if (TB) {
            const int bxy = __builtin_amdgcn_readlane(bxy_l, j);
            const int wx = bxy & 0xFFFF, wy = bxy >> 16;
            n.sh = wx & 15;
            const int tc = wx >> 4;
            n.v0 = *(const uint4 *)tile_row(bl0, bpitch, wy + pr[0], tc + pc[0]);
            n.v1 = *(const uint4 *)tile_row(bl0, bpitch, wy + pr[1], tc + pc[1]);
            n.d3 = 0;
            if (n.sh >= 12 && lane < OD_SPAN)  // wave-uniform slot test, then the 37 row lanes
                n.d3 = *(const uint32_t *)tile_row(bl0, bpitch, wy + lane, tc + 3);
        } else {
            n.sh = (int)((uintptr_t)bl0 & 3);
            const uint8_t *bw = bl0 - n.sh;
            n.v0 = *(const uint4 *)(bw + (int64_t)pr[0] * bpitch + 16 * pc[0]);
            n.v1 = *(const uint4 *)(bw + (int64_t)pr[1] * bpitch + 16 * pc[1]);
            n.d3 = 0;
        }
        return n;
    };
    Nbhd nbh[OD_PFD + 1];
    // ---- A: IC_Angle moments (ORBextractor.cc:83-111), slot j's sums kept by lane j ----
    // Software-pipelined over the slots: the patch loads of slot j + 1 are in flight while
    // slot j's moments are summed (the kernel is bound by the latency of these scattered row
    // loads, not by issue); two register buffers alternate.
    auto load_patch = [&](int j, uint4 (&wd)[2], int (&sh)[2]) {
        const int lev = __builtin_amdgcn_readlane(lev_l, j);
        const int pitch = __builtin_amdgcn_readlane(ppitch_l, j);
        const uint8_t *ctr = (lev == 0 ? img0 : pyr) + readlane64(poff_l, j);
        // 16 bytes per lane from each row's 4-byte-aligned start (the level-0 pitch may be
        // odd, so the alignment is per row)
#pragma unroll
        for (int k = 0; k < 2; k++) {
            // pointer arithmetic (not an integer round trip): global_, not flat_, loads
            const uint8_t *pa = ctr + (int64_t)(par[k] - ORBG_HALF_PATCH) * pitch - ORBG_HALF_PATCH;
            sh[k] = (int)((uintptr_t)pa & 3);
            wd[k] = *(const uint4 *)(pa - sh[k] + 16 * pac[k]);
        }
    };
    int M01 = 0, M10 = 0;
    {
        uint4 wbuf[OD_PFD + 1][2];
        int sbuf[OD_PFD + 1][2];
#pragma unroll
        for (int j = 0; j < OD_PFD; j++) load_patch(j, wbuf[j], sbuf[j]);
#pragma unroll
        for (int j = 0; j < OD_KPW; j++) {
            if (j + OD_PFD < OD_KPW)
                load_patch(j + OD_PFD, wbuf[(j + OD_PFD) % (OD_PFD + 1)], sbuf[(j + OD_PFD) % (OD_PFD + 1)]);
            // phase C's first ORBG_OD_EARLYC neighbourhoods, issued in A's last slots
            if (j >= OD_KPW - ORBG_OD_EARLYC) nbh[j - (OD_KPW - ORBG_OD_EARLYC)] = load_nbhd(j - (OD_KPW - ORBG_OD_EARLYC));
            const uint4(&wd)[2] = wbuf[j % (OD_PFD + 1)];
            const int(&sh)[2] = sbuf[j % (OD_PFD + 1)];
            int m01 = 0, m10 = 0;
#pragma unroll
            for (int k = 0; k < 2; k++) {
                const int w = lane + 64 * k;
                if (w < OD_TABW) {
                    const int v = par[k] - ORBG_HALF_PATCH;
                    const uint4 tw = tab[(2 * sh[k]) * OD_TABW + w];
                    const uint4 to = tab[(2 * sh[k] + 1) * OD_TABW + w];
                    uint32_t su = 0, sv = 0;
                    su = __builtin_amdgcn_udot4(wd[k].x, tw.x, su, false);
                    su = __builtin_amdgcn_udot4(wd[k].y, tw.y, su, false);
                    su = __builtin_amdgcn_udot4(wd[k].z, tw.z, su, false);
                    su = __builtin_amdgcn_udot4(wd[k].w, tw.w, su, false);
                    sv = __builtin_amdgcn_udot4(wd[k].x, to.x, sv, false);
                    sv = __builtin_amdgcn_udot4(wd[k].y, to.y, sv, false);
                    sv = __builtin_amdgcn_udot4(wd[k].z, to.z, sv, false);
                    sv = __builtin_amdgcn_udot4(wd[k].w, to.w, sv, false);
                    m10 += (int)su - ORBG_HALF_PATCH * (int)sv;
                    m01 += v * (int)sv;
                }
            }
            m01 = wave_sum(m01);
            m10 = wave_sum(m10);
            if (lane == j) {
                M01 = m01;
                M10 = m10;
            }
        }
    }

    if (g->dbg == 21) {  // developer phase timing (ORBG_DBG, dev builds): stop after A
        // keep the sums live without a store per wave to one address (that alone would
        // serialise): lane j's sums into its own slot's descriptor row
        if (my_ok) ((int *)(desc + (drow0 + my_i) * 32))[0] = M01 + M10;
        return;
    }
    // ---- B: angle = fastAtan2(m_01, m_10) (:110), cos / sin of it (:121-122), and the
    // keypoint record (:1115-1122, :1387-1393), lane j for slot j ----
    const float factorPI = (float)(3.14159265358979323846 / 180.f);
    const float angle_l = fast_atan2((float)M01, (float)M10);
    float a_l, b_l;
    if (g->sincos_mode == 0) {  // glibc cosf / sinf (the reference's libm), default
        glibc_sincosf(angle_l * factorPI, &b_l, &a_l);
    } else {                    // round 1's correctly rounded double evaluation
        double sd, cd;
        pinned_sincos((double)(angle_l * factorPI), &sd, &cd);
        a_l = (float)cd;
        b_l = (float)sd;
    }
    if (my_ok) {
        const OrbgLevel &lv = g->lv[my_lev];
        OrbgKeypointDev kp;
        float fx = (float)(orbg_px(kl) + ORBG_MIN_BORDER), fy = (float)(orbg_py(kl) + ORBG_MIN_BORDER);
        if (my_lev != 0) {
            fx *= lv.scale;
            fy *= lv.scale;
        }
        kp.x = fx;
        kp.y = fy;
        kp.size = (float)lv.patch_size;
        kp.angle = angle_l;
        kp.response = (float)orbg_ps(kl);
        kp.octave = my_lev;
        kp.class_id = -1;
        kps[(int64_t)f * g->frame_cap + my_i] = kp;
        if (HC) ((OrbgKeypointDev *)(hc.base + hc.okp))[my_i] = kp;
    }

    if (g->dbg == 22) return;  // developer phase timing: stop after B
    // ---- C: rBRIEF (ORBextractor.cc:117-157) on the blurred level ----
    // lane L owns tests L + 64t (t = 0..3), one pattern word (x0, y0, x1, y1) each
    int pat[4];
#pragma unroll
    for (int t = 0; t < 4; t++) pat[t] = ((const int *)od_pattern_i8)[lane + 64 * t];
    uint8_t *bp = (uint8_t *)bpatch[wv];
    // pipelined like phase A: slot j + 1's neighbourhood loads are issued right after slot j
    // is staged, and land while slot j's samples are read
#pragma unroll
    for (int j = ORBG_OD_EARLYC; j < OD_PFD; j++) nbh[j] = load_nbhd(j);
#pragma unroll
    for (int j = 0; j < OD_KPW; j++) {
        constexpr int ROWB = TB ? OD_ROWB_T : OD_ROWB;
        wave_sync_lds();  // the previous slot's sample reads are done
        {
            const Nbhd &n = nbh[j % (OD_PFD + 1)];
            if (TB) {  // 52-byte rows: 4-byte aligned dword stores (ds_write2_b32)
                uint32_t *r0 = (uint32_t *)(bp + pr[0] * ROWB + 16 * pc[0]);
                uint32_t *r1 = (uint32_t *)(bp + pr[1] * ROWB + 16 * pc[1]);
                r0[0] = n.v0.x, r0[1] = n.v0.y, r0[2] = n.v0.z, r0[3] = n.v0.w;
                r1[0] = n.v1.x, r1[1] = n.v1.y, r1[2] = n.v1.z, r1[3] = n.v1.w;
                if (n.sh >= 12 && lane < OD_SPAN) {  // a fresh address: no VGPR held (spill)
                    int la = lane * ROWB + 48;
                    asm volatile("" : "+v"(la));
                    *(uint32_t *)(bp + la) = n.d3;
                }
            } else {
                *(uint4 *)(bp + pr[0] * ROWB + 16 * pc[0]) = n.v0;
                *(uint4 *)(bp + pr[1] * ROWB + 16 * pc[1]) = n.v1;  // clamped lanes: same word twice
            }
        }
        wave_sync_lds();
        const int cur_bsh = nbh[j % (OD_PFD + 1)].sh;
        if (j + OD_PFD < OD_KPW) nbh[(j + OD_PFD) % (OD_PFD + 1)] = load_nbhd(j + OD_PFD);
        const float a = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, a_l), j));
        const float b = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, b_l), j));
        // cvRound (round half to even) by the 1.5 * 2^23 shift: the float sum rounds r to an
        // integer, ties to even, so bits(r + M) = 0x4B400000 + cvRound(r) for |r| < 2^22 and its
        // low 24 bits are 2^22 + cvRound(r); one v_mad_u32_u24 then gives
        // ROWB (2^22 + ry) + bits(rx + M) = ry * ROWB + rx + MK (mod 2^32), and the centre's byte
        // index minus MK turns that into the sample's index in the staged neighbourhood
        constexpr float M = 12582912.0f;
        constexpr uint32_t MK = (uint32_t)ROWB * 0x400000u + 0x4B400000u;
        const uint32_t cbase = (uint32_t)(OD_R * ROWB + cur_bsh + OD_R) - MK;
        // opaque per slot: keeps the offset decode inside the loop (hoisted, the 16 floats
        // stay live through phase C and push the kernel past 64 VGPRs)
        int pt[4] = {pat[0], pat[1], pat[2], pat[3]};
        asm volatile("" : "+v"(pt[0]), "+v"(pt[1]), "+v"(pt[2]), "+v"(pt[3]));
        // all 8 sample offsets first, then the 8 LDS reads in flight together, then the 4
        // ballots
        int off[8];
#if ORBG_OD_PK
        // (ry, rx) as one packed pair: v_pk_mul / v_pk_add (v_pk_fma) process both lanes of a
        // pair per instruction with the scalar ops' IEEE rounding; rx = px a + py (-b) is
        // px a - py b exactly (negation is exact)
        const od_f2 ba = {b, a}, anb = {a, -b}, MM = {M, M};
#endif
#pragma unroll
        for (int t = 0; t < 4; t++) {
#pragma unroll
            for (int s = 0; s < 2; s++) {
                const float px = (float)(int8_t)(pt[t] >> (16 * s));
                const float py = (float)(int8_t)(pt[t] >> (16 * s + 8));
#if ORBG_OD_PK
                const od_f2 P = {px, px}, Q = {py, py};
                const od_f2 q = Q * anb;
                const od_f2 r = (BFMA ? __builtin_elementwise_fma(P, ba, q) : P * ba + q) + MM;
                // the elements through float copies: __builtin_bit_cast of a vector element
                // (r.y) reads element 0 with this clang
                const float ryM = r.x, rxM = r.y;
                const uint32_t iy = __builtin_bit_cast(uint32_t, ryM);
                const uint32_t ix = __builtin_bit_cast(uint32_t, rxM);
#else
                const float t0 = px * b, t1 = py * a, t2 = px * a, t3 = py * b;
                const float ry = BFMA ? fmaf(px, b, t1) : t0 + t1;
                const float rx = BFMA ? fmaf(px, a, -t3) : t2 - t3;
                const uint32_t iy = __builtin_bit_cast(uint32_t, ry + M);
                const uint32_t ix = __builtin_bit_cast(uint32_t, rx + M);
#endif
                off[2 * t + s] = (int)((iy & 0xFFFFFFu) * (uint32_t)ROWB + ix + cbase);
            }
        }
        int val[8];
#pragma unroll
        for (int i = 0; i < 8; i++) val[i] = bp[off[i]];
        uint32_t word = 0;
#pragma unroll
        for (int t = 0; t < 4; t++) {
            // bit L of ballot t = test 64t + L = descriptor bit 64t + L; dword d of the
            // descriptor is half (d & 1) of ballot d >> 1
            const unsigned long long m = __ballot(val[2 * t] < val[2 * t + 1]);
            if ((lane >> 1) == t) word = (uint32_t)(m >> (32 * (lane & 1)));
        }
        const int i = __builtin_amdgcn_readlane(my_i, j);
        if (((okmask >> j) & 1u) && lane < 8) {
            // the row address is scalar and the lane's byte offset a fresh 32-bit value
            // (global_store with saddr): a hoisted 64-bit per-lane pointer would hold two
            // VGPRs across the slot loop -- spilled at 64, and each reload's vmcnt(0) wait
            // drained the next slots' prefetched neighbourhoods
            int lo = lane * 4;
            asm volatile("" : "+v"(lo));
            *(uint32_t *)(desc + (drow0 + i) * 32 + lo) = word;
            if (HC) *(uint32_t *)(hc.base + hc.ods + (int64_t)i * 32 + lo) = word;
        }
    }
}

hipError_t launch_orient_desc(bool bfma, bool tiled, dim3 grid, hipStream_t st, const OrbgGeom *g,
                              const uint8_t *img0, int64_t img_fs, int img_pitch,
                              const uint8_t *pyr, const uint8_t *blur, const uint4 *odtab,
                              const uint32_t *lvl_kp, const uint16_t *lvl_idx,
                              const int32_t *lvl_cnt, OrbgKeypointDev *kps, uint8_t *desc,
                              int32_t *counts, uint8_t *hc_base, const int32_t *hc_err,
                              size_t hc_okp, size_t hc_ods, int32_t hc_tag)
{
    const OdHostCopy hc{hc_base, hc_err, (int32_t)hc_okp, (int32_t)hc_ods, hc_tag};
#define OD_LAUNCH(BF, H, T)                                                                    \
    hipLaunchKernelGGL((k_orient_desc<BF, H, T>), grid, dim3(256), 0, st, g, img0, img_fs,     \
                       img_pitch, pyr, blur, odtab, lvl_kp, lvl_idx, lvl_cnt, kps, desc, counts, \
                       hc)
#define OD_LAUNCH_T(BF, H)          \
    if (tiled) OD_LAUNCH(BF, H, true); \
    else OD_LAUNCH(BF, H, false)
    if (hc_base) {
        if (bfma) OD_LAUNCH_T(true, true);
        else OD_LAUNCH_T(false, true);
    } else {
        if (bfma) OD_LAUNCH_T(true, false);
        else OD_LAUNCH_T(false, false);
    }
#undef OD_LAUNCH_T
#undef OD_LAUNCH
    return hipGetLastError();
}

}  // namespace orbg
