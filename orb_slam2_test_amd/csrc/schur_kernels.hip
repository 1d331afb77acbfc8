// schur_kernels.hip -- g2o BlockSolver<6,3>::solve with the Schur complement
// (Thirdparty/g2o/g2o/core/block_solver.hpp:354-486) for LocalBundleAdjustment windows, on
// gfx950, fp64.  Inputs are the linearisation's blocks (H_pp, b_p per pose; H_ll, b_l per
// point; H_pl per edge) after setLambda(lambda); outputs the pose and point increments.  The
// structure is a SchurPlanHost built once per graph (schur_args.h), so an LM iteration's
// build -> errors -> solve runs on one stream with no host copy (orbg_ba_graph_schur_solve).
//
//   k_schur_points   thread per active edge (point-major slot): D^-1 = (H_ll + lambda I)^-1
//                    (Eigen's cofactor 3x3 inverse), D^-1 b_l, and for an edge to a free
//                    pose B D^-1 (6x3) and B D^-1 b_l (6), stored by slot, coalesced
//   k_schur_blocks   workgroup per upper block (i1 <= i2): S = H_pp + lambda I (diagonal
//                    blocks) minus sum B_i D^-1 B_j^T over its landmark pairs, one
//                    v_mfma_f64_4x4x4f64 per pair (the 6x6 block padded to the 8x8 of the
//                    instruction's four 4x4 blocks, K = the 3 inner terms + a zero), pair t
//                    into accumulator chain t % 16 = wave t % 16 of the workgroup, the chains
//                    combined by a pairwise tree; written upper + mirrored into the
//                    segment's dense system
//   k_schur_rhs      wave per free pose: b_schur = b_p - sum B D^-1 b_l over its landmarks
//                    (64 lane partials in list order, xor butterfly)
//   k_schur_ldlt     workgroup per segment: right-looking dense LDLT (no pivoting; each
//                    element's updates in k order: the left-looking oracle's bits) and the
//                    two triangular solves column by column, in LDS when it fits
//   k_schur_backsub  thread per landmark: x_l = D^-1 (b_l - B^T x_p)
// Every sum runs in the order oracle/ba_oracle.c (orc_ba_schur_solve) pins -- including the
// MFMA's own: a fused chain over k in order (tools/microbench/mfma_f64_pin.hip) -- so the
// increments are bit-identical to it.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>

#include "../../include/orbg.h"
#include "orbg_device.h"
#include "schur_args.h"

#pragma clang fp contract(off)

namespace orbg {

void prof_begin(void *prof, hipStream_t s, const char *n, hipEvent_t *a);
void prof_end(void *prof, hipStream_t s, const char *n, hipEvent_t a);

// (H_ll + lambda I)^-1 by Eigen's cofactor 3x3 inverse (orc inv3_eigen) and D^-1 b_l
__device__ __forceinline__ void schur_dinv(const SchurArgs &A, int p, double d[9], double db[3])
{
    double m[9];
    for (int k = 0; k < 9; k++) m[k] = A.hpoint[9 * (size_t)p + k];
    m[0] += A.lambda;
    m[4] += A.lambda;
    m[8] += A.lambda;
#define M(i, j) m[(i) * 3 + (j)]
#define COF(i, j) (M(((i) + 1) % 3, ((j) + 1) % 3) * M(((i) + 2) % 3, ((j) + 2) % 3) - \
                   M(((i) + 1) % 3, ((j) + 2) % 3) * M(((i) + 2) % 3, ((j) + 1) % 3))
    const double c0 = COF(0, 0), c1 = COF(1, 0), c2 = COF(2, 0);
    const double det = (c0 * M(0, 0) + c1 * M(1, 0)) + c2 * M(2, 0);
    const double invdet = 1.0 / det;
    d[0] = c0 * invdet;
    d[1] = c1 * invdet;
    d[2] = c2 * invdet;
    d[3] = COF(0, 1) * invdet;
    d[4] = COF(1, 1) * invdet;
    d[5] = COF(2, 1) * invdet;
    d[6] = COF(0, 2) * invdet;
    d[7] = COF(1, 2) * invdet;
    d[8] = COF(2, 2) * invdet;
#undef COF
#undef M
    const double *bl = A.bpoint + 3 * (size_t)p;
    for (int r = 0; r < 3; r++) db[r] = (d[r * 3] * bl[0] + d[r * 3 + 1] * bl[1]) + d[r * 3 + 2] * bl[2];
}

// thread per slot (active edge, point-major): the point's D^-1 recomputed (a few dozen flops;
// no per-point array), then for an edge to a free pose the record B D^-1 (6x3) | B D^-1 b_l
// (6); the workgroup's 256 records are staged in LDS and stored as one contiguous 48 KB run
#define SCHUR_REC 24
__global__ __launch_bounds__(256) void k_schur_points(SchurArgs A)
{
    __shared__ double2 rec[256 * SCHUR_REC / 2];
    const int tid = threadIdx.x, base = blockIdx.x * 256, a = base + tid;
    if (a == 0) *A.ok = 1;  // k_schur_ldlt clears it on a bad pivot (stream order)
    // the dense systems zeroed here (block pairs without a shared landmark are never written
    // by k_schur_blocks): no separate fill launch
    for (int64_t z = a; z < A.s_total; z += (int64_t)gridDim.x * 256) A.S[z] = 0.0;
    double v[SCHUR_REC];
#pragma unroll
    for (int k = 0; k < SCHUR_REC; k++) v[k] = 0.0;
    const int fi = a < A.nslot ? A.slot_fidx[a] : -1;
    if (fi >= 0) {
        const int e = A.pt_edges[a];
        {
            double d[9], db[3];
            schur_dinv(A, A.slot_point[a], d, db);
            const double *h = A.hpl + (size_t)e * A.hpl_stride;  // B = h^T (6 x 3), h[k][r] = h[6k + r]
            double hh[18];
#pragma unroll
            for (int k = 0; k < 18; k++) hh[k] = h[k];
#pragma unroll
            for (int r = 0; r < 6; r++) {
#pragma unroll
                for (int c = 0; c < 3; c++)
                    v[r * 3 + c] = (hh[r] * d[c] + hh[6 + r] * d[3 + c]) + hh[12 + r] * d[6 + c];
                v[18 + r] = (hh[r] * db[0] + hh[6 + r] * db[1]) + hh[12 + r] * db[2];
            }
        }
    }
    // (the record in registers, staged as double2: 150 VGPRs; writing rows straight to LDS
    // as doubles, ~80 VGPRs, measured slower: 0.105 against 0.085 ms, r05l)
#pragma unroll
    for (int k = 0; k < SCHUR_REC; k += 2) rec[tid * (SCHUR_REC / 2) + k / 2] = make_double2(v[k], v[k + 1]);
    // records of edges to fixed poses are never read (k_schur_blocks / k_schur_rhs take free
    // poses' slots only): not stored
    __shared__ uint8_t keep[256];
#ifdef SCHUR_KEEP_ALL  // A/B: every record stored
    keep[tid] = 1;
#else
    keep[tid] = fi >= 0;
#endif
    __syncthreads();
    const int nrec = min(256, A.nslot - base);
    double2 *out = (double2 *)(A.rec + (size_t)base * SCHUR_REC);
    for (int i = tid; i < nrec * (SCHUR_REC / 2); i += 256)
        if (keep[i / (SCHUR_REC / 2)]) out[i] = rec[i];
}

// workgroup per upper block, wave u = accumulator chain u: the block's pairs t = u, u + 16, ...
// (landmark order) by one v_mfma_f64_4x4x4f64 each into that wave's chain (16 chains: a
// diagonal block sums every landmark of its pose, ~3000 in a KITTI window, so its gathers
// need that many waves in flight), the chains combined by a pairwise tree through LDS.  Operand layout of the instruction
// (ba_kernels.hip): A[b][i][k] at lane 16k + 4b + i, B[b][k][j] at lane 16k + 4b + j,
// C[b][i][j] at lane 16i + 4b + j; block b = 2I + J holds rows 4I + i, columns 4J + j of the
// padded 8x8.  A = -B D^-1 of the pair's first edge (6x3, k = its column), B = H_pl of the
// second (3x6, k = its row).
#ifndef ORBG_SCHUR_XCD
#define ORBG_SCHUR_XCD 1
#endif
#define SCHUR_CHAINS 16
#ifndef SCHUR_BATCH
#define SCHUR_BATCH 11  // pairs per step and chain (11: 62 VGPRs, two 16-wave workgroups per CU; 16: 82)
#endif  // waves per block workgroup = accumulator chains (the oracle's)
__global__ __launch_bounds__(64 * SCHUR_CHAINS) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_schur_blocks(SchurArgs A)
{
    __shared__ double tile[SCHUR_CHAINS][64];
    // XCD-aware: consecutive blocks (one window's, sorted by segment) share an XCD's L2, so a
    // window's records and H_pl are fetched into one L2 rather than into all eight
    const int lane = threadIdx.x & 63, u = threadIdx.x >> 6,
              bk = A.blk_order[ORBG_SCHUR_XCD ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x];
    const int i1 = A.blk_i1[bk], i2 = A.blk_i2[bk], sg = A.blk_seg[bk];
    const int lo = A.seg_lo[sg], n = 6 * (A.seg_lo[sg + 1] - lo);
    const int k = lane >> 4, b = (lane >> 2) & 3, t = lane & 3;
    const int ra = 4 * (b >> 1) + t, cb = 4 * (b & 1) + t;  // A's row, B's column
    const bool va = ra < 6 && k < 3, vb = k < 3 && cb < 6;
    const int oa = ra * 3 + k, ob = 6 * k + cb;
    const int ro = 4 * (b >> 1) + k, co = 4 * (b & 1) + t;  // this lane's C entry (i = lane >> 4)
    double c = 0.0;
    if (u == 0 && i1 == i2 && ro < 6 && co < 6)
        c = A.hpose[36 * (size_t)A.free_pose[i1] + 6 * ro + co] + (ro == co ? A.lambda : 0.0);
    const int p0 = A.blk_off[bk], np = A.blk_off[bk + 1] - p0;
    const int nu = np > u ? (np - u + SCHUR_CHAINS - 1) / SCHUR_CHAINS : 0;  // p0 + u + 16 j
    // SCHUR_BATCH pairs per step: lane l < SCHUR_BATCH holds pair j0 + l's ids, the wave takes
    // them by readlane, so all 2 SCHUR_BATCH operand loads of the step are in flight together;
    // the next step's ids are loaded during this step's gathers.  Every load is unconditional
    // (clamped pair / entry, the value then selected away), so the waits before the MFMAs
    // leave the ids of the next step in flight.
    const int oac = va ? oa : 0, obc = vb ? ob : 0;
    auto ids = [&](int j) -> int2 {
        return A.blk_pairs[p0 + u + SCHUR_CHAINS * min(j + lane, nu - 1)];
    };
    int2 prl = nu > 0 ? ids(0) : make_int2(0, 0);
    for (int j0 = 0; j0 < nu; j0 += SCHUR_BATCH) {
        const int m = min(SCHUR_BATCH, nu - j0);
        double av[SCHUR_BATCH], bv[SCHUR_BATCH];
#pragma unroll
        for (int q = 0; q < SCHUR_BATCH; q++) {
            const int s1 = __builtin_amdgcn_readlane(prl.x, q), e2 = __builtin_amdgcn_readlane(prl.y, q);
            av[q] = A.rec[(size_t)s1 * SCHUR_REC + oac];
            bv[q] = A.hpl[(size_t)e2 * A.hpl_stride + obc];
        }
        const int2 nxt = j0 + SCHUR_BATCH < nu ? ids(j0 + SCHUR_BATCH) : prl;
#pragma unroll
        for (int q = 0; q < SCHUR_BATCH; q++)
            if (q < m)
                c = __builtin_amdgcn_mfma_f64_4x4x4f64(va ? -av[q] : 0.0, vb ? bv[q] : 0.0, c, 0, 0, 0);
        prl = nxt;
    }
    tile[u][lane] = c;
    __syncthreads();
    if (u != 0) return;
    // the chains' pairwise tree (oracle schur_tree16)
    double a8[8], b4[4];
#pragma unroll
    for (int i = 0; i < 8; i++) a8[i] = tile[2 * i][lane] + tile[2 * i + 1][lane];
#pragma unroll
    for (int i = 0; i < 4; i++) b4[i] = a8[2 * i] + a8[2 * i + 1];
    const double v = (b4[0] + b4[1]) + (b4[2] + b4[3]);
    if (ro < 6 && co < 6) {
        double *S = A.S + A.seg_soff[sg];
        const int r = 6 * (i1 - lo) + ro, cc = 6 * (i2 - lo) + co;
        if (i1 != i2 || ro <= co) S[(size_t)r * n + cc] = v;  // upper
        if (i1 != i2 || ro < co) S[(size_t)cc * n + r] = v;   // lower = mirror of the upper
    }
}

// k_schur_blocks with its operands staged: the same chains, pairs and MFMAs (so the same
// bits), but a batch's SCHUR_SBATCH B D^-1 records (the first 18 doubles of a slot's record)
// and H_pl blocks (18 doubles) are fetched as whole 16-byte pieces -- 9 per block, one per
// lane, 2 x 9 x SCHUR_SBATCH pieces in ceil(18 SCHUR_SBATCH / 64) load instructions -- into
// the wave's own LDS region, and the MFMA operands are read from there.  The gather version
// issues two 64-lane loads of 8 bytes per pair (each touching a 192- and a 144-byte block);
// this one about a quarter as many vector-memory instructions, with the next batch's pieces
// in flight (registers) while the current batch's MFMAs run.
#ifndef SCHUR_SBATCH
#define SCHUR_SBATCH 7  // pairs per batch: 2 x 9 x 7 = 126 pieces = 2 loads of 64 lanes (14: 4 loads, +5%; 21: +16%, r06c)
#endif
#define SCHUR_SPIECES (2 * 9 * SCHUR_SBATCH)
#define SCHUR_SLOADS ((SCHUR_SPIECES + 63) / 64)
__global__ __launch_bounds__(64 * SCHUR_CHAINS) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_schur_blocks_lds(SchurArgs A)
{
    __shared__ double tile[SCHUR_CHAINS][64];
    __shared__ double2 stage[SCHUR_CHAINS][SCHUR_SPIECES];
    const int lane = threadIdx.x & 63, u = threadIdx.x >> 6,
              bk = A.blk_order[ORBG_SCHUR_XCD ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x];
    const int i1 = A.blk_i1[bk], i2 = A.blk_i2[bk], sg = A.blk_seg[bk];
    const int lo = A.seg_lo[sg], n = 6 * (A.seg_lo[sg + 1] - lo);
    const int k = lane >> 4, b = (lane >> 2) & 3, t = lane & 3;
    const int ra = 4 * (b >> 1) + t, cb = 4 * (b & 1) + t;  // A's row, B's column
    const bool va = ra < 6 && k < 3, vb = k < 3 && cb < 6;
    const int oa = va ? ra * 3 + k : 0, ob = vb ? 6 * k + cb : 0;
    const int ro = 4 * (b >> 1) + k, co = 4 * (b & 1) + t;  // this lane's C entry (i = lane >> 4)
    double c = 0.0;
    if (u == 0 && i1 == i2 && ro < 6 && co < 6)
        c = A.hpose[36 * (size_t)A.free_pose[i1] + 6 * ro + co] + (ro == co ? A.lambda : 0.0);
    const int p0 = A.blk_off[bk], np = A.blk_off[bk + 1] - p0;
    const int nu = np > u ? (np - u + SCHUR_CHAINS - 1) / SCHUR_CHAINS : 0;  // p0 + u + 16 j
    // piece c of a batch: c < 9 B: the A block of pair c / 9, else the B block of pair
    // (c - 9 B) / 9; piece c % 9 of it (16 bytes).  Pairs past the chain's end are clamped
    // (the MFMA skips them).
    const double2 *recp = (const double2 *)A.rec, *hplp = (const double2 *)A.hpl;
    const int hstride2 = A.hpl_stride / 2;  // 16-byte pieces per H_pl row (hpl_stride even)
    auto fetch = [&](int j0, double2 (&v)[SCHUR_SLOADS]) {
        // this lane's pairs' ids: lane q < SCHUR_SBATCH holds pair j0 + q
        const int2 id = nu > 0 ? A.blk_pairs[p0 + u + SCHUR_CHAINS * min(j0 + min(lane, SCHUR_SBATCH - 1), nu - 1)]
                               : make_int2(0, 0);
#pragma unroll
        for (int i = 0; i < SCHUR_SLOADS; i++) {
            const int pc = lane + 64 * i;
            const bool isb = pc >= 9 * SCHUR_SBATCH;
            const int rel = isb ? pc - 9 * SCHUR_SBATCH : pc;
            const int q = min(rel / 9, SCHUR_SBATCH - 1), part = rel - 9 * (rel / 9);
            const int s1 = __shfl(id.x, q, 64), e2 = __shfl(id.y, q, 64);
            const double2 *src = isb ? hplp + (size_t)e2 * hstride2 + part
                                     : recp + (size_t)s1 * (SCHUR_REC / 2) + part;
            v[i] = (pc < SCHUR_SPIECES) ? *src : make_double2(0.0, 0.0);
        }
    };
    double2 cur[SCHUR_SLOADS];
    if (nu > 0) fetch(0, cur);
    const double *sd = (const double *)stage[u];
    for (int j0 = 0; j0 < nu; j0 += SCHUR_SBATCH) {
        const int m = min(SCHUR_SBATCH, nu - j0);
#pragma unroll
        for (int i = 0; i < SCHUR_SLOADS; i++) {
            const int pc = lane + 64 * i;
            if (pc < SCHUR_SPIECES) stage[u][pc] = cur[i];
        }
        wave_sync_lds();
        if (j0 + SCHUR_SBATCH < nu) fetch(j0 + SCHUR_SBATCH, cur);  // in flight during the MFMAs
#pragma unroll
        for (int q = 0; q < SCHUR_SBATCH; q++)
            if (q < m) {
                const double av = sd[18 * q + oa], bv = sd[18 * (SCHUR_SBATCH + q) + ob];
                c = __builtin_amdgcn_mfma_f64_4x4x4f64(va ? -av : 0.0, vb ? bv : 0.0, c, 0, 0, 0);
            }
        wave_sync_lds();  // every lane's reads of this batch before the next batch's writes
    }
    tile[u][lane] = c;
    __syncthreads();
    if (u != 0) return;
    double a8[8], b4[4];
#pragma unroll
    for (int i = 0; i < 8; i++) a8[i] = tile[2 * i][lane] + tile[2 * i + 1][lane];
#pragma unroll
    for (int i = 0; i < 4; i++) b4[i] = a8[2 * i] + a8[2 * i + 1];
    const double v = (b4[0] + b4[1]) + (b4[2] + b4[3]);
    if (ro < 6 && co < 6) {
        double *S = A.S + A.seg_soff[sg];
        const int r = 6 * (i1 - lo) + ro, cc = 6 * (i2 - lo) + co;
        if (i1 != i2 || ro <= co) S[(size_t)r * n + cc] = v;
        if (i1 != i2 || ro < co) S[(size_t)cc * n + r] = v;
    }
}

// b_schur = b_p - coefficients, per free pose: the landmark-ordered B D^-1 b_l terms summed
// as 64 lane partials (term t into partial t % 64, in order) and an xor butterfly
__device__ __forceinline__ void schur_rhs_wave(const SchurArgs &A, int i, int lane)
{
    if (i >= A.nfree) return;
    const int pose = A.free_pose[i], e0 = A.pose_off[i], e1 = A.pose_off[i + 1];
    double part[6] = {0, 0, 0, 0, 0, 0};
    // all six partials per step, four list entries per lane in flight (each partial still
    // adds its entries t = lane, lane + 64, ... in order)
    int t = e0 + lane;
    for (; t + 192 < e1; t += 256) {
        int sl[4];
#pragma unroll
        for (int q = 0; q < 4; q++) sl[q] = A.pose_slots[t + 64 * q];
        double v[4][6];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const double2 *cf = (const double2 *)(A.rec + (size_t)sl[q] * SCHUR_REC + 18);
            const double2 x0 = cf[0], x1 = cf[1], x2 = cf[2];
            v[q][0] = x0.x; v[q][1] = x0.y; v[q][2] = x1.x; v[q][3] = x1.y; v[q][4] = x2.x; v[q][5] = x2.y;
        }
#pragma unroll
        for (int q = 0; q < 4; q++)
#pragma unroll
            for (int r = 0; r < 6; r++) part[r] += v[q][r];
    }
    for (; t < e1; t += 64) {
        const double *cf = A.rec + (size_t)A.pose_slots[t] * SCHUR_REC + 18;
#pragma unroll
        for (int r = 0; r < 6; r++) part[r] += cf[r];
    }
#pragma unroll
    for (int r = 0; r < 6; r++) {
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) part[r] = part[r] + __shfl_xor(part[r], off, 64);
    }
    if (lane < 6) {
        double pr = part[0];
#pragma unroll
        for (int r = 1; r < 6; r++) pr = lane == r ? part[r] : pr;
        A.x[6 * i + lane] = A.bpose[6 * (size_t)pose + lane] - pr;
    }
}

__global__ __launch_bounds__(256) void k_schur_rhs(SchurArgs A)
{
    const int i = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * 4 + (threadIdx.x >> 6)));
    schur_rhs_wave(A, i, threadIdx.x & 63);
}

// one workgroup per segment: right-looking LDLT of the segment's n x n system (lower
// triangle), then L y = b (column by column), y /= d, L^T x = y (column by column, k
// descending), in LDS when LDSM (the matrix fits), else in place in HBM
template <bool LDSM>
__global__ __launch_bounds__(256) void k_schur_ldlt(SchurArgs A)
{
    extern __shared__ __attribute__((aligned(16))) double sl_lds[];
    const int sg = blockIdx.x, tid = threadIdx.x;
    const int lo = A.seg_lo[sg], n = 6 * (A.seg_lo[sg + 1] - lo);
    if (n == 0) return;  // workgroup-uniform
    double *Sg = A.S + A.seg_soff[sg], *xg = A.x + 6 * lo;
    double *M = LDSM ? sl_lds : Sg, *x = LDSM ? sl_lds + (size_t)n * n : xg;
    if (LDSM) {
        for (int e = tid; e < n * n; e += 256) M[e] = Sg[e];
        for (int e = tid; e < n; e += 256) x[e] = xg[e];
    }
    __syncthreads();
    bool bad = false;
    for (int j = 0; j < n; j++) {
        const double d = M[(size_t)j * n + j];  // every update of step k < j is in
        if (d == 0.0 || !isfinite(d)) {         // uniform: the oracle stops here, ok = 0
            bad = true;
            break;
        }
        for (int i = j + 1 + tid; i < n; i += 256) M[(size_t)i * n + j] = M[(size_t)i * n + j] / d;
        __syncthreads();
        // trailing lower triangle: M[r][c] -= (L_rj L_cj) d_j, the oracle's
        // A[i][k] * A[j][k] * A[k][k] at k = j, in k order for every element.  (One barrier
        // per column, each update dividing its two column entries itself, measured slower:
        // 0.071 against 0.061 ms, r06f: the f64 divisions)
        for (int r = j + 1 + (tid >> 4); r < n; r += 16) {
            const double lr = M[(size_t)r * n + j];
            for (int c = j + 1 + (tid & 15); c <= r; c += 16)
                M[(size_t)r * n + c] -= lr * M[(size_t)c * n + j] * d;
        }
        __syncthreads();
    }
    if (bad) {  // uniform: every thread read the same pivot
        if (tid == 0) *A.ok = 0;
        return;
    }
    if (LDSM) {
        // the triangular solves by one wave (2 n dependent steps: a wave's LDS operations
        // complete in order, so no workgroup barrier per step)
        if (tid >= 64) return;
        for (int k = 0; k < n; k++) {
            const double xk = x[k];
            for (int i = k + 1 + tid; i < n; i += 64) x[i] -= M[(size_t)i * n + k] * xk;
            wave_sync_lds();
        }
        for (int i = tid; i < n; i += 64) x[i] /= M[(size_t)i * n + i];
        wave_sync_lds();
        for (int k = n - 1; k > 0; k--) {
            const double xk = x[k];
            for (int i = tid; i < k; i += 64) x[i] -= M[(size_t)k * n + i] * xk;
            wave_sync_lds();
        }
        for (int e = tid; e < n; e += 64) xg[e] = x[e];
        return;
    }
    // L y = b: x_i -= L_ik x_k, k ascending (the oracle's row loop, element by element)
    for (int k = 0; k < n; k++) {
        const double xk = x[k];
        for (int i = k + 1 + tid; i < n; i += 256) x[i] -= M[(size_t)i * n + k] * xk;
        __syncthreads();
    }
    for (int i = tid; i < n; i += 256) x[i] /= M[(size_t)i * n + i];
    __syncthreads();
    // L^T x = y: x_i -= L_ki x_k, k descending
    for (int k = n - 1; k > 0; k--) {
        const double xk = x[k];
        for (int i = tid; i < k; i += 256) x[i] -= M[(size_t)k * n + i] * xk;
        __syncthreads();
    }
    if (LDSM)
        for (int e = tid; e < n; e += 256) xg[e] = x[e];
}

// The same factorisation and solves by ONE wave per segment, the system in LDS: a 6 n_free
// system of an LBA window (n ~ 60) gives a wave plenty of lanes per step, and a wave's LDS
// operations complete in order, so the 2 n steps need no workgroup barriers (the 256-thread
// form above pays two per column).  The trailing update walks the step's lower triangle
// flattened, 64 elements per instruction; every element still takes its updates in k order.
#ifndef ORBG_SCHUR_LDLT_WAVE
#define ORBG_SCHUR_LDLT_WAVE 0  // one wave per segment: the 8 x 8 lane grid measured 0.116 ms (r06g), the round-5 flattened walk 0.193, against 0.060 for the 256-thread form
#endif
__global__ __launch_bounds__(64) void k_schur_ldlt_wave(SchurArgs A)
{
    extern __shared__ __attribute__((aligned(16))) double sl_lds[];
    const int sg = blockIdx.x, lane = threadIdx.x;
    const int lo = A.seg_lo[sg], n = 6 * (A.seg_lo[sg + 1] - lo);
    if (n == 0) return;
    double *Sg = A.S + A.seg_soff[sg], *xg = A.x + 6 * lo;
    double *M = sl_lds, *x = sl_lds + (size_t)n * n;
    for (int e = lane; e < n * n; e += 64) M[e] = Sg[e];
    for (int e = lane; e < n; e += 64) x[e] = xg[e];
    wave_sync_lds();
    for (int j = 0; j < n; j++) {
        const double d = M[(size_t)j * n + j];
        if (d == 0.0 || !isfinite(d)) {  // uniform: the oracle stops here, ok = 0
            if (lane == 0) *A.ok = 0;
            return;
        }
        for (int i = j + 1 + lane; i < n; i += 64) M[(size_t)i * n + j] = M[(size_t)i * n + j] / d;
        wave_sync_lds();
        // the trailing lower triangle on an 8 x 8 lane grid (rows j+1+(lane>>3) step 8,
        // columns j+1+(lane&7) step 8; the round-5 flattened walk measured 0.193 ms)
        for (int r = j + 1 + (lane >> 3); r < n; r += 8) {
            const double lr = M[(size_t)r * n + j];
#pragma unroll 2
            for (int c = j + 1 + (lane & 7); c <= r; c += 8)
                M[(size_t)r * n + c] -= lr * M[(size_t)c * n + j] * d;
        }
        wave_sync_lds();
    }
    for (int k = 0; k < n; k++) {
        const double xk = x[k];
        for (int i = k + 1 + lane; i < n; i += 64) x[i] -= M[(size_t)i * n + k] * xk;
        wave_sync_lds();
    }
    for (int i = lane; i < n; i += 64) x[i] /= M[(size_t)i * n + i];
    wave_sync_lds();
    for (int k = n - 1; k > 0; k--) {
        const double xk = x[k];
        for (int i = lane; i < k; i += 64) x[i] -= M[(size_t)k * n + i] * xk;
        wave_sync_lds();
    }
    for (int e = lane; e < n; e += 64) xg[e] = x[e];
}

// x_l = D^-1 (b_l - B^T x_p); pose increments scattered out
__global__ void k_schur_backsub(SchurArgs A)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const bool ok = *A.ok != 0;
    if (t < A.npose * 6) {
        const int i = A.pidx[t / 6];
        A.dx_pose[t] = (ok && i >= 0) ? A.x[6 * i + t % 6] : 0.0;
    }
    if (t >= A.npoint) return;
    const int p = t;
    double *xl = A.dx_point + 3 * (size_t)p;
    const int a0 = A.pt_off[p], a1 = A.pt_off[p + 1];
    if (!ok || a0 == a1) {
        xl[0] = xl[1] = xl[2] = 0.0;
        return;
    }
    const double *bl = A.bpoint + 3 * (size_t)p;
    double cl[3] = {bl[0], bl[1], bl[2]};
    for (int a = a0; a < a1; a++) {
        // (slot_fidx here instead of pidx[edge_pose[e]] measured 0.0625 against 0.0597 ms, r06f)
        const int e = A.pt_edges[a], i1 = A.pidx[A.edge_pose[e]];
        if (i1 < 0) continue;
        const double *h = A.hpl + (size_t)e * A.hpl_stride;
        for (int k = 0; k < 3; k++) {
            double s = 0;
            for (int r = 0; r < 6; r++) s += h[6 * k + r] * -A.x[6 * i1 + r];
            cl[k] += s;
        }
    }
    double Di[9], db[3];
    schur_dinv(A, p, Di, db);
    for (int r = 0; r < 3; r++) xl[r] = (Di[r * 3] * cl[0] + Di[r * 3 + 1] * cl[1]) + Di[r * 3 + 2] * cl[2];
}

int launch_schur(hipStream_t st, const SchurArgs &A, void *prof)
{
    const int T = 256;
    hipEvent_t ev = nullptr;
    prof_begin(prof, st, "schur_points", &ev);
    hipLaunchKernelGGL(k_schur_points, dim3((std::max(A.nslot, 1) + T - 1) / T), dim3(T), 0, st, A);
    prof_end(prof, st, "schur_points", ev);
    if (A.nfree > 0) {
        prof_begin(prof, st, "schur_blocks", &ev);
        // ORBG_SCHUR_STAGE=0: the per-pair gather form (A/B); staging needs 16-byte H_pl rows
        static const int stage_env = getenv("ORBG_SCHUR_STAGE") ? atoi(getenv("ORBG_SCHUR_STAGE")) : 1;
        // (b_schur folded into this launch as trailing workgroups measured slower: 0.24 ms
        // against 0.110 + 0.028, r06e)
        if (stage_env && (A.hpl_stride % 2) == 0)
            hipLaunchKernelGGL(k_schur_blocks_lds, dim3(A.nblk), dim3(64 * SCHUR_CHAINS), 0, st, A);
        else
            hipLaunchKernelGGL(k_schur_blocks, dim3(A.nblk), dim3(64 * SCHUR_CHAINS), 0, st, A);
        prof_end(prof, st, "schur_blocks", ev);
        prof_begin(prof, st, "schur_rhs", &ev);
        hipLaunchKernelGGL(k_schur_rhs, dim3((A.nfree + 3) / 4), dim3(T), 0, st, A);
        prof_end(prof, st, "schur_rhs", ev);
        const int n = 6 * A.max_seg;
        const size_t lds = ((size_t)n * n + n) * sizeof(double);
        prof_begin(prof, st, "schur_ldlt", &ev);
        static const int ldlt_wave = getenv("ORBG_SCHUR_LDLT_WAVE") ? atoi(getenv("ORBG_SCHUR_LDLT_WAVE"))
                                                                    : ORBG_SCHUR_LDLT_WAVE;
        if (ldlt_wave && lds <= 160 * 1024 - 64) {
            if (lds > 64 * 1024 &&
                hipFuncSetAttribute((const void *)k_schur_ldlt_wave,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
                return ORBG_EIO;
            hipLaunchKernelGGL(k_schur_ldlt_wave, dim3(A.nseg), dim3(64), lds, st, A);
        } else if (lds <= 160 * 1024 - 64) {
            if (lds > 64 * 1024 &&
                hipFuncSetAttribute((const void *)k_schur_ldlt<true>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
                return ORBG_EIO;
            hipLaunchKernelGGL(k_schur_ldlt<true>, dim3(A.nseg), dim3(T), lds, st, A);
        } else {
            hipLaunchKernelGGL(k_schur_ldlt<false>, dim3(A.nseg), dim3(T), 0, st, A);
        }
        prof_end(prof, st, "schur_ldlt", ev);
    }
    const int m = std::max(A.npoint, A.npose * 6);
    prof_begin(prof, st, "schur_backsub", &ev);
    if (m > 0) hipLaunchKernelGGL(k_schur_backsub, dim3((m + T - 1) / T), dim3(T), 0, st, A);
    prof_end(prof, st, "schur_backsub", ev);
    return hipGetLastError() == hipSuccess ? ORBG_OK : ORBG_EIO;
}

}  // namespace orbg

namespace orbg {

// ---------------------------------------------------------------------------
// host: the solve's structure (schur_args.h), in the orders orc_ba_schur_solve pins
// ---------------------------------------------------------------------------
void build_schur_plan(int npose, int npoint, int nedge, const int32_t *epose,
                      const int32_t *epoint, const uint8_t *eactive, const uint8_t *fixed,
                      SchurPlanHost &P)
{
    P = SchurPlanHost{};
    P.npose = npose;
    P.npoint = npoint;
    P.pidx.assign(std::max(npose, 1), -1);
    for (int i = 0; i < npose; i++)
        if (!fixed[i]) {
            P.pidx[i] = P.nfree++;
            P.free_pose.push_back(i);
        }
    const int nfree = P.nfree;
    if (P.free_pose.empty()) P.free_pose.push_back(0);
    // active edges per point, ascending pose (stable: at most one edge per (pose, point))
    P.pt_off.assign(npoint + 1, 0);
    P.edge_pose.assign(std::max(nedge, 1), 0);
    for (int e = 0; e < nedge; e++) {
        P.edge_pose[e] = epose[e];
        if (eactive[e]) P.pt_off[epoint[e] + 1]++;
    }
    for (int q = 0; q < npoint; q++) P.pt_off[q + 1] += P.pt_off[q];
    P.pt_edges.assign(std::max(P.pt_off[npoint], 1), 0);
    P.slot_point.assign(std::max(P.pt_off[npoint], 1), 0);
    {
        std::vector<int32_t> fill(P.pt_off.begin(), P.pt_off.end() - 1);
        for (int e = 0; e < nedge; e++)
            if (eactive[e]) P.pt_edges[fill[epoint[e]]++] = e;
        for (int q = 0; q < npoint; q++) {
            std::stable_sort(P.pt_edges.begin() + P.pt_off[q], P.pt_edges.begin() + P.pt_off[q + 1],
                             [&](int a, int b) { return epose[a] < epose[b]; });
            for (int a = P.pt_off[q]; a < P.pt_off[q + 1]; a++) P.slot_point[a] = q;
        }
    }
    P.slot_fidx.assign(P.pt_edges.size(), -1);
    for (int a = 0; a < P.pt_off[npoint]; a++) P.slot_fidx[a] = P.pidx[epose[P.pt_edges[a]]];
    // (block, pair) in landmark order, then grouped by upper block (i1 <= i2) with a stable
    // sort: each block's pairs keep the landmark order; the free poses' edge lists likewise
    struct BP {
        int64_t key;
        int2 pr;
    };
    std::vector<BP> bps;
    std::vector<int32_t> pcount(nfree + 1, 0);
    for (int q = 0; q < npoint; q++)
        for (int a = P.pt_off[q]; a < P.pt_off[q + 1]; a++) {
            const int e1 = P.pt_edges[a], i1 = P.pidx[epose[e1]];
            if (i1 < 0) continue;
            pcount[i1 + 1]++;
            for (int b = a; b < P.pt_off[q + 1]; b++) {
                const int e2 = P.pt_edges[b], i2 = P.pidx[epose[e2]];
                if (i2 < 0) continue;
                bps.push_back(BP{(int64_t)i1 * nfree + i2, make_int2(a, e2)});
            }
        }
    for (int i = 0; i < nfree; i++)  // every diagonal block exists (H_pp + lambda I)
        bps.push_back(BP{(int64_t)i * nfree + i, make_int2(-1, -1)});
    std::stable_sort(bps.begin(), bps.end(), [](const BP &x, const BP &y) { return x.key < y.key; });
    P.blk_off.push_back(0);
    for (size_t s = 0; s < bps.size();) {
        size_t t = s;
        while (t < bps.size() && bps[t].key == bps[s].key) t++;
        P.blk_i1.push_back((int32_t)(bps[s].key / nfree));
        P.blk_i2.push_back((int32_t)(bps[s].key % nfree));
        for (size_t u = s; u < t; u++)
            if (bps[u].pr.x >= 0) P.blk_pairs.push_back(bps[u].pr);
        P.blk_off.push_back((int32_t)P.blk_pairs.size());
        s = t;
    }
    P.nblk = (int)P.blk_i1.size();
    if (P.blk_pairs.empty()) P.blk_pairs.push_back(make_int2(0, 0));
    for (int i = 0; i < nfree; i++) pcount[i + 1] += pcount[i];
    P.pose_off = pcount;
    P.pose_slots.assign(std::max(pcount[nfree], 1), 0);
    {
        std::vector<int32_t> fill(pcount.begin(), pcount.end() - 1);
        for (int q = 0; q < npoint; q++)
            for (int a = P.pt_off[q]; a < P.pt_off[q + 1]; a++) {
                const int e = P.pt_edges[a], i = P.pidx[epose[e]];
                if (i >= 0) P.pose_slots[fill[i]++] = a;
            }
    }
    // segments: connected free poses (union-find over the off-diagonal blocks, the root of a
    // component its least free index), each component's [root, max] interval, overlapping
    // intervals merged into one segment
    std::vector<int32_t> par(std::max(nfree, 1));
    for (int i = 0; i < nfree; i++) par[i] = i;
    auto find = [&](int x) {
        while (par[x] != x) x = par[x] = par[par[x]];
        return x;
    };
    for (int b = 0; b < P.nblk; b++)
        if (P.blk_i1[b] != P.blk_i2[b]) {
            const int a = find(P.blk_i1[b]), c = find(P.blk_i2[b]);
            if (a != c) par[std::max(a, c)] = std::min(a, c);
        }
    std::vector<int32_t> hi(std::max(nfree, 1), -1);
    for (int i = 0; i < nfree; i++) {
        const int r = find(i);
        hi[r] = std::max(hi[r], i);
    }
    std::vector<int32_t> seg_of(std::max(nfree, 1), 0);
    P.seg_lo.push_back(0);
    for (int i = 0, end = -1; i < nfree; i++) {
        if (find(i) == i) end = std::max(end, hi[i]);
        seg_of[i] = (int)P.seg_lo.size() - 1;
        if (i == end) P.seg_lo.push_back(i + 1);  // no open interval reaches past i: close
    }
    P.nseg = (int)P.seg_lo.size() - 1;
    P.seg_soff.assign(P.nseg + 1, 0);
    for (int s = 0; s < P.nseg; s++) {
        const int64_t n = 6 * (int64_t)(P.seg_lo[s + 1] - P.seg_lo[s]);
        P.seg_soff[s + 1] = P.seg_soff[s] + n * n;
        P.max_seg = std::max(P.max_seg, P.seg_lo[s + 1] - P.seg_lo[s]);
    }
    P.blk_seg.assign(std::max(P.nblk, 1), 0);
    for (int b = 0; b < P.nblk; b++) P.blk_seg[b] = seg_of[P.blk_i1[b]];
    // dispatch order of k_schur_blocks: segment by segment (one window's blocks on one XCD),
    // within a segment the blocks with the most pairs first (the diagonal blocks are ~4x the
    // others: longest-first keeps them off the kernel's tail); any order gives the same bits
    P.blk_order.resize(std::max(P.nblk, 1));
    for (int b = 0; b < std::max(P.nblk, 1); b++) P.blk_order[b] = b;
    std::stable_sort(P.blk_order.begin(), P.blk_order.begin() + P.nblk, [&](int a, int b) {
        if (P.blk_seg[a] != P.blk_seg[b]) return P.blk_seg[a] < P.blk_seg[b];
        return P.blk_off[a + 1] - P.blk_off[a] > P.blk_off[b + 1] - P.blk_off[b];
    });
    if (P.nblk == 0) {
        P.blk_i1.push_back(0);
        P.blk_i2.push_back(0);
    }
}

}  // namespace orbg
