// extract_kernels.hip -- ORBextractor::operator() as batched HIP kernels for gfx950.
//
// The two general-geometry stages of the extraction (one launch per stage for a whole batch
// of frames):
//   k_resize        ComputePyramid (ORBextractor.cc:1400-1443), cv::resize INTER_LINEAR 8U,
//                   one launch per level: the pyramid for scale factors k_pyramid's band
//                   plan does not cover (pyramid_kernels.hip; the plan decides)
//   k_octree        DistributeOctTree (:668-951) as a data-parallel quadtree with global
//                   scratch: one workgroup per (frame, level), for levels with more FAST
//                   candidates than k_octree_lds holds in LDS (octree_kernels.hip)
// Bit-exactness pins: no FMA contraction (-ffp-contract=off + pragma),
// cvRound = round-half-even.
#include <hip/hip_runtime.h>

#include "orbg_internal.h"
#include "orbg_device.h"

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
    uint16_t *__restrict__ lvl_idx, int32_t *__restrict__ lvl_cnt, int32_t *__restrict__ err_flag,
    int gate)
{
    // gate (pipelined batches): err_flag[2] was cleared before this batch's k_octree_lds
    // launches, which set it for every level they leave here; clear = no level to take
    if (gate && err_flag[2] == 0) return;
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
    uint16_t *oidx = lvl_idx + (int64_t)f * g->out_frame + lv.out_off;
    const int nout = min(alive, lv.out_cap);
    for (int i = tid; i < nout; i += nthr) {  // slots in list order (k_octree_lds: tile order)
        const uint32_t k = 0xFFFFFFu - (S.u.best[i] & 0xFFFFFFu);
        out[i] = keys[k];
        oidx[i] = (uint16_t)i;
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
