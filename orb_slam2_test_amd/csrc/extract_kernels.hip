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

#pragma clang fp contract(off)

namespace orbg {

__constant__ int8_t c_pattern[1024] = {
#define ORBG_PAIR(a, b, c, d) a, b, c, d,
#include "orb_pattern.inc"
#undef ORBG_PAIR
};

__device__ __forceinline__ int cv_round(float v) { return __float2int_rn(v); }

// ---------------------------------------------------------------------------
// block-wide helpers (blockDim.x == 256)
// ---------------------------------------------------------------------------
__device__ __forceinline__ int wave_incl_scan(int x)
{
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    return x;
}

__device__ __forceinline__ int wave_sum(int x)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}

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
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_resize(const uint8_t *__restrict__ src, int64_t sfs,
                                                int spitch, int sw, uint8_t *__restrict__ dst,
                                                int64_t dfs, int dpitch, int dw, int dh,
                                                const int2 *__restrict__ xtab,
                                                const int2 *__restrict__ ytab, int bulk_end)
{
    const int dx = blockIdx.x * 64 + (threadIdx.x & 63);
    const int dy = blockIdx.y * 4 + (threadIdx.x >> 6);
    const int f = blockIdx.z;
    if (dx >= dw || dy >= dh) return;
    const int2 xt = xtab[dx];
    const int2 yt = ytab[dy];
    const int sx = xt.x, sx1 = min(sx + 1, sw - 1);
    const int a0 = (int)(short)(xt.y & 0xFFFF), a1 = (int)(short)(xt.y >> 16);
    const int sy0 = yt.x & 0xFFFF, sy1 = yt.x >> 16;
    const int b0 = (int)(short)(yt.y & 0xFFFF), b1 = (int)(short)(yt.y >> 16);
    const uint8_t *s0 = src + f * sfs + (int64_t)sy0 * spitch;
    const uint8_t *s1 = src + f * sfs + (int64_t)sy1 * spitch;
    const int r0 = s0[sx] * a0 + s0[sx1] * a1;
    const int r1 = s1[sx] * a0 + s1[sx1] * a1;
    int v;
    if (dx < bulk_end) {
        const int a = ((r0 >> 4) * b0) >> 16;
        const int b = ((r1 >> 4) * b1) >> 16;
        v = (a + b + 2) >> 2;
    } else {
        v = (r0 * b0 + r1 * b1 + (1 << 21)) >> 22;
    }
    dst[f * dfs + (int64_t)dy * dpitch + dx] = (uint8_t)min(max(v, 0), 255);
}

// ---------------------------------------------------------------------------
// FAST-9 score: max(M) - 1 where M = max over the 16 contiguous 9-arcs of
// max(min d, min -d), d = centre - circle.  Equals cornerScore<16> for every
// corner and "corner at threshold th" <=> score >= th.  -1: not a corner.
// Circle offsets (x, y) of makeOffsets(16).
// ---------------------------------------------------------------------------
__device__ __forceinline__ int fast_score_lds(const uint8_t *t, int stride)
{
    const int v = t[0];
    int d[16];
    d[0] = v - t[3 * stride];
    d[1] = v - t[3 * stride + 1];
    d[2] = v - t[2 * stride + 2];
    d[3] = v - t[stride + 3];
    d[4] = v - t[3];
    d[5] = v - t[-stride + 3];
    d[6] = v - t[-2 * stride + 2];
    d[7] = v - t[-3 * stride + 1];
    d[8] = v - t[-3 * stride];
    d[9] = v - t[-3 * stride - 1];
    d[10] = v - t[-2 * stride - 2];
    d[11] = v - t[-stride - 3];
    d[12] = v - t[-3];
    d[13] = v - t[stride - 3];
    d[14] = v - t[2 * stride - 2];
    d[15] = v - t[3 * stride - 1];
    // sliding 9-window min / max over the circular sequence
    int mn2[16], mx2[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        mn2[k] = min(d[k], d[(k + 1) & 15]);
        mx2[k] = max(d[k], d[(k + 1) & 15]);
    }
    int mn4[16], mx4[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        mn4[k] = min(mn2[k], mn2[(k + 2) & 15]);
        mx4[k] = max(mx2[k], mx2[(k + 2) & 15]);
    }
    int best_pos = -1000, best_neg = 1000;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int mn9 = min(min(mn4[k], mn4[(k + 4) & 15]), d[(k + 8) & 15]);
        const int mx9 = max(max(mx4[k], mx4[(k + 4) & 15]), d[(k + 8) & 15]);
        best_pos = max(best_pos, mn9);
        best_neg = min(best_neg, mx9);
    }
    const int M = max(best_pos, -best_neg);
    return M >= 1 ? M - 1 : -1;
}

// ---------------------------------------------------------------------------
// k_fast_cells: one workgroup per (cell, frame)
// ---------------------------------------------------------------------------
#define FAST_MAXPIX (ORBG_MAX_WIN * ORBG_MAX_WIN)

__global__ __launch_bounds__(256) void k_fast_cells(const OrbgGeom *__restrict__ g,
                                                    const OrbgCell *__restrict__ cells,
                                                    const uint8_t *__restrict__ img0,
                                                    int64_t img_fs, int img_pitch,
                                                    const uint8_t *__restrict__ pyr,
                                                    int32_t *__restrict__ cell_cnt,
                                                    uint32_t *__restrict__ cell_kp)
{
    __shared__ uint8_t tile[FAST_MAXPIX];
    __shared__ int16_t sc[FAST_MAXPIX];
    __shared__ int red[8];
    const int c = blockIdx.x, f = blockIdx.y, tid = threadIdx.x;
    const OrbgCell cl = cells[c];
    const int l = cl.level;
    const int W = cl.w, H = cl.h;
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
    for (int i = tid; i < W * H; i += 256) {
        const int y = i / W, x = i - y * W;
        tile[i] = base[(int64_t)y * pitch + x];
    }
    __syncthreads();

    const int RW = W - 6, RH = H - 6;  // detection region [3, W-3) x [3, H-3)
    const int npix = (RW > 0 && RH > 0) ? RW * RH : 0;
    const int chunk = (npix + 255) / 256;
    const int p0 = min(tid * chunk, npix), p1 = min(p0 + chunk, npix);
    for (int p = p0; p < p1; p++) {
        const int ry = p / RW, rx = p - ry * RW;
        const int idx = (ry + 3) * W + rx + 3;
        sc[idx] = (int16_t)fast_score_lds(&tile[idx], W);
    }
    __syncthreads();

    // NMS at threshold th over this thread's raster chunk; bitmask of survivors
    auto nms = [&](int th, uint32_t &mask) -> int {
        int cnt = 0;
        mask = 0;
        for (int p = p0; p < p1; p++) {
            const int ry = p / RW, rx = p - ry * RW;
            const int idx = (ry + 3) * W + rx + 3;
            const int s = sc[idx];
            if (s < th) continue;
            bool keep = true;
#pragma unroll
            for (int dy = -1; dy <= 1; dy++)
#pragma unroll
                for (int dx = -1; dx <= 1; dx++) {
                    if (dx == 0 && dy == 0) continue;
                    const int qy = ry + dy, qx = rx + dx;
                    int q = 0;
                    if (qy >= 0 && qy < RH && qx >= 0 && qx < RW) {
                        const int sq = sc[(qy + 3) * W + qx + 3];
                        q = sq >= th ? sq : 0;
                    }
                    keep = keep && (s > q);
                }
            if (keep) {
                mask |= 1u << (p - p0);
                cnt++;
            }
        }
        return cnt;
    };
    uint32_t mask;
    int cnt = nms(g->ini_th, mask);
    const int tot_ini = block_sum(cnt, red);
    if (tot_ini == 0) cnt = nms(g->min_th, mask);
    int total;
    int off = block_excl_scan(cnt, &total, red);
    const int64_t slot = (int64_t)f * g->ncells + c;
    uint32_t *out = cell_kp + slot * g->cell_cap;
    const int xo = cl.x0 - ORBG_MIN_BORDER, yo = cl.y0 - ORBG_MIN_BORDER;
    for (int p = p0; p < p1; p++) {
        if (!(mask & (1u << (p - p0)))) continue;
        const int ry = p / RW, rx = p - ry * RW;
        const int s = sc[(ry + 3) * W + rx + 3];
        out[off++] = orbg_pack(xo + rx + 3, yo + ry + 3, s);
    }
    if (tid == 0) cell_cnt[slot] = total;
}

// ---------------------------------------------------------------------------
// k_blur: GaussianBlur(7x7, sigma 2, BORDER_REFLECT_101), bit-exact fixed point
// out = sat((sum_v k_v * sum_h k_h * p + 2^15) >> 16).  64x16 output tile.
// blockIdx.x enumerates tiles of all levels (tile_base per level in g).
// ---------------------------------------------------------------------------
__device__ __forceinline__ int reflect101(int i, int n)
{
    if (n == 1) return 0;
    while (i < 0 || i >= n) {
        if (i < 0) i = -i;
        if (i >= n) i = 2 * n - 2 - i;
    }
    return i;
}

__global__ __launch_bounds__(256) void k_blur(const OrbgGeom *__restrict__ g,
                                              const int32_t *__restrict__ tile_base,
                                              const uint8_t *__restrict__ img0, int64_t img_fs,
                                              int img_pitch, const uint8_t *__restrict__ pyr,
                                              uint8_t *__restrict__ blur)
{
    __shared__ uint8_t in[22][72];
    __shared__ int rows[22][64];
    const int f = blockIdx.y, tid = threadIdx.x;
    int l = 0;
    while (l + 1 < g->L && (int)blockIdx.x >= tile_base[l + 1]) l++;
    const int t = blockIdx.x - tile_base[l];
    const OrbgLevel &lv = g->lv[l];
    const int ntx = (lv.w + 63) / 64;
    const int tx0 = (t % ntx) * 64, ty0 = (t / ntx) * 16;
    const uint8_t *src;
    int pitch;
    if (l == 0) {
        src = img0 + f * img_fs;
        pitch = img_pitch;
    } else {
        src = pyr + f * g->pyr_frame + lv.pyr_off;
        pitch = lv.pitch;
    }
    for (int i = tid; i < 22 * 70; i += 256) {
        const int yy = i / 70, xx = i - yy * 70;
        const int sy = reflect101(ty0 + yy - 3, lv.h), sx = reflect101(tx0 + xx - 3, lv.w);
        in[yy][xx] = src[(int64_t)sy * pitch + sx];
    }
    __syncthreads();
    const int k0 = g->gk[0], k1 = g->gk[1], k2 = g->gk[2], k3 = g->gk[3], k4 = g->gk[4],
              k5 = g->gk[5], k6 = g->gk[6];
    for (int i = tid; i < 22 * 64; i += 256) {
        const int yy = i >> 6, xx = i & 63;
        const uint8_t *r = &in[yy][xx];
        rows[yy][xx] = k0 * r[0] + k1 * r[1] + k2 * r[2] + k3 * r[3] + k4 * r[4] + k5 * r[5] +
                       k6 * r[6];
    }
    __syncthreads();
    uint8_t *dst = blur + f * g->blur_frame + lv.blur_off;
    for (int i = tid; i < 16 * 64; i += 256) {
        const int yy = i >> 6, xx = i & 63;
        const int gy = ty0 + yy, gx = tx0 + xx;
        if (gy >= lv.h || gx >= lv.w) continue;
        const int acc = k0 * rows[yy][xx] + k1 * rows[yy + 1][xx] + k2 * rows[yy + 2][xx] +
                        k3 * rows[yy + 3][xx] + k4 * rows[yy + 4][xx] + k5 * rows[yy + 5][xx] +
                        k6 * rows[yy + 6][xx];
        dst[(int64_t)gy * lv.pitch + gx] = (uint8_t)min(max((acc + (1 << 15)) >> 16, 0), 255);
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
    const uint32_t *__restrict__ cell_kp, uint32_t *__restrict__ keys_all,
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
    const uint32_t *ckp = cell_kp + ((int64_t)f * g->ncells + lv.cell_base) * g->cell_cap;
    int n = 0;
    {
        int run = 0;
        for (int c0 = 0; c0 < lv.ncells; c0 += nthr) {
            const int c = c0 + tid;
            const int cn = c < lv.ncells ? ccount[c] : 0;
            int tot;
            const int off = block_excl_scan(cn, &tot, S.red) + run;
            for (int i = 0; i < cn; i++) keys[off + i] = ckp[(int64_t)c * g->cell_cap + i];
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
        if (alive > lv.out_cap) atomicOr(err_flag, 1 << 8);
    }
}

// ---------------------------------------------------------------------------
// pinned sincos (double Cody-Waite + Taylor, identical to oracle/orb_oracle.c)
// ---------------------------------------------------------------------------
__device__ void pinned_sincos(double x, double *s, double *c)
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

// cv::fastAtan2 (OpenCV 3.4 atan_f32), degrees in [0, 360]
__device__ float fast_atan2(float y, float x)
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
// k_orient_desc: one wave per output keypoint (level-major, octree list order)
// ---------------------------------------------------------------------------
struct OrbgKeypointDev {
    float x, y, size, angle, response;
    int32_t octave, class_id;
};

__global__ __launch_bounds__(256) void k_orient_desc(
    const OrbgGeom *__restrict__ g, const uint8_t *__restrict__ img0, int64_t img_fs,
    int img_pitch, const uint8_t *__restrict__ pyr, const uint8_t *__restrict__ blur,
    const uint32_t *__restrict__ lvl_kp, const int32_t *__restrict__ lvl_cnt,
    OrbgKeypointDev *__restrict__ kps, uint8_t *__restrict__ desc, int32_t *__restrict__ counts)
{
    const int f = blockIdx.y;
    const int lane = threadIdx.x & 63;
    const int i = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int L = g->L;
    const int32_t *lc = lvl_cnt + (int64_t)f * L;
    int total = 0, level = -1, idx = 0;
    for (int l = 0; l < L; l++) {
        const int c = lc[l];
        if (level < 0 && i < total + c) {
            level = l;
            idx = i - total;
        }
        total += c;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) counts[f] = total;
    if (level < 0 || i >= g->frame_cap) return;
    const OrbgLevel &lv = g->lv[level];
    const uint32_t key = lvl_kp[(int64_t)f * g->out_frame + lv.out_off + idx];
    const int x = orbg_px(key) + ORBG_MIN_BORDER, y = orbg_py(key) + ORBG_MIN_BORDER;
    const uint8_t *im;
    int pitch;
    if (level == 0) {
        im = img0 + f * img_fs;
        pitch = img_pitch;
    } else {
        im = pyr + f * g->pyr_frame + lv.pyr_off;
        pitch = lv.pitch;
    }
    // ---- IC_Angle: lanes 0..30 own column u = lane - 15 ----
    int m01 = 0, m10 = 0;
    if (lane < 31) {
        const int u = lane - ORBG_HALF_PATCH;
        const uint8_t *ctr = im + (int64_t)y * pitch + x;
        m10 = u * ctr[u];
        const int au = u < 0 ? -u : u;
        for (int v = 1; v <= ORBG_HALF_PATCH; v++) {
            if (au <= g->umax[v]) {
                const int vp = ctr[u + v * pitch], vm = ctr[u - v * pitch];
                m10 += u * (vp + vm);
                m01 += v * (vp - vm);
            }
        }
    }
    m01 = wave_sum(m01);
    m10 = wave_sum(m10);
    const float angle = fast_atan2((float)m01, (float)m10);

    // ---- rBRIEF on the blurred level: lane owns tests 4*lane .. 4*lane+3 ----
    const float factorPI = (float)(3.14159265358979323846 / 180.f);
    double sd, cd;
    pinned_sincos((double)(angle * factorPI), &sd, &cd);
    const float a = (float)cd, b = (float)sd;
    const uint8_t *bl = blur + f * g->blur_frame + lv.blur_off + (int64_t)y * lv.pitch + x;
    const int bpitch = lv.pitch;
    int nib = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int t = 4 * lane + j;
        int val[2];
#pragma unroll
        for (int s = 0; s < 2; s++) {
            const float px = (float)c_pattern[4 * t + 2 * s];
            const float py = (float)c_pattern[4 * t + 2 * s + 1];
            float ry, rx;
            if (g->brief_fma) {
                ry = fmaf(px, b, py * a);
                rx = fmaf(px, a, -(py * b));
            } else {
                const float t0 = px * b, t1 = py * a, t2 = px * a, t3 = py * b;
                ry = t0 + t1;
                rx = t2 - t3;
            }
            val[s] = bl[cv_round(ry) * bpitch + cv_round(rx)];
        }
        nib |= (val[0] < val[1]) << j;
    }
    const int hi = __shfl_down(nib, 1, 64);
    const int64_t o = (int64_t)f * g->frame_cap + i;
    if ((lane & 1) == 0) desc[o * 32 + (lane >> 1)] = (uint8_t)(nib | (hi << 4));
    if (lane == 0) {
        OrbgKeypointDev kp;
        float fx = (float)x, fy = (float)y;
        if (level != 0) {
            fx *= lv.scale;
            fy *= lv.scale;
        }
        kp.x = fx;
        kp.y = fy;
        kp.size = (float)lv.patch_size;
        kp.angle = angle;
        kp.response = (float)orbg_ps(key);
        kp.octave = level;
        kp.class_id = -1;
        kps[o] = kp;
    }
}

}  // namespace orbg
