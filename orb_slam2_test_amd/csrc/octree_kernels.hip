// octree_kernels.hip -- DistributeOctTree (ORBextractor.cc:668-951) on gfx950, LDS version.
//
// k_octree_lds handles every (frame, level) with <= OCT_KEY_CAP FAST candidates; levels
// with more fall back to k_octree (extract_kernels.hip, global-memory key scans).
//
// Every candidate's quadtree path is a 32-bit code: root index (4 bits, :705-724) then 14
// quadrant digits (n1=0, n2=1, n3=2, n4=3) computed with DivideNode's boundaries
// (:539-594).  (code, candidate index) pairs are sorted in LDS, so a node of depth d is a
// contiguous range whose children split at digit d: a split is three binary searches
// and no pass touches individual keys.  The std::list is an array of u64 node records
// {lo:16 | cnt:16 | seq:16 | depth:8} rebuilt every pass with the reference's
// push_front/erase order; seq = creation order = the pinned pointer tie-break of the
// sort at :869.  The best key of a node (:932-948) is the max of (response << 24 |
// ~index) over its range: max response, then lowest candidate index.
#include <hip/hip_runtime.h>

#include "orbg_device.h"
#include "orbg_internal.h"
#include "octree_args.h"

#pragma clang fp contract(off)

#ifndef ORBG_OCT_PRIO
#define ORBG_OCT_PRIO 2  // wave priority (s_setprio) of k_octree_lds (0: -1% per step)
#endif

namespace orbg {

// threads per quadtree workgroup: a template parameter (NT) of the kernel and its block-wide
// helpers; OCT_T names it inside them.  The single-frame launches take 512 (one workgroup per
// level on an idle chip: more lanes per phase), batches OCT_T_BATCH
#define OCT_T NT
#ifndef OCT_T_BATCH
#define OCT_T_BATCH 256  // batches: 0.612 -> 0.787 ms serial, but the pipelined step 5.42 -> 5.37 ms (r06bl; 128: 5.52, r06bm)
#endif
#define OCT_T_SMALL 512
#define OCT_CODE_DEPTH 14

// OCT_PC: cells per wave with their candidate loads in flight (per_cell).  Batches take 4
// (registers: several workgroups per CU); small batches (the single-frame drop-in: one
// workgroup per level on an idle chip, the candidate walks are chains of L2 round trips)
// OCT_PC_SMALL.
#ifndef OCT_PC_SMALL
#define OCT_PC_SMALL 8  // (16: +5 us per B = 1 extraction, profiles/r06an_single_knobs.txt)
#endif
#ifndef OCT_PC_BATCH
#define OCT_PC_BATCH 8  // at 256 threads: 4 -> 8 step 5.340-5.352 -> 5.317-5.334 ms, serial octree 0.787 -> 0.737 (r06bn; 16: 5.39, r06bp)
#endif

#define OCT_NBUCKET 16384  // counting-sort buckets: root (4 bits) + first 5 quadtree digits
#define OCT_BSHIFT 18      // code >> 18 = root (4 bits) + digits 0..4

// LDS: a static header plus a dynamic area sized per launch (OctLdsDims, host
// octree_lds_bytes): codes[kcap] u32 | sidx[kcap] u16 | resp[kcap] u8 | uni | aux[acap2] u16
// | coff[acap2] u16, where uni is the bucket counters (nbw u32, two u16 counters each) during
// the sort and afterwards the two list buffers + the phase-2 sort keys (3 x acap u64); resp
// is each candidate's FAST response and coff the cells' first candidate index, so the
// candidates never go through global scratch: the scatter and the winners re-read the
// cell lists (cell_kp, L2-resident).  A launch whose levels need little LDS runs several
// workgroups per CU.
struct OctLdsView {
    uint32_t *codes;
    uint16_t *sidx;
    uint8_t *resp;
    uint16_t *coff;
    uint32_t *bcnt;
    unsigned long long *list0, *list1;
    __device__ unsigned long long *list(int k) const { return k ? list1 : list0; }
    unsigned long long *sortv;
    uint16_t *aux;
};

__device__ __forceinline__ unsigned long long rec_make(int lo, int cnt, int seq, int depth)
{
    return (unsigned long long)(uint32_t)lo | ((unsigned long long)(uint32_t)cnt << 16) |
           ((unsigned long long)(uint32_t)seq << 32) | ((unsigned long long)(uint32_t)depth << 48);
}
__device__ __forceinline__ int rec_lo(unsigned long long r) { return (int)(r & 0xFFFF); }
__device__ __forceinline__ int rec_cnt(unsigned long long r) { return (int)((r >> 16) & 0xFFFF); }
__device__ __forceinline__ int rec_seq(unsigned long long r) { return (int)((r >> 32) & 0xFFFF); }
__device__ __forceinline__ int rec_depth(unsigned long long r) { return (int)((r >> 48) & 0xFF); }

// exclusive block scan for OCT_T threads (8 waves); sh: 16 ints, used as two halves in turn
// (par, flipped by every call; every thread makes the same calls): one barrier.  A wave that
// reaches the next-but-one scan has passed the next scan's barrier, which no wave reaches
// before it read this scan's half, so the half is free again (ORBG_OCT_SCAN_2BAR=1: the
// round-5 form, one half and a second barrier)
#ifndef ORBG_OCT_SCAN_2BAR
#define ORBG_OCT_SCAN_2BAR 0
#endif
template <int NT>
__device__ int oct_scan(int v, int *total, int *sh, int &par)
{
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int *h = ORBG_OCT_SCAN_2BAR ? sh : sh + (OCT_T / 64) * par;
    par ^= 1;
    int x = wave_incl_scan(v);
    if (lane == 63) h[wid] = x;
    __syncthreads();
    int before = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < OCT_T / 64; i++) {
        const int s = h[i];
        before += (i < wid) ? s : 0;
        tot += s;
    }
    if (ORBG_OCT_SCAN_2BAR) __syncthreads();
    *total = tot;
    return before + x - v;
}

// In-place ascending sort of u64 v[0..n) without padding (flip bitonic; virtual +inf
// entries at [n, pw) never move, so comparators touching them are skipped).
template <int NT>
__device__ void flip_bitonic_u64(unsigned long long *v, int n)
{
    int pw = 1;
    while (pw < n) pw <<= 1;
    const int half = pw >> 1;
    for (int k = 2; k <= pw; k <<= 1) {
        const int lhk = __builtin_ctz(k) - 1;
        for (int i = threadIdx.x; i < half; i += OCT_T) {
            const int blk = i >> lhk, r = i & ((k >> 1) - 1);
            const int a = blk * k + r, b = blk * k + k - 1 - r;
            if (b < n) {
                const unsigned long long x = v[a], y = v[b];
                if (x > y) {
                    v[a] = y;
                    v[b] = x;
                }
            }
        }
        __syncthreads();
        for (int j = k >> 2; j > 0; j >>= 1) {
            const int lj = __builtin_ctz(j);
            for (int i = threadIdx.x; i < half; i += OCT_T) {
                const int a = ((i >> lj) << (lj + 1)) + (i & (j - 1)), b = a + j;
                if (b < n) {
                    const unsigned long long x = v[a], y = v[b];
                    if (x > y) {
                        v[a] = y;
                        v[b] = x;
                    }
                }
            }
            __syncthreads();
        }
    }
}

// In-place ascending sort of n distinct u64 keys by rank counting: each thread holds up to
// OCT_RANK_R keys in registers, counts the smaller keys (LDS broadcast reads: every lane reads
// the same v[j]), then after one barrier writes each key at its rank.  Two barriers against
// flip_bitonic_u64's log2(n) (log2(n) + 1) / 2 -- the phase-2 sort is a chain of barriers of a
// single workgroup, the B = 1 critical path.  n <= OCT_RANK_R * OCT_T.
#define OCT_RANK_R 4
template <int NT>
__device__ void rank_sort_u64(unsigned long long *v, int n)
{
    const int tid = threadIdx.x;
    if (n <= OCT_T) {
        const unsigned long long x = tid < n ? v[tid] : 0ull;
        int c = 0;
#pragma unroll 8
        for (int j = 0; j < n; j++) c += v[j] < x;
        __syncthreads();
        if (tid < n) v[c] = x;
    } else {
        unsigned long long x[OCT_RANK_R];
        int c[OCT_RANK_R];
#pragma unroll
        for (int k = 0; k < OCT_RANK_R; k++) {
            const int i = tid + k * OCT_T;
            x[k] = i < n ? v[i] : ~0ull;
            c[k] = 0;
        }
#pragma unroll 4
        for (int j = 0; j < n; j++) {
            const unsigned long long y = v[j];
#pragma unroll
            for (int k = 0; k < OCT_RANK_R; k++) c[k] += y < x[k];
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < OCT_RANK_R; k++)
            if (tid + k * OCT_T < n) v[c[k]] = x[k];
    }
    __syncthreads();
}

#ifndef ORBG_OCT_RANK
#define ORBG_OCT_RANK 1  // phase-2 sort: 1 rank counting, 0 flip bitonic
#endif

// Candidates sit in counting-sort bucket order (root + first OCT_BDEPTH digits), unordered
// inside a bucket.  A node shallower than OCT_BDEPTH is a run of whole buckets, so its next
// digit is already monotone; a node of depth OCT_BDEPTH is exactly one bucket and is put in
// full-code order (insertion sort, buckets hold a handful of keys) by the one thread that
// splits it -- every deeper node is a sub-range of it.  Idempotent.
#define OCT_BDEPTH 5

__device__ __forceinline__ void oct_sort_bucket(uint32_t *codes, uint16_t *sidx, int lo, int hi)
{
    for (int i = lo + 1; i < hi; i++) {
        const uint32_t c = codes[i];
        if (codes[i - 1] <= c) continue;
        const uint16_t v = sidx[i];
        int j = i - 1;
        while (j >= lo && codes[j] > c) {
            codes[j + 1] = codes[j];
            sidx[j + 1] = sidx[j];
            j--;
        }
        codes[j + 1] = c;
        sidx[j + 1] = v;
    }
}

// children of the node record r: child start offsets b[0..4] (b[0] = lo, b[4] = lo + cnt)
__device__ __forceinline__ void oct_children(uint32_t *codes, uint16_t *sidx,
                                             unsigned long long r, int b[5])
{
    const int lo = rec_lo(r), hi = lo + rec_cnt(r), d = rec_depth(r);
    if (d == OCT_BDEPTH) oct_sort_bucket(codes, sidx, lo, hi);
    const int shift = 26 - 2 * d;
    b[0] = lo;
    b[4] = hi;
#pragma unroll
    for (int q = 1; q < 4; q++) {
        int a = b[q - 1], z = hi;  // first index in [a, z) with digit >= q
        while (a < z) {
            const int m = (a + z) >> 1;
            if ((int)((codes[m] >> shift) & 3) < q)
                a = m + 1;
            else
                z = m;
        }
        b[q] = a;
    }
}

// phase 2: a processed parent's split points as the cut pass left them in its sort entry
// (pos << 48 | b3 << 32 | b2 << 16 | b1); returns the parent's record
__device__ __forceinline__ unsigned long long oct_split_points(const OctLdsView &V, int cur,
                                                               unsigned long long w, int b[5],
                                                               int &pos)
{
    pos = (int)(w >> 48);
    const unsigned long long r = V.list(cur)[pos];
    b[0] = rec_lo(r);
    b[1] = (int)(w & 0xFFFF);
    b[2] = (int)((w >> 16) & 0xFFFF);
    b[3] = (int)((w >> 32) & 0xFFFF);
    b[4] = rec_lo(r) + rec_cnt(r);
    return r;
}

// frame = blockIdx.x, level = level0 + blockIdx.y (the dispatcher walks x fastest, so every
// frame's largest level starts first and the small levels fill the tail); handles a level iff
// its candidate count
// n <= D.kcap (k_octree takes the rest, same threshold)
template <int OCT_PC, int NT>
__global__ __launch_bounds__(NT) void k_octree_lds(
    const OrbgGeom *__restrict__ g, const int32_t *__restrict__ cell_cnt,
    const uint2 *__restrict__ cell_kp, uint32_t *__restrict__ lvl_kp,
    uint16_t *__restrict__ lvl_idx, int32_t *__restrict__ lvl_cnt, int32_t *__restrict__ err_flag,
    OctLdsDims D)
{
    __shared__ OctLdsHdr S;
    extern __shared__ __attribute__((aligned(16))) uint8_t oct_dyn[];
    OctLdsView V;
    {
        uint8_t *p = oct_dyn;
        V.codes = (uint32_t *)p;
        p += (size_t)D.kcap * 4;
        V.sidx = (uint16_t *)p;
        p += (size_t)D.kcap * 2;
        V.resp = p;
        p += (size_t)D.kcap;  // kcap: multiple of 64, so uni stays 8-byte aligned
        V.bcnt = (uint32_t *)p;
        V.list0 = (unsigned long long *)p;
        V.list1 = V.list0 + D.acap;
        V.sortv = V.list1 + D.acap;
        p += D.uni_bytes;
        V.aux = (uint16_t *)p;
        V.coff = V.aux + D.acap2;
    }
#if ORBG_OCT_PRIO
    // the keypoint half's stream is the pipelined step's critical path, and this kernel is a
    // latency-bound chain of barriers sharing the SIMDs with VALU-heavy waves: issue first
    __builtin_amdgcn_s_setprio(ORBG_OCT_PRIO);
#endif
    // the split pair's second launch: nothing to take unless the first flagged a level
    // (err_flag[3], cleared ahead of the pair by launch_octree_l0)
    if (D.kmin > 0 && err_flag[3] == 0) return;
    int spar = 0;  // oct_scan's half of S.red
    const int l = D.level0 + blockIdx.y, f = blockIdx.x, tid = threadIdx.x;
    const OrbgLevel &lv = g->lv[l];
    const int N = lv.nfeat, nIni = lv.nini;

    // ---- candidate count; larger levels (or > ALIVE-1 cells) belong to k_octree ----
    const int32_t *ccount = cell_cnt + (int64_t)f * g->ncells + lv.cell_base;
    const uint2 *ckp = cell_kp + ((int64_t)f * g->ncells + lv.cell_base) * g->cell_cap;
    const int ncells = lv.ncells;
    // a level left to k_octree: noted in err_flag[2] (not an error; the single-frame path
    // reruns a frame for which it skipped k_octree) and left empty, so a consumer that runs
    // before k_octree (or without it) never reads a stale count
    auto leave_to_fallback = [&]() {
        if (tid == 0) {
            // the split pair's first launch flags err_flag[3] (its second launch runs only
            // when set), every other launch err_flag[2]
            if (D.tag)
                err_flag[4] = D.tag;
            else
                atomicOr(err_flag + (D.first ? 3 : 2), 1);
            if (!D.keep_cnt) lvl_cnt[(int64_t)f * g->L + l] = 0;
        }
    };
    if (ncells + 1 > D.acap2) {
        leave_to_fallback();
        return;
    }
    int n = 0;
    for (int c0 = 0; c0 < ncells; c0 += OCT_T) {
        const int c = c0 + tid;
        int tot;
        const int off = oct_scan<NT>(c < ncells ? ccount[c] : 0, &tot, S.red, spar) + n;
        if (c < ncells) V.aux[c] = V.coff[c] = (uint16_t)min(off, 65535);
        n += tot;
    }
    if (D.kmin > 0 && n <= D.kmin) return;  // the first launch of a split pair holds it
    if (n > D.kcap) {
        leave_to_fallback();
        return;
    }
    if (tid == 0) V.aux[ncells] = V.coff[ncells] = (uint16_t)n;
    for (int i = tid; i < D.nbw; i += OCT_T) V.bcnt[i] = 0;
    __syncthreads();

    // ---- bucket histogram over the candidates (vToDistributeKeys order: cell-major, FAST
    //      order inside a cell; candidate k = coff[c] + slot), responses to LDS: one wave per
    //      cell (lane = slot), OCT_PC cells' loads in flight.  per_cell(fn) walks the cell lists;
    //      the scatter walks them again (the lists are L2-resident by then) ----
    auto per_cell = [&](auto &&fn) {
        const int lane = tid & 63, wv = tid >> 6;
        constexpr int NW = OCT_T / 64;
        for (int c0 = wv; c0 < ncells; c0 += OCT_PC * NW) {
            uint2 e[OCT_PC];
            int k[OCT_PC], cnt[OCT_PC];
#pragma unroll
            for (int u = 0; u < OCT_PC; u++) {
                const int c = c0 + u * NW;
                cnt[u] = 0;
                k[u] = 0;
                e[u] = make_uint2(0, 0);
                if (c < ncells) {
                    const int lo = V.coff[c];
                    cnt[u] = (int)V.coff[c + 1] - lo;
                    k[u] = lo + lane;
                    if (lane < cnt[u]) e[u] = ckp[(int64_t)c * g->cell_cap + lane];
                }
            }
#pragma unroll
            for (int u = 0; u < OCT_PC; u++) {
                if (lane < cnt[u]) fn(k[u], e[u]);
                for (int kl = lane + 64; kl < cnt[u]; kl += 64) {  // cells with > 64 corners
                    const int c = c0 + u * NW;
                    fn(k[u] - lane + kl, ckp[(int64_t)c * g->cell_cap + kl]);
                }
            }
        }
    };
    per_cell([&](int k, uint2 e) {
        V.resp[k] = (uint8_t)orbg_ps(e.x);
        const uint32_t b = e.y >> OCT_BSHIFT;
        atomicAdd(&V.bcnt[b >> 1], 1u << (16 * (b & 1)));
    });
    __syncthreads();
    // developer phase stops (ORBG_DBG 1-4, developer builds only): the level is left empty
    auto dbg_stop = [&](int d) {
        if (g->dbg != d) return false;
        if (tid == 0) lvl_cnt[(int64_t)f * g->L + l] = 0;
        return true;
    };
    if (dbg_stop(1)) return;
    // ---- exclusive scan of the nini * 1024 u16 bucket counters (2 * nini per thread) ----
    {
        const int PER = D.nbw / OCT_T;  // words per thread (= roots)
        uint32_t *wb = V.bcnt + tid * PER;
        int sum = 0;
        for (int i = 0; i < PER; i++) sum += (int)(wb[i] & 0xFFFF) + (int)(wb[i] >> 16);
        int tot;
        int run = oct_scan<NT>(sum, &tot, S.red, spar);
        for (int i = 0; i < PER; i++) {
            const uint32_t w = wb[i];
            const int a = (int)(w & 0xFFFF), b = (int)(w >> 16);
            wb[i] = (uint32_t)run | ((uint32_t)(run + a) << 16);
            run += a + b;
        }
    }
    __syncthreads();
    // ---- scatter into bucket order (unordered inside a bucket) ----
    per_cell([&](int k, uint2 e) {
        const uint32_t code = e.y, b = code >> OCT_BSHIFT;
        const uint32_t old = atomicAdd(&V.bcnt[b >> 1], 1u << (16 * (b & 1)));
        const int slot = (int)((old >> (16 * (b & 1))) & 0xFFFF);
        V.codes[slot] = code;
        V.sidx[slot] = (uint16_t)k;
    });
    __syncthreads();
    if (dbg_stop(2)) return;

    // ---- roots (:705-739): contiguous by the top 4 code bits ----
    if (tid <= nIni) S.rootlo[tid] = 0;
    __syncthreads();
    for (int i = tid; i < n; i += OCT_T) {
        const int r = (int)(V.codes[i] >> 28);
        const int rp = i > 0 ? (int)(V.codes[i - 1] >> 28) : -1;
        if (r != rp)
            for (int q = rp + 1; q <= r; q++) S.rootlo[q] = i;
    }
    if (tid == 0) {
        const int rl = n > 0 ? (int)(V.codes[n - 1] >> 28) : -1;
        for (int q = rl + 1; q <= nIni; q++) S.rootlo[q] = n;
    }
    __syncthreads();
    if (tid == 0) {
        int a = 0;
        for (int r = 0; r < nIni; r++) {
            const int cnt = S.rootlo[r + 1] - S.rootlo[r];
            if (cnt > 0) V.list(0)[a++] = rec_make(S.rootlo[r], cnt, 0, 0);
        }
        S.s_alive = a;
        S.s_err = 0;
    }
    __syncthreads();
    // the list state is workgroup-uniform and every thread derives it from the scans' totals,
    // so it lives in registers (no tid-0 update and barrier per pass); S.s_err collects the
    // depth errors any thread may raise, read after each pass's barrier
    int st_alive = S.s_alive, st_cur = 0, st_seq = 1;  // roots never enter vSizeAndPointerToNode
    int st_vbase = 0, st_vend = 0, st_err = 0;
    bool st_phase2 = false;

    // ================= phase 1 passes (:751-852) =================
    while (true) {
        const int alive = st_alive, cur = st_cur, nxt = cur ^ 1, seq0 = st_seq;
        // sweep 1: children of every splitting node (kept in registers for sweep 2)
        constexpr int MAXCH = ORBG_OCT_ALIVE / OCT_T;
        int bb[MAXCH][5];
        int ee[MAXCH], spp[MAXCH];
        int tot_e = 0, nexp = 0;
#pragma unroll
        for (int ch = 0; ch < MAXCH; ch++) {
            const int i = ch * OCT_T + tid;
            int e = 0, m = 0, sp = 0;
#pragma unroll
            for (int q = 0; q < 5; q++) bb[ch][q] = 0;
            if (ch * OCT_T < alive) {
                if (i < alive) {
                    const unsigned long long r = V.list(cur)[i];
                    if (rec_cnt(r) > 1) {
                        if (rec_depth(r) >= OCT_CODE_DEPTH) {
                            S.s_err = 4;
                        } else {
                            sp = 1;
                            oct_children(V.codes, V.sidx, r, bb[ch]);
#pragma unroll
                            for (int q = 0; q < 4; q++) {
                                e += bb[ch][q + 1] > bb[ch][q];
                                m += bb[ch][q + 1] - bb[ch][q] > 1;
                            }
                        }
                    }
                }
                int t;  // both totals from one scan (each < 2^16: e, m <= 4 per node)
                oct_scan<NT>(e | (m << 16), &t, S.red, spar);
                tot_e += t & 0xFFFF;
                nexp += t >> 16;
            }
            ee[ch] = e;
            spp[ch] = sp;
        }
        int nsplit_total = 0;
        // sweep 2: place children (reverse parent order, n4..n1) and the untouched nodes
        {
            int run = 0;
#pragma unroll
            for (int ch = 0; ch < MAXCH; ch++) {
                if (ch * OCT_T >= alive) break;
                const int i = ch * OCT_T + tid;
                const int e = ee[ch], sp = spp[ch];
                int tot;
                const int pre = oct_scan<NT>(e | (sp << 16), &tot, S.red, spar) + run;
                const int E = pre & 0xFFFF, splits_before = pre >> 16;
                if (i < alive) {
                    const unsigned long long r = V.list(cur)[i];
                    if (sp) {
                        const int blk = tot_e - E - e;
                        int k = 0;
#pragma unroll
                        for (int q = 0; q < 4; q++) {
                            const int cnt = bb[ch][q + 1] - bb[ch][q];
                            if (cnt == 0) continue;
                            V.list(nxt)[blk + (e - 1 - k)] =
                                rec_make(bb[ch][q], cnt, seq0 + E + k, rec_depth(r) + 1);
                            k++;
                        }
                    } else {
                        V.list(nxt)[tot_e + i - splits_before] = r;
                    }
                }
                run += tot;
            }
            nsplit_total = run >> 16;
        }
        const int na = tot_e + alive - nsplit_total;
        __syncthreads();  // this pass's list writes (and any S.s_err) before the next pass
        st_alive = na;
        st_cur = nxt;
        st_seq = seq0 + tot_e;
        st_vbase = seq0;
        st_vend = seq0 + tot_e;
        st_err = S.s_err;
        if (!st_err && (na > D.acap || seq0 + tot_e > 65535)) st_err = 5;
        if (st_err) break;
        if (na >= N || na == alive) break;   // :849-852
        if (na + nexp * 3 > N) {              // :856
            st_phase2 = true;
            break;
        }
    }

    if (dbg_stop(3)) return;
    // ================= phase 2 rounds (:859-924) =================
    if (st_phase2 && !st_err) {
        while (true) {
            const int alive = st_alive, cur = st_cur, nxt = cur ^ 1, seq0 = st_seq;
            const int vbase = st_vbase, vend = st_vend;
            // vPrevSizeAndPointerToNode: multi-key nodes created last round -> (cnt, seq, pos)
            int np = 0;
            for (int i0 = 0; i0 < alive; i0 += OCT_T) {
                const int i = i0 + tid;
                int fl = 0;
                unsigned long long r = 0;
                if (i < alive) {
                    r = V.list(cur)[i];
                    const int sq = rec_seq(r);
                    fl = rec_cnt(r) > 1 && sq >= vbase && sq < vend;
                }
                int tot;
                const int o = oct_scan<NT>(fl, &tot, S.red, spar) + np;
                if (fl)
                    V.sortv[o] = ((unsigned long long)rec_cnt(r) << 32) |
                                 ((unsigned long long)rec_seq(r) << 16) | (unsigned)i;
                np += tot;
            }
            for (int i = tid; i < alive; i += OCT_T) V.aux[i] = 0;
            __syncthreads();
            if (ORBG_OCT_RANK && np <= OCT_RANK_R * OCT_T)
                rank_sort_u64<NT>(V.sortv, np);
            else
                flip_bitonic_u64<NT>(V.sortv, np);
            // processing order p = largest (cnt, seq) first (:872); cut at the first p with
            // alive + sum_{p' <= p} (children - 1) >= N (:917-918)
            if (tid == 0) S.s_nproc = np;
            __syncthreads();
            {
                int run = 0;
                for (int p0 = 0; p0 < np; p0 += OCT_T) {
                    const int p = p0 + tid;
                    int dl = 0;
                    if (p < np) {
                        const int pos = (int)(V.sortv[np - 1 - p] & 0xFFFF);
                        const unsigned long long r = V.list(cur)[pos];
                        if (rec_depth(r) >= OCT_CODE_DEPTH) S.s_err = 6;
                        int b[5];
                        oct_children(V.codes, V.sidx, r, b);
                        int e = 0;
#pragma unroll
                        for (int q = 0; q < 4; q++) e += b[q + 1] > b[q];
                        dl = e - 1;
                        // the sort key is dead: keep the split points for the two passes below
                        // (this thread's own entry; b[0], b[4] are the record's range)
                        V.sortv[np - 1 - p] = (unsigned long long)pos << 48 |
                                              (unsigned long long)b[3] << 32 |
                                              (unsigned long long)b[2] << 16 | (unsigned)b[1];
                    }
                    int tot;
                    const int incl = oct_scan<NT>(dl, &tot, S.red, spar) + run + dl;
                    if (p < np && alive + incl >= N) atomicMin(&S.s_nproc, p + 1);
                    run += tot;
                }
            }
            __syncthreads();
            const int nproc = S.s_nproc;
            // children of processed parents (creation order = processing order)
            int tot_e = 0;
            for (int p0 = 0; p0 < nproc; p0 += OCT_T) {
                const int p = p0 + tid;
                int e = 0;
                if (p < nproc) {
                    int b[5], pos;
                    oct_split_points(V, cur, V.sortv[np - 1 - p], b, pos);
#pragma unroll
                    for (int q = 0; q < 4; q++) e += b[q + 1] > b[q];
                    V.aux[pos] = 1;  // processed parent
                }
                int t;
                oct_scan<NT>(e, &t, S.red, spar);
                tot_e += t;
            }
            {
                int run = 0;
                for (int p0 = 0; p0 < nproc; p0 += OCT_T) {
                    const int p = p0 + tid;
                    int e = 0, b[5] = {0, 0, 0, 0, 0};
                    unsigned long long r = 0;
                    if (p < nproc) {
                        int pos;
                        r = oct_split_points(V, cur, V.sortv[np - 1 - p], b, pos);
#pragma unroll
                        for (int q = 0; q < 4; q++) e += b[q + 1] > b[q];
                    }
                    int tot;
                    const int E = oct_scan<NT>(e, &tot, S.red, spar) + run;
                    if (p < nproc) {
                        const int blk = tot_e - E - e;
                        int k = 0;
#pragma unroll
                        for (int q = 0; q < 4; q++) {
                            const int cnt = b[q + 1] - b[q];
                            if (cnt == 0) continue;
                            V.list(nxt)[blk + (e - 1 - k)] =
                                rec_make(b[q], cnt, seq0 + E + k, rec_depth(r) + 1);
                            k++;
                        }
                    }
                    run += tot;
                }
                int runp = 0;
                for (int i0 = 0; i0 < alive; i0 += OCT_T) {
                    const int i = i0 + tid;
                    const int fl = (i < alive) ? (int)V.aux[i] : 0;
                    int tot;
                    const int before = oct_scan<NT>(fl, &tot, S.red, spar) + runp;
                    if (i < alive && !fl) V.list(nxt)[tot_e + i - before] = V.list(cur)[i];
                    runp += tot;
                }
            }
            const int na = tot_e + alive - nproc;
            __syncthreads();  // this round's list writes (and any S.s_err) before the next
            st_alive = na;
            st_cur = nxt;
            st_seq = seq0 + tot_e;
            st_vbase = seq0;
            st_vend = seq0 + tot_e;
            st_err = S.s_err;
            if (!st_err && (na > D.acap || seq0 + tot_e > 65535)) st_err = 7;
            if (st_err) break;
            if (na >= N || na == alive) break;  // :921-922
        }
    }

    if (dbg_stop(4)) return;
    // ================= best key per node, list order (:932-948) =================
    const int alive = st_alive, cur = st_cur;
    if (st_err) {
        if (tid == 0) {
            atomicOr(err_flag, 1 << st_err);
            atomicMin(err_flag + 1, f);
            lvl_cnt[(int64_t)f * g->L + l] = 0;
        }
        return;
    }
    // label every sorted position with its node's list position, then one flat pass
    uint32_t *best = (uint32_t *)V.sortv;
    for (int i = tid; i < alive; i += OCT_T) {
        const unsigned long long r = V.list(cur)[i];
        const int lo = rec_lo(r), cnt = rec_cnt(r);
        for (int p = lo; p < lo + cnt; p++) V.codes[p] = (uint32_t)i;
        best[i] = 0;
    }
    __syncthreads();
    for (int p = tid; p < n; p += OCT_T) {
        const uint32_t idx = V.sidx[p], pos = V.codes[p];
        atomicMax(&best[pos], ((uint32_t)V.resp[idx] << 24) | (0xFFFFFFu - idx));
    }
    __syncthreads();
    // winners: candidate index -> its cell (last c with coff[c] <= idx) -> the cell list entry.
    // Slot order: winner i (the reference's list order, the output row) goes to the slot its
    // image tile's counting sort gives it, with lvl_idx[slot] = i, so k_orient_desc's waves get
    // keypoints whose patches share cache lines; identity when D.tile_sort = 0.  The codes
    // array (dead here) holds the keys, sidx (dead) the tile counters.
    uint32_t *out = lvl_kp + (int64_t)f * g->out_frame + lv.out_off;
    uint16_t *oidx = lvl_idx + (int64_t)f * g->out_frame + lv.out_off;
    const int nout = min(alive, lv.out_cap);
    uint32_t *tcnt = (uint32_t *)V.sidx;
    const bool tsort = D.tile_sort && D.kcap >= 64;  // kcap / 2 >= 1 tile counter
    int xs = 7, ys = 5, ntx = 0, nbins = 0;
    if (tsort) {
        for (;; xs++, ys++) {
            ntx = (lv.w >> xs) + 1;
            nbins = ntx * ((lv.h >> ys) + 1);
            if (nbins <= D.kcap / 2) break;
        }
        for (int t = tid; t < nbins; t += OCT_T) tcnt[t] = 0;
        __syncthreads();
    }
    for (int i = tid; i < nout; i += OCT_T) {
        const int idx = (int)(0xFFFFFFu - (best[i] & 0xFFFFFFu));
        int a = 0, z = ncells;  // coff[a] <= idx < coff[z]
        while (z - a > 1) {
            const int m = (a + z) >> 1;
            if ((int)V.coff[m] <= idx)
                a = m;
            else
                z = m;
        }
        const uint32_t key = ckp[(int64_t)a * g->cell_cap + (idx - (int)V.coff[a])].x;
        if (tsort) {
            V.codes[i] = key;
            atomicAdd(&tcnt[(orbg_py(key) >> ys) * ntx + (orbg_px(key) >> xs)], 1u);
        } else {
            out[i] = key;
            oidx[i] = (uint16_t)i;
        }
    }
    if (tsort) {
        __syncthreads();
        // exclusive scan of the tile counters: thread t owns a run of consecutive tiles
        const int per = (nbins + OCT_T - 1) / OCT_T, t0 = min(tid * per, nbins),
                  t1 = min(t0 + per, nbins);
        int sum = 0;
        for (int t = t0; t < t1; t++) sum += (int)tcnt[t];
        int tot;
        int run = oct_scan<NT>(sum, &tot, S.red, spar);
        for (int t = t0; t < t1; t++) {
            const int c = (int)tcnt[t];
            tcnt[t] = (uint32_t)run;
            run += c;
        }
        __syncthreads();
        for (int i = tid; i < nout; i += OCT_T) {
            const uint32_t key = V.codes[i];
            const int slot =
                (int)atomicAdd(&tcnt[(orbg_py(key) >> ys) * ntx + (orbg_px(key) >> xs)], 1u);
            out[slot] = key;
            oidx[slot] = (uint16_t)i;
        }
    }
    if (tid == 0) {
        lvl_cnt[(int64_t)f * g->L + l] = nout;
        if (alive > lv.out_cap) {
            atomicOr(err_flag, 1 << 8);
            atomicMin(err_flag + 1, f);
        }
    }
}

// small: B <= ORBG_SIDE_BLUR_B (OCT_PC_SMALL cells in flight per wave), else OCT_PC_BATCH
hipError_t launch_octree_lds(bool small, dim3 grid, size_t lds, hipStream_t st, const OrbgGeom *g,
                             const int32_t *cell_cnt, const uint2 *cell_kp, uint32_t *lvl_kp,
                             uint16_t *lvl_idx, int32_t *lvl_cnt, int32_t *err_flag, OctLdsDims D)
{
    if (small)
        hipLaunchKernelGGL((k_octree_lds<OCT_PC_SMALL, OCT_T_SMALL>), grid, dim3(OCT_T_SMALL), lds, st,
                           g, cell_cnt, cell_kp, lvl_kp, lvl_idx, lvl_cnt, err_flag, D);
    else
        hipLaunchKernelGGL((k_octree_lds<OCT_PC_BATCH, OCT_T_BATCH>), grid, dim3(OCT_T_BATCH), lds, st,
                           g, cell_cnt, cell_kp, lvl_kp, lvl_idx, lvl_cnt, err_flag, D);
    return hipGetLastError();
}

hipError_t octree_lds_attr(int bytes)
{
    for (const void *k : {(const void *)k_octree_lds<OCT_PC_BATCH, OCT_T_BATCH>,
                          (const void *)k_octree_lds<OCT_PC_SMALL, OCT_T_SMALL>}) {
        const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace orbg
