// match_kernels.hip -- ORBmatcher hot loops for gfx950.
//
//   k_knn2_*          brute-force 2-NN over ORBmatcher::DescriptorDistance
//                     (ORBmatcher.cc:1846-1862; best/second update rule :541-556) on the
//                     matrix cores: bits expanded to +-1.0 e2m1, v_mfma_scale_f32_32x32x64_f8f6f4
//                     dot products (affine in the distance), top-2 keys per query.
//   k_init_cands      SearchForInitialization's data-parallel part (ORBmatcher.cc:508-545):
//                     per level-0 query, the window candidates of F2.GetFeaturesInArea
//                     (Frame.cc:421-504) with their distances, kept as the K smallest
//                     (dist, grid-enumeration order) keys.  One wave per query.
//   k_init_resolve    the order-dependent part (:536-631): vMatchedDistance filter,
//                     best/second, TH_LOW, ratio, conflict stealing, rotation histogram,
//                     ComputeThreeMaxima (:1800-1841).  One wave per frame pair walks the
//                     queries in index order; an exact wave-parallel rescan covers the
//                     rare query whose K-list is exhausted by the filter.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>

#include "../../include/orbg.h"
#include "orbg_internal.h"
#include "orbg_device.h"
#include "match_device.h"

#pragma clang fp contract(off)

namespace orbg {

void prof_begin(void *prof, hipStream_t s, const char *n, hipEvent_t *a);
void prof_end(void *prof, hipStream_t s, const char *n, hipEvent_t a);
bool prof_skip_name(const char *n);

// reductions over a 16-lane row (the query groups of init_cands_block): every lane gets the
// row's result by DPP row_ror 8 / 4 and quad_perm [2,3,0,1] / [1,0,3,2] (in the ALU; a
// __shfl_xor ladder is four LDS-pipeline round trips per 32-bit step)
#ifndef ORBG_ROW16_SHFL
__device__ __forceinline__ int row16_sum(int x)
{
    x += __builtin_amdgcn_mov_dpp(x, 0x128, 0xf, 0xf, false);  // row_ror:8
    x += __builtin_amdgcn_mov_dpp(x, 0x124, 0xf, 0xf, false);  // row_ror:4
    x += __builtin_amdgcn_mov_dpp(x, 0x4e, 0xf, 0xf, false);   // quad_perm [2,3,0,1]
    x += __builtin_amdgcn_mov_dpp(x, 0xb1, 0xf, 0xf, false);   // quad_perm [1,0,3,2]
    return x;
}
__device__ __forceinline__ unsigned long long row16_min_u64(unsigned long long v)
{
    auto step = [&](auto CTRL) {
        constexpr int c = decltype(CTRL)::value;
        const uint32_t lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)v, c, 0xf, 0xf, false);
        const uint32_t hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(v >> 32), c, 0xf, 0xf, false);
        const unsigned long long u = (unsigned long long)hi << 32 | lo;
        v = u < v ? u : v;
    };
    step(std::integral_constant<int, 0x128>{});
    step(std::integral_constant<int, 0x124>{});
    step(std::integral_constant<int, 0x4e>{});
    step(std::integral_constant<int, 0xb1>{});
    return v;
}
#else  // the round-5 form, A/B builds
__device__ __forceinline__ int row16_sum(int x)
{
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) x += __shfl_xor(x, o, 16);
    return x;
}
__device__ __forceinline__ unsigned long long row16_min_u64(unsigned long long mn)
{
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) {
        const unsigned long long u = __shfl_xor(mn, o, 16);
        mn = u < mn ? u : mn;
    }
    return mn;
}
#endif

#define TH_LOW 50
#define HISTO_LENGTH 30

// knn2 on the matrix cores: every 256-bit DescriptorDistance of a 32 x 32 block of (train,
// query) pairs is one MFMA dot product of +-1 bit vectors, offset so that the accumulator IS
// the key  d << 13 | train index  (k_knn2_* below; the train index fits the 13 low bits).
//
// best/second (ORBmatcher.cc:541-556's strict-< scan in train order): the smallest key is
// (min distance, first index); the distance of the second smallest key is the multiset
// second minimum, which is what the in-order rule leaves in bestDist2.  Per value: a max and
// a min (second) and a min (best).
typedef int knn_v4i __attribute__((ext_vector_type(4)));
typedef int knn_v16i __attribute__((ext_vector_type(16)));

#define KNN_MAX_TRAIN 8192   // train index in the 13 low key bits
#define KNN_NONE 0x40000000  // C tag of the rows past nt: keys above any real one

// key is read straight out of the MFMA result, so everything here stays compiler-visible (the
// compiler places the MFMA -> VALU wait states; it does not for inline asm).  Three VOP2
// ops: med3(k1, k2, key) with k1 <= k2, then the new minimum.
__device__ __forceinline__ void knn_key_update(int key, int &k1, int &k2)
{
    k2 = min(k2, max(k1, key));
    k1 = min(k1, key);
}

// knn2 on the fp4 matrix cores: v_mfma_scale_f32_32x32x64_f8f6f4 with e2m1 operands runs
// K = 64 in the cycles the i8 form needs for K = 32, so K = 256 is four MFMAs (round 1's i8
// v_mfma_i32_32x32x32_i8 form needed eight; removed in round 3).  Every bit becomes +-1.0 in
// e2m1 (0x2 = +1, 0xA = -1): train (A) b=1 -> -1, query (B) b=1 -> +1 (b=0 the opposite), so
// one product is -1 where the bits agree and +1 where they differ; the E8M0 scale 2^12 on A
// makes the dot product 4096 (d - (256 - d)) = 8192 d - 2^20, and the C input is the train
// index + 2^20, so the key is 8192 d + index >= 0.  Every partial sum is an integer below
// 2^22 in magnitude, exact in the f32 accumulator whatever the summation order; a
// non-negative f32 orders like its bit pattern, so the top-2 runs on the u32 bits (integer
// min / med3: no NaN canonicalisation).  Past-nt rows carry 2^30 (rounded sums stay
// >= 2^30 - 2^20, above every real key).  k order (A and B alike): step s, lane half h -> descriptor dword 2s + h; VGPR
// q, nibble j -> bit 4j + q of that dword.
typedef int knn_v8i __attribute__((ext_vector_type(8)));
typedef float knn_v16f __attribute__((ext_vector_type(16)));
#ifndef ORBG_KNN_MED3
#define ORBG_KNN_MED3 1
#endif
#define KNN4_ROWB 144  // expanded train row: 128 B + 16 B pad (16 lanes' b128 reads: 64 banks)
#define KNN4_SCALE_A (127 + 12)  // E8M0 2^12
#define KNN4_SCALE_B 127         // E8M0 1.0

// e2m1 nibbles of bits q, q+4, .., q+28 of x: b=1 -> 0xA (-1.0), b=0 -> 0x2 (+1.0)
__device__ __forceinline__ uint32_t knn4_neg(uint32_t x, int q)
{
    return (((x >> q) & 0x11111111u) << 3) | 0x22222222u;
}
// b=1 -> 0x2 (+1.0), b=0 -> 0xA (-1.0)
__device__ __forceinline__ uint32_t knn4_pos(uint32_t x, int q)
{
    return knn4_neg(x, q) ^ 0x88888888u;
}

__device__ __forceinline__ void knn2_block_fp4(const uint8_t *__restrict__ q, int nq,
                                               const uint8_t *__restrict__ t, int nt,
                                               int32_t *__restrict__ out, int qbase)
{
    __shared__ __attribute__((aligned(16))) uint8_t tile[2][64 * KNN4_ROWB];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int col = lane & 31, h = lane >> 5;
    // B fragments: query qbase + 64 wv + 32 u + col, step s: dword 2s + h
    knn_v8i bq[2][4];
#pragma unroll
    for (int u = 0; u < 2; u++) {
        const int qi = qbase + wv * 64 + u * 32 + col;
        uint32_t x[4] = {0, 0, 0, 0};
        if (qi < nq) {
            const uint32_t *p = (const uint32_t *)(q + (size_t)qi * 32);
#pragma unroll
            for (int s = 0; s < 4; s++) x[s] = p[2 * s + h];
        }
#pragma unroll
        for (int s = 0; s < 4; s++) {
#pragma unroll
            for (int qd = 0; qd < 4; qd++) {
                bq[u][s][qd] = (int)knn4_pos(x[s], qd);
                bq[u][s][qd + 4] = 0;  // e2m1 uses the first four VGPRs only
            }
        }
    }
    uint32_t k1[2] = {UINT_MAX, UINT_MAX}, k2[2] = {UINT_MAX, UINT_MAX};

    // expansion of stage s0 (64 rows) into buffer bf: thread -> rows (tid >> 3) and
    // (tid >> 3) + 32, dword tid & 7 -> 16 bytes at row offset 16 * dword
    const int er = tid >> 3, esd = tid & 7;
    auto fetch1 = [&](int row) -> uint32_t {
        return ((const uint32_t *)(t + (size_t)min(row, nt - 1) * 32))[esd];
    };
    auto expand1 = [&](uint32_t x, uint8_t *dst) {
        uint4 w;
        w.x = knn4_neg(x, 0); w.y = knn4_neg(x, 1);
        w.z = knn4_neg(x, 2); w.w = knn4_neg(x, 3);
        *(uint4 *)dst = w;
    };
    auto expand = [&](uint32_t x0, uint32_t x1, int bf) {
        expand1(x0, tile[bf] + er * KNN4_ROWB + esd * 16);
        expand1(x1, tile[bf] + (er + 32) * KNN4_ROWB + esd * 16);
    };
    uint32_t xr0 = 0, xr1 = 0;
    if (nt > 0) {
        expand(fetch1(er), fetch1(er + 32), 0);
        xr0 = fetch1(64 + er);
        xr1 = fetch1(96 + er);
    }
    // two accumulator sets, one per 32-row subtile of a stage: the top-2 epilogue of one set
    // runs while the MFMAs of the other are in flight (no accumulator copies)
    knn_v16f accA[2], accB[2];
    auto epilogue = [&](const knn_v16f (&acc)[2]) {
#pragma unroll
        for (int r = 0; r < 16; r++) {
#pragma unroll
            for (int u = 0; u < 2; u++) {
                // k1 <= k2: the new second key is med3(k1, k2, key), then the new minimum
                // (via a scalar: __builtin_bit_cast of an ext_vector element lvalue reads
                // element 0 under this clang)
                const float kf = acc[u][r];
                const uint32_t key = __float_as_uint(kf);
#if ORBG_KNN_MED3
                // the min reads the MFMA result first (the compiler places the MFMA -> VALU
                // wait states there); v_med3_u32 of (k1, k2, key) with k1 <= k2 is the new
                // second key -- one op where the compiler's min/max form takes two
                const uint32_t k1o = k1[u];
                k1[u] = min(k1o, key);
                asm volatile("v_med3_u32 %0, %1, %2, %3" : "=v"(k2[u]) : "v"(k1o), "v"(k2[u]), "v"(key));
#else
                k2[u] = min(k2[u], max(k1[u], key));
                k1[u] = min(k1[u], key);
#endif
            }
        }
    };
    auto subtile = [&](int tb, int bf, int sub, knn_v16f (&acc)[2]) {
        knn_v16f ctag;
        const float tbh = (float)(tb + 4 * h + (1 << 20));
#pragma unroll
        for (int r = 0; r < 16; r++) ctag[r] = tbh + (float)((r & 3) + 8 * (r >> 2));
        if (tb + 32 > nt) {  // last subtile: rows past nt get keys above every real one
#pragma unroll
            for (int r = 0; r < 16; r++)
                if (ctag[r] >= (float)(nt + (1 << 20))) ctag[r] = (float)KNN_NONE;
        }
        const uint8_t *arow = tile[bf] + (32 * sub + col) * KNN4_ROWB + h * 16;
#pragma unroll
        for (int s = 0; s < 4; s++) {
            const knn_v4i a4 = *(const knn_v4i *)(arow + s * 32);
            const knn_v8i a = {a4[0], a4[1], a4[2], a4[3], 0, 0, 0, 0};
            acc[0] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(
                a, bq[0][s], s ? acc[0] : ctag, 4, 4, 0, KNN4_SCALE_A, 0, KNN4_SCALE_B);
            acc[1] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(
                a, bq[1][s], s ? acc[1] : ctag, 4, 4, 0, KNN4_SCALE_A, 0, KNN4_SCALE_B);
        }
    };
    bool pendB = false;
    for (int s0 = 0, bf = 0; s0 < nt; s0 += 64, bf ^= 1) {
        __syncthreads();
        if (s0 + 64 < nt) {
            expand(xr0, xr1, bf ^ 1);
            xr0 = fetch1(s0 + 128 + er);
            xr1 = fetch1(s0 + 160 + er);
        }
        subtile(s0, bf, 0, accA);
        if (pendB) epilogue(accB);
        pendB = s0 + 32 < nt;
        if (pendB) subtile(s0 + 32, bf, 1, accB);
        epilogue(accA);
    }
    if (pendB) epilogue(accB);
    const uint32_t none = 0x4E000000u;  // bits of 2^29: real keys < 2^22, past-nt >= 2^30 - 2^20
#pragma unroll
    for (int u = 0; u < 2; u++) {
        const uint32_t o1 = (uint32_t)__shfl_xor((int)k1[u], 32, 64);
        const uint32_t o2 = (uint32_t)__shfl_xor((int)k2[u], 32, 64);
        const uint32_t b1 = min(k1[u], o1);
        const uint32_t b2 = min(min(k2[u], o2), max(k1[u], o1));
        const int qi = qbase + wv * 64 + u * 32 + col;
        if (h == 0 && qi < nq) {
            const bool v1 = b1 < none, v2 = b2 < none;
            const int e1 = v1 ? (int)__builtin_bit_cast(float, b1) : 0;
            const int e2 = v2 ? (int)__builtin_bit_cast(float, b2) : 0;
            out[(size_t)qi * 3 + 0] = v1 ? (e1 & (KNN_MAX_TRAIN - 1)) : -1;
            out[(size_t)qi * 3 + 1] = v1 ? (e1 >> 13) : INT_MAX;
            out[(size_t)qi * 3 + 2] = v2 ? (e2 >> 13) : INT_MAX;
        }
    }
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8))) void k_knn2_single(
    const uint8_t *q, int nq, const uint8_t *t, int nt, int32_t *out)
{
    knn2_block_fp4(q, nq, t, nt, out, blockIdx.x * 256);
}

// batch: queries = F2 (current) keypoints of pair p, train = F1 (previous).  1-D grid of nbx
// blocks per pair, remapped so one pair's blocks share an XCD (and the L2 copy of the train
// descriptors they all stream)
#define KNN2_PAIRS_BODY(BLOCK)                                                                 \
    const int nbx = (fc + 255) >> 8;                                                           \
    const int id = xcd_remap(blockIdx.x, gridDim.x);                                           \
    const int p = id / nbx, bx = id - p * nbx;                                                 \
    const int a = f1[p], b = f2[p];                                                            \
    const int nq = counts[b], nt = counts[a];                                                  \
    if (bx * 256 >= nq) return;                                                                \
    BLOCK(desc + (size_t)b * fc * 32, nq, desc + (size_t)a * fc * 32, nt,                      \
          out + (size_t)p * fc * 3, bx * 256);
// fp4: 128 VGPRs (4 waves per SIMD; two dwords spill outside the train loop)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8))) void k_knn2_pairs(
    const uint8_t *desc, const int32_t *counts, int fc, const int32_t *f1, const int32_t *f2,
    int32_t *out)
{
    KNN2_PAIRS_BODY(knn2_block_fp4)
}

// ---------------------------------------------------------------------------
// SearchForInitialization
// ---------------------------------------------------------------------------
// LDS image of F2's level-0 keypoints: x, y, index
struct F2Key {
    float x, y;
    int idx;
};

#ifndef INIT_QPW
#define INIT_QPW 8  // queries per wave in k_init_cands_pairs (4: +7% there)
#endif
#ifndef INIT_QPW_SINGLE
#define INIT_QPW_SINGLE 4  // ... in k_init_cands_single (B = 1: twice the blocks, -4 us)
#endif
#define INIT_F2_CAP 4608  // host-data path bound (frame capacity at 4000 features)

// one 256-thread block: load F2 level-0 keys to LDS, then each wave handles INIT_QPW queries
// force-inlined: as a called function its pointer arguments would be generic (flat_ loads
// and stores, which also count in lgkmcnt)
// dynamic LDS of init_cands_block: 2 f2cap keys (16-byte padded), + f2cap descriptor rows
// with LDSD when that fits 64 KB
__host__ __device__ constexpr size_t init_cands_keys_bytes(int f2cap)
{
    return ((size_t)2 * f2cap * sizeof(F2Key) + 15) & ~(size_t)15;
}
#ifndef ORBG_INIT_LDSD
#define ORBG_INIT_LDSD 1  // the single-pair entry (B = 1); 0: descriptors from global memory (A/B)
#endif
__host__ __device__ constexpr bool init_cands_lds(int f2cap)
{
    return ORBG_INIT_LDSD && init_cands_keys_bytes(f2cap) + (size_t)f2cap * 32 <= 65536;
}

// LDSD: F2's descriptors (the first f2cap rows) are staged in LDS after the keys, so the
// candidate loop's Hamming distances read LDS instead of one dependent global load per
// candidate (the host takes it when 2 f2cap keys + f2cap rows fit, init_cands_lds)
template <bool LDSD, int QPW>
__device__ __forceinline__ void init_cands_block(const orbg_keypoint *__restrict__ k1,
                                 const uint8_t *__restrict__ d1, int n1,
                                 const orbg_keypoint *__restrict__ k2,
                                 const uint8_t *__restrict__ d2, int n2, orbg_bounds b,
                                 const float *__restrict__ prev, int prev_stride, int window,
                                 unsigned long long *__restrict__ topk, int32_t *__restrict__ topn,
                                 int qbase, int f2cap)
{
    // F2's level-0 keys (dynamic LDS, 2 x f2cap entries: batch: level-0 capacity; host-data
    // path: n2), counting-sorted by grid column PosInGrid-x (Frame.cc:292-307): a query's
    // window spans columns cx0..cx1 only, so it scans just those keys (the K-list order is
    // (distance, grid order, index), independent of the scan order)
    extern __shared__ __attribute__((aligned(16))) F2Key f2mem[];
    F2Key *f2raw = f2mem, *f2 = f2mem + f2cap;
    uint4 *d2l = (uint4 *)((uint8_t *)f2mem + init_cands_keys_bytes(f2cap));  // LDSD
    __shared__ int nf2;
    __shared__ int colstart[ORBG_GRID_COLS + 1];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const GridPrm g = grid_prm(b);
    if (tid == 0) nf2 = 0;
    if (tid <= ORBG_GRID_COLS) colstart[tid] = 0;
    __syncthreads();
    // batch: level-major output, every level-0 key sits below f2cap = level-0 capacity
    const int n2s = min(n2, f2cap);
    if (LDSD) {
        // rows 0 .. n2s-1, 16-byte words, four loads in flight per thread
        const uint4 *src = (const uint4 *)d2;
        for (int i0 = 0; i0 < 2 * n2s; i0 += 4 * 256) {
            uint4 v[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int i = i0 + u * 256 + tid;
                v[u] = src[i < 2 * n2s ? i : 0];
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int i = i0 + u * 256 + tid;
                if (i < 2 * n2s) d2l[i] = v[u];
            }
        }
    }
    for (int i = tid; i < n2s; i += 256) {
        const orbg_keypoint kp = k2[i];
        if (kp.octave == 0) {
            const int px = (int)roundf((kp.x - g.min_x) * g.inv_w);
            if (px < 0 || px >= ORBG_GRID_COLS) continue;  // outside the grid: never a candidate
            const int s = atomicAdd(&nf2, 1);
            if (s < f2cap) {
                f2raw[s] = F2Key{kp.x, kp.y, i};
                atomicAdd(&colstart[px + 1], 1);
            }
        }
    }
    __syncthreads();
    const int m = min(nf2, f2cap);
    if (wv == 0) {  // 64 columns: one wave's inclusive scan
        const int c = colstart[lane + 1];
        const int incl = wave_incl_scan(c);
        colstart[lane + 1] = incl;
    }
    __syncthreads();
    __shared__ int cursor[ORBG_GRID_COLS];
    if (tid < ORBG_GRID_COLS) cursor[tid] = colstart[tid];
    __syncthreads();
    for (int j = tid; j < m; j += 256) {
        const F2Key fk = f2raw[j];
        const int px = (int)roundf((fk.x - g.min_x) * g.inv_w);
        f2[atomicAdd(&cursor[px], 1)] = fk;
    }
    __syncthreads();
    // queries: 16-lane groups, 4 queries per wave at a time (~50 candidates per query: a
    // 16-way split keeps every lane busy and the K-round merge is 4 shuffle steps deep)
    const float r = (float)window;
    const int grp = lane >> 4, sub = lane & 15;
    for (int qq = 0; qq < QPW; qq += 4) {
        const int i1 = qbase + wv * QPW + qq + grp;
        bool act = i1 < n1;
        if (act && k1[i1].octave > 0) {
            if (sub == 0) topn[i1] = -1;  // not a query
            act = false;
        }
        if (!__any(act)) continue;
        unsigned long long loc[ORBG_MATCH_TOPK];
#pragma unroll
        for (int k = 0; k < ORBG_MATCH_TOPK; k++) loc[k] = ~0ull;
        int cnt = 0;
        if (act) {
            const Window w = make_window(g, prev[(size_t)i1 * prev_stride],
                                         prev[(size_t)i1 * prev_stride + 1], r);
            uint32_t qd[8];
            {
                const uint4 *p = (const uint4 *)(d1 + (size_t)i1 * 32);
                const uint4 a = p[0], c = p[1];
                qd[0] = a.x; qd[1] = a.y; qd[2] = a.z; qd[3] = a.w;
                qd[4] = c.x; qd[5] = c.y; qd[6] = c.z; qd[7] = c.w;
            }
            if (!w.empty) {
                const int j0 = colstart[w.cx0], j1 = colstart[w.cx1 + 1];
                for (int j = j0 + sub; j < j1; j += 16) {
                    const F2Key fk = f2[j];
                    const int ord = cand_order(g, w, fk.x, fk.y);
                    if (ord < 0) continue;
                    const int d = LDSD ? hamming8(qd, (const uint32_t *)(d2l + 2 * fk.idx))
                                       : hamming8(qd, (const uint32_t *)(d2 + (size_t)fk.idx * 32));
                    unsigned long long key = ((unsigned long long)d << 32) |
                                             ((unsigned long long)ord << 20) | (unsigned)fk.idx;
                    cnt++;
#pragma unroll
                    for (int k = 0; k < ORBG_MATCH_TOPK; k++) {
                        const unsigned long long lo = key < loc[k] ? key : loc[k];
                        const unsigned long long hi = key < loc[k] ? loc[k] : key;
                        loc[k] = lo;
                        key = hi;
                    }
                }
            }
        }
        cnt = row16_sum(cnt);
        // merge: K rounds of group-min over the lanes' sorted heads
        int head = 0;
        unsigned long long *out = topk + (size_t)i1 * ORBG_MATCH_TOPK;
        for (int k = 0; k < ORBG_MATCH_TOPK; k++) {
            unsigned long long mine = ~0ull;
#pragma unroll
            for (int h = 0; h < ORBG_MATCH_TOPK; h++)
                if (h == head) mine = loc[h];
            const unsigned long long mn = row16_min_u64(mine);
            if (mn != ~0ull && mine == mn) head++;  // keys are unique (index in low bits)
            if (act && sub == 0) out[k] = mn;
        }
        if (act && sub == 0) topn[i1] = cnt;
    }
}

template <bool LDSD>
__global__ __launch_bounds__(256) void k_init_cands_single(
    const orbg_keypoint *k1, const uint8_t *d1, int n1, const orbg_keypoint *k2,
    const uint8_t *d2, int n2, orbg_bounds b, const float *prev, int window,
    unsigned long long *topk, int32_t *topn)
{
    init_cands_block<LDSD, INIT_QPW_SINGLE>(k1, d1, n1, k2, d2, n2, b, prev, 2, window, topk, topn,
                                            blockIdx.x * 4 * INIT_QPW_SINGLE, n2);
}

// batch: F1 = frame f1[p] (its keypoints are vbPrevMatched), F2 = frame f2[p]
template <bool LDSD>
__global__ __launch_bounds__(256) void k_init_cands_pairs(
    const orbg_keypoint *kps, const uint8_t *desc, const int32_t *counts, int fc,
    const int32_t *f1, const int32_t *f2, orbg_bounds b, int window, unsigned long long *topk,
    int32_t *topn, int cap)
{
    // queries are level-0 keypoints: indices below the level-0 capacity
    const int nbx = (cap + 4 * INIT_QPW - 1) / (4 * INIT_QPW);
    const int id = xcd_remap(blockIdx.x, gridDim.x);
    const int p = id / nbx, bx = id - p * nbx;
    const int a = f1[p], c = f2[p];
    const int n1 = counts[a], n2 = counts[c];
    const int qbase = bx * 4 * INIT_QPW;
    if (qbase >= n1) return;
    const orbg_keypoint *k1 = kps + (size_t)a * fc;
    // extractor output is level-major: a block whose first query is above level 0 has no
    // SearchForInitialization query (octave > 0 only, ORBmatcher.cc:500-502)
    if (k1[qbase].octave > 0) {
        for (int i = qbase + threadIdx.x; i < min(n1, qbase + 4 * INIT_QPW); i += 256)
            topn[(size_t)p * fc + i] = -1;
        return;
    }
    // vbPrevMatched = F1.mvKeysUn[i].pt: read x, y straight out of the keypoint records
    init_cands_block<LDSD, INIT_QPW>(k1, desc + (size_t)a * fc * 32, n1, kps + (size_t)c * fc,
                     desc + (size_t)c * fc * 32, n2, b, (const float *)k1,
                     (int)(sizeof(orbg_keypoint) / sizeof(float)), window,
                     topk + (size_t)p * fc * ORBG_MATCH_TOPK, topn + (size_t)p * fc, qbase, cap);
}

// prev stride: the batch path reads x,y out of orbg_keypoint records (stride 7 floats)
#define RESOLVE_CHUNK 64
#define RESOLVE_N2_CAP 4608  // n1, n2 <= frame capacity (4000 features + 8 x 3)

// LDS of one resolver, dynamic: only keypoint indices < cap are held.  SearchForInit-
// ialization reads level-0 keypoints only (queries: octave 0; candidates:
// GetFeaturesInArea(.., 0, 0)), and the batch extractor's output is level-major, so the
// batch path uses cap = level-0 capacity (~440 at 2000 features) instead of the frame
// capacity; the host-data path uses cap = max(n1, n2).  vMatchedDistance is u16 (sentinel
// 0xFFFF > any distance), match indices i16.
struct ResolveShared {
    unsigned long long (*chunk)[RESOLVE_CHUNK * ORBG_MATCH_TOPK];
    int (*chunkn)[RESOLVE_CHUNK];
    int nbuf;  // chunk buffers: 2 (double buffer, wave 1 prefetches) or every chunk (preloaded)
    int *hsize;
    int *nmp;
    float *ang1, *ang2;
    uint16_t *mdist;
    int16_t *m21, *m12;
    int8_t *hbin;
    int32_t *owner;  // lowest applying lane of a speculative round (64 = none)
};

#define RESOLVE_CHUNK_BYTES (RESOLVE_CHUNK * ORBG_MATCH_TOPK * 8 + RESOLVE_CHUNK * 4)
#define RESOLVE_FIXED_BYTES (32 * 4 + 16)

// Every chunk's candidate lists preloaded into LDS up front (all loads in flight at once)
// when the level-0 capacity is at most RESOLVE_PRELOAD_CAP queries, instead of wave 1's
// per-chunk prefetch (two dependent global round trips per chunk on the sequential walk's
// path).  RESOLVE_PRELOAD: 0 never (default: 1 measured a tie at B = 1, 2 +5% on the batch
// resolver, profiles/r05p_single_ab.txt), 1 the single-pair entry (B = 1), 2 also the batch.
#ifndef RESOLVE_PRELOAD
#define RESOLVE_PRELOAD 0
#endif
#define RESOLVE_PRELOAD_CAP 1024

__host__ __device__ constexpr int resolve_nbuf(int cap, bool single)
{
    return (RESOLVE_PRELOAD >= (single ? 1 : 2) && cap <= RESOLVE_PRELOAD_CAP)
               ? (cap + RESOLVE_CHUNK - 1) / RESOLVE_CHUNK > 2 ? (cap + RESOLVE_CHUNK - 1) / RESOLVE_CHUNK : 2
               : 2;
}

__host__ __device__ constexpr size_t resolve_lds_bytes(int cap, int nbuf)
{
    return (size_t)nbuf * RESOLVE_CHUNK_BYTES + RESOLVE_FIXED_BYTES + (size_t)cap * 8 +
           (((size_t)cap * 7 + 15) & ~(size_t)15) + (size_t)cap * 4;
}

__device__ __forceinline__ ResolveShared resolve_layout(uint8_t *base, int cap, int nbuf)
{
    ResolveShared S;
    S.nbuf = nbuf;
    S.chunk = (unsigned long long(*)[RESOLVE_CHUNK * ORBG_MATCH_TOPK])base;
    base += (size_t)nbuf * RESOLVE_CHUNK * ORBG_MATCH_TOPK * 8;
    S.chunkn = (int(*)[RESOLVE_CHUNK])base;
    base += (size_t)nbuf * RESOLVE_CHUNK * 4;
    S.hsize = (int *)base;
    base += 32 * 4;
    S.nmp = (int *)base;
    base += 16;
    S.ang1 = (float *)base;
    S.ang2 = S.ang1 + cap;
    base += (size_t)cap * 8;
    S.mdist = (uint16_t *)base;
    S.m21 = (int16_t *)(S.mdist + cap);
    S.m12 = S.m21 + cap;
    S.hbin = (int8_t *)(S.m12 + cap);
    S.owner = (int32_t *)(base + (((size_t)cap * 7 + 15) & ~(size_t)15));
    return S;
}

// developer builds: cycle counts of the resolver's parts (thread 0, i.e. wave 0's lane 0):
// [0] init, [1] chunk walks (wave 0), [2] of which rescans, [3] chunk-end barriers, [4] tail,
// [5] speculative rounds, [6] rescans, [7] resolver calls (orbg_dev_resolve_prof)
#ifdef ORBG_DEV_KNOBS
__device__ unsigned long long g_rprof[8];
#define RP_NOW() __builtin_readcyclecounter()
#define RP_ADD(k, v)                                                                         \
    do {                                                                                     \
        if (threadIdx.x == 0) atomicAdd(&g_rprof[k], (unsigned long long)(v));               \
    } while (0)
#else
#define RP_NOW() 0ull
#define RP_ADD(k, v) \
    do {             \
    } while (0)
#endif

// exact fallback: sequential-scan semantics, wave-parallel
__device__ void rescan(const orbg_keypoint *k2, const uint8_t *d2, int n2, const GridPrm &g,
                       const Window &w, const uint32_t qd[8], const uint16_t *mdist, int *best,
                       int *best2, int *bidx)
{
    const int lane = threadIdx.x & 63;
    unsigned long long m1 = ~0ull, m2 = ~0ull;
    for (int j = lane; j < n2; j += 64) {
        const orbg_keypoint kp = k2[j];
        if (kp.octave != 0) continue;
        const int ord = cand_order(g, w, kp.x, kp.y);
        if (ord < 0) continue;
        const int d = hamming8(qd, (const uint32_t *)(d2 + (size_t)j * 32));
        if ((int)mdist[j] <= d) continue;
        const unsigned long long key =
            ((unsigned long long)d << 32) | ((unsigned long long)ord << 20) | (unsigned)j;
        if (key < m1) {
            m2 = m1;
            m1 = key;
        } else if (key < m2) {
            m2 = key;
        }
    }
    const unsigned long long a = wave_min_u64(m1);
    unsigned long long rest = (m1 == a) ? m2 : m1;
    const unsigned long long b = wave_min_u64(rest);
    *best = a == ~0ull ? INT_MAX : (int)(a >> 32);
    *bidx = a == ~0ull ? -1 : (int)(a & 0xFFFFF);
    *best2 = b == ~0ull ? INT_MAX : (int)(b >> 32);
}

// Two waves per pair.  Wave 0's lane 0 walks the queries in index order (the
// reference's sequential semantics) over candidate lists in LDS while wave 1 prefetches
// the next chunk of lists (double buffer); wave 0 runs the exact rescan for a query
// whose K-list the vMatchedDistance filter exhausted.
#define RESOLVE_T 128

__device__ void init_resolve_block(ResolveShared &S, int cap, const orbg_keypoint *__restrict__ k1,
                                   const uint8_t *__restrict__ d1, int n1,
                                   const orbg_keypoint *__restrict__ k2,
                                   const uint8_t *__restrict__ d2, int n2, orbg_bounds b,
                                   const float *prev, int prev_stride, int window, float nnratio,
                                   int check_ori, const unsigned long long *__restrict__ topk,
                                   const int32_t *__restrict__ topn, int32_t *__restrict__ m12,
                                   int32_t *__restrict__ nm_out, float *prev_out)
{
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int n1c = min(n1, cap), n2c = min(n2, cap);  // indices any query / candidate can have
    [[maybe_unused]] unsigned long long rp_t = RP_NOW();
    RP_ADD(7, 1);
    for (int i0 = 0; i0 < n2c; i0 += 4 * RESOLVE_T) {
        float a[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int i = i0 + u * RESOLVE_T + tid;
            a[u] = i < n2c ? k2[i].angle : 0.f;
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int i = i0 + u * RESOLVE_T + tid;
            if (i < n2c) {
                S.mdist[i] = 0xFFFF;
                S.m21[i] = -1;
                S.ang2[i] = a[u];
                S.owner[i] = 64;
            }
        }
    }
    for (int i0 = 0; i0 < n1c; i0 += 4 * RESOLVE_T) {
        float a[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int i = i0 + u * RESOLVE_T + tid;
            a[u] = i < n1c ? k1[i].angle : 0.f;
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int i = i0 + u * RESOLVE_T + tid;
            if (i < n1c) {
                S.hbin[i] = -1;
                S.m12[i] = -1;
                S.ang1[i] = a[u];
            }
        }
    }
    if (tid < HISTO_LENGTH) S.hsize[tid] = 0;
    if (tid == 0) *S.nmp = 0;
    const GridPrm g = grid_prm(b);
    const float factor = 1.0f / HISTO_LENGTH;
    // lane 0 of wave 0: sequential state update for query i1
    auto apply = [&](int i1, int bestDist, int bestDist2, int bestIdx2) {
        if (bestDist <= TH_LOW && bestDist < (float)bestDist2 * nnratio) {
            const int old = S.m21[bestIdx2];
            const float rot0 = S.ang1[i1] - S.ang2[bestIdx2];
            if (old >= 0) {
                S.m12[old] = -1;
                (*S.nmp)--;
            }
            S.m12[i1] = (int16_t)bestIdx2;
            S.m21[bestIdx2] = (int16_t)i1;
            S.mdist[bestIdx2] = (uint16_t)bestDist;
            (*S.nmp)++;
            if (check_ori) {
                float rot = rot0;
                if (rot < 0.0f) rot += 360.0f;
                int bin = (int)roundf(rot * factor);
                if (bin == HISTO_LENGTH) bin = 0;
                S.hbin[i1] = (int8_t)bin;
                S.hsize[bin]++;
            }
        }
    };
    // wave 1: load chunk c into buffer c & 1 (lists only when the chunk has a live query)
    const int nchunks = (n1c + RESOLVE_CHUNK - 1) / RESOLVE_CHUNK;
    const bool preload = S.nbuf >= nchunks && S.nbuf > 2;
    auto prefetch = [&](int c) {
        const int c0 = c * RESOLVE_CHUNK;
        if (c0 >= n1c) return;
        const int cn = min(RESOLVE_CHUNK, n1c - c0);
        const int t = lane < cn ? topn[c0 + lane] : -1;
        S.chunkn[c % S.nbuf][lane] = t;
        if (__ballot(t > 0) == 0ull) return;
        unsigned long long e[ORBG_MATCH_TOPK];
#pragma unroll
        for (int u = 0; u < ORBG_MATCH_TOPK; u++) {
            const int i = u * 64 + lane;
            e[u] = i < cn * ORBG_MATCH_TOPK ? topk[(size_t)c0 * ORBG_MATCH_TOPK + i] : ~0ull;
        }
#pragma unroll
        for (int u = 0; u < ORBG_MATCH_TOPK; u++) S.chunk[c % S.nbuf][u * 64 + lane] = e[u];
    };
    if (preload) {
        // every list at once: both waves, 8 unconditional loads in flight per batch (entries
        // past a query's count are never read)
        unsigned long long *flat = &S.chunk[0][0];
        const int nk = n1c * ORBG_MATCH_TOPK;
        for (int i0 = 0; i0 < nk; i0 += 8 * RESOLVE_T) {
            unsigned long long e[8];
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const int i = min(i0 + u * RESOLVE_T + tid, nk - 1);
                e[u] = topk[i];
            }
#pragma unroll
            for (int u = 0; u < 8; u++)
                if (i0 + u * RESOLVE_T + tid < nk) flat[i0 + u * RESOLVE_T + tid] = e[u];
        }
        int *flatn = &S.chunkn[0][0];
        for (int i = tid; i < nchunks * RESOLVE_CHUNK; i += RESOLVE_T) flatn[i] = i < n1c ? topn[i] : -1;
    } else if (wv == 1) {
        prefetch(0);
    }
    __syncthreads();
    {
        const unsigned long long t = RP_NOW();
        RP_ADD(0, t - rp_t);
        rp_t = t;
    }
    int nm_reg = 0;  // wave 0: this resolver's committed-match count (lane-uniform)
    for (int c = 0; c < nchunks; c++) {
        if (wv == 1) {
            if (!preload) prefetch(c + 1);
        } else {
            // Speculative parallel walk, one query per lane (see track_kernels.hip): each
            // pending lane picks best / second from its K-list against the current
            // vMatchedDistance; a pick is exact unless an earlier pending lane that applies
            // rewrites vMatchedDistance of a keypoint at or before the lane's last consulted
            // list position.  owner[i2] (lowest applying lane) finds the first such lane l*;
            // lanes below l* and below the first exhausted K-list commit (their best
            // keypoints are distinct, so their steals and writes are independent), the rest
            // go again.
            const int c0 = c * RESOLVE_CHUNK, cn = min(RESOLVE_CHUNK, n1c - c0);
            const int *cnt = S.chunkn[c % S.nbuf];
            const unsigned long long *lists = S.chunk[c % S.nbuf];
            const int total = lane < cn ? cnt[lane] : 0;
            unsigned long long e[ORBG_MATCH_TOPK];
#pragma unroll
            for (int k = 0; k < ORBG_MATCH_TOPK; k++) e[k] = lists[lane * ORBG_MATCH_TOPK + k];
            const int kk = min(total, ORBG_MATCH_TOPK);
            const int i1 = c0 + lane;
            const float a1 = S.ang1[min(i1, cap - 1)];  // vbPrevMatched's keypoint angle
            unsigned long long pending = __ballot(total > 0);
            while (pending) {
                RP_ADD(5, 1);
                const bool pend = (pending >> lane) & 1ull;
                int found = 0, bd = INT_MAX, bd2 = INT_MAX, bi = -1, lastpos = kk - 1;
                // every list entry's vMatchedDistance read at once (indices clamped: entries
                // past the list are read and ignored), then the in-order pick on registers --
                // not one dependent LDS round trip per consulted entry
                int md[ORBG_MATCH_TOPK];
#pragma unroll
                for (int k = 0; k < ORBG_MATCH_TOPK; k++)
                    md[k] = S.mdist[min((int)(e[k] & 0xFFFFF), cap - 1)];
#pragma unroll
                for (int k = 0; k < ORBG_MATCH_TOPK; k++) {
                    if (!pend || k >= kk || found >= 2) continue;
                    const int d = (int)(e[k] >> 32), i2 = (int)(e[k] & 0xFFFFF);
                    if (md[k] <= d) continue;
                    if (found == 0) {
                        bd = d;
                        bi = i2;
                    } else {
                        bd2 = d;
                    }
                    if (++found == 2) lastpos = k;
                }
                const bool resc = pend && found < 2 && total > ORBG_MATCH_TOPK;
                const bool app = pend && !resc && bd <= TH_LOW && bd < (float)bd2 * nnratio;
                // the commit's reads of the pick, issued before the conflict check: vnMatches21
                // changes only in commits, and committing lanes have distinct picks
                const int bic = max(bi, 0);
                const int m21_pre = S.m21[bic];
                const float a2 = S.ang2[bic];
                if (app) atomicMin(&S.owner[bi], lane);
                wave_sync_lds();
                bool conf = false;
                int ow[ORBG_MATCH_TOPK];
#pragma unroll
                for (int k = 0; k < ORBG_MATCH_TOPK; k++)
                    ow[k] = S.owner[min((int)(e[k] & 0xFFFFF), cap - 1)];
#pragma unroll
                for (int k = 0; k < ORBG_MATCH_TOPK; k++)
                    if (pend && k < kk && k <= lastpos && ow[k] < lane) conf = true;
                const unsigned long long cm = __ballot(conf), rm = __ballot(resc);
                const int lc = cm ? __builtin_ctzll(cm) : 64, lr = rm ? __builtin_ctzll(rm) : 64;
                const int lstar = min(lc, lr);
                const unsigned long long below = lstar >= 64 ? ~0ull : ((1ull << lstar) - 1ull);
                const bool commit = app && lane < lstar;
                if (app) S.owner[bi] = 64;
                bool stole = false;
                if (commit) {
                    const int old = m21_pre;
                    if (old >= 0) {
                        S.m12[old] = -1;
                        stole = true;
                    }
                    S.m12[i1] = (int16_t)bi;
                    S.m21[bi] = (int16_t)i1;
                    S.mdist[bi] = (uint16_t)bd;
                    if (check_ori) {
                        float rot = a1 - a2;
                        if (rot < 0.0f) rot += 360.0f;
                        int bin = (int)roundf(rot * factor);
                        if (bin == HISTO_LENGTH) bin = 0;
                        S.hbin[i1] = (int8_t)bin;
                        atomicAdd(&S.hsize[bin], 1);
                    }
                }
                nm_reg += __popcll(__ballot(commit)) - __popcll(__ballot(stole));
                pending &= ~below;
                wave_sync_lds();
                if (lr < 64 && lr == lstar) {
                    [[maybe_unused]] const unsigned long long rs0 = RP_NOW();
                    RP_ADD(6, 1);
                    // K-list exhausted: exact rescan of query c0 + lr against the committed state
                    const int q1 = c0 + lr;
                    const float px = prev[(size_t)q1 * prev_stride];
                    const float py = prev[(size_t)q1 * prev_stride + 1];
                    const Window w = make_window(g, px, py, (float)window);
                    uint32_t qd[8];
                    const uint32_t *qp = (const uint32_t *)(d1 + (size_t)q1 * 32);
#pragma unroll
                    for (int k = 0; k < 8; k++) qd[k] = qp[k];
                    int bestDist, bestDist2, bestIdx2;
                    rescan(k2, d2, n2c, g, w, qd, S.mdist, &bestDist, &bestDist2, &bestIdx2);
                    if (lane == 0) apply(q1, bestDist, bestDist2, bestIdx2);
                    pending &= ~(1ull << lr);
                    wave_sync_lds();
                    RP_ADD(2, RP_NOW() - rs0);
                }
            }
        }
        {
            const unsigned long long t = RP_NOW();
            RP_ADD(1, t - rp_t);
            rp_t = t;
        }
        __syncthreads();
        {
            const unsigned long long t = RP_NOW();
            RP_ADD(3, t - rp_t);
            rp_t = t;
        }
    }
    if (tid == 0) *S.nmp += nm_reg;
    __syncthreads();
    int nmatches = *S.nmp;
    if (check_ori) {
        __shared__ int ind[3];
        if (tid == 0) {
            // ComputeThreeMaxima (:1800-1841)
            int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
            for (int i = 0; i < HISTO_LENGTH; i++) {
                const int s = S.hsize[i];
                if (s > max1) {
                    max3 = max2; max2 = max1; max1 = s;
                    ind3 = ind2; ind2 = ind1; ind1 = i;
                } else if (s > max2) {
                    max3 = max2; max2 = s;
                    ind3 = ind2; ind2 = i;
                } else if (s > max3) {
                    max3 = s;
                    ind3 = i;
                }
            }
            if (max2 < 0.1f * (float)max1) {
                ind2 = -1;
                ind3 = -1;
            } else if (max3 < 0.1f * (float)max1) {
                ind3 = -1;
            }
            ind[0] = ind1;
            ind[1] = ind2;
            ind[2] = ind3;
        }
        __syncthreads();
        int removed = 0;
        for (int i = tid; i < n1c; i += RESOLVE_T) {
            const int bn = S.hbin[i];
            if (bn < 0 || bn == ind[0] || bn == ind[1] || bn == ind[2]) continue;
            if (S.m12[i] >= 0) {
                S.m12[i] = -1;
                removed++;
            }
        }
        removed = wave_isum(removed);
        __shared__ int rem2[2];
        if (lane == 0) rem2[wv] = removed;
        __syncthreads();
        nmatches -= rem2[0] + rem2[1];
    }
    __syncthreads();
    for (int i = tid; i < n1; i += RESOLVE_T) m12[i] = i < n1c ? S.m12[i] : -1;
    if (prev_out) {
        for (int i = tid; i < n1c; i += RESOLVE_T) {
            const int j = S.m12[i];
            if (j >= 0) {
                prev_out[2 * i] = k2[j].x;
                prev_out[2 * i + 1] = k2[j].y;
            }
        }
    }
    if (tid == 0) *nm_out = nmatches;
    RP_ADD(4, RP_NOW() - rp_t);
}

// prev_out, m12, nm may be host-mapped (the host entry's zero-copy outputs): written once each
__global__ __launch_bounds__(RESOLVE_T) void k_init_resolve_single(
    const orbg_keypoint *k1, const uint8_t *d1, int n1, const orbg_keypoint *k2,
    const uint8_t *d2, int n2, orbg_bounds b, const float *prev, float *prev_out, int window,
    float nnratio, int check_ori, const unsigned long long *topk, const int32_t *topn,
    int32_t *m12, int32_t *nm, int cap)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t rs_lds[];
    ResolveShared S = resolve_layout(rs_lds, cap, resolve_nbuf(cap, true));
    init_resolve_block(S, cap, k1, d1, n1, k2, d2, n2, b, prev, 2, window, nnratio, check_ori, topk,
                       topn, m12, nm, prev_out);
}

__global__ __launch_bounds__(RESOLVE_T) void k_init_resolve_pairs(
    const orbg_keypoint *kps, const uint8_t *desc, const int32_t *counts, int fc,
    const int32_t *f1, const int32_t *f2, orbg_bounds b, int window, float nnratio,
    int check_ori, const unsigned long long *topk, const int32_t *topn, int32_t *m12,
    int32_t *nm, int cap)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t rs_lds[];
    ResolveShared S = resolve_layout(rs_lds, cap, resolve_nbuf(cap, false));
    const int p = blockIdx.x;
    const int a = f1[p], c = f2[p];
    const orbg_keypoint *k1 = kps + (size_t)a * fc;
    init_resolve_block(S, cap, k1, desc + (size_t)a * fc * 32, counts[a], kps + (size_t)c * fc,
                      desc + (size_t)c * fc * 32, counts[c], b, (const float *)k1,
                      (int)(sizeof(orbg_keypoint) / sizeof(float)), window, nnratio, check_ori,
                      topk + (size_t)p * fc * ORBG_MATCH_TOPK, topn + (size_t)p * fc,
                      m12 + (size_t)p * fc, nm + p, nullptr);
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
#define PL(prof, st, name, ...)                                                            \
    do {                                                                                   \
        if (prof_skip_name(name)) break;                                                   \
        hipEvent_t a_ = nullptr;                                                           \
        prof_begin(prof, st, name, &a_);                                                   \
        __VA_ARGS__;                                                                       \
        prof_end(prof, st, name, a_);                                                      \
    } while (0)

// vnMatches12 of every pair into a caller buffer [npairs][frame_cap]: entries past the
// pair's first-frame keypoint count are -1 (the match kernels leave them unwritten)
__global__ __launch_bounds__(256) void k_match_export(const int32_t *__restrict__ m12,
                                                      const int32_t *__restrict__ f1,
                                                      const int32_t *__restrict__ counts,
                                                      int frame_cap, int npairs,
                                                      int32_t *__restrict__ out)
{
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)npairs * frame_cap) return;
    const int p = (int)(i / frame_cap), k = (int)(i - (int64_t)p * frame_cap);
    out[i] = k < counts[f1[p]] ? m12[i] : -1;
}

int launch_match_export(hipStream_t st, const int32_t *m12, const int32_t *f1,
                        const int32_t *counts, int frame_cap, int npairs, int32_t *out)
{
    const int64_t n = (int64_t)npairs * frame_cap;
    if (n <= 0) return ORBG_OK;
    hipLaunchKernelGGL(k_match_export, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, m12,
                       f1, counts, frame_cap, npairs, out);
    return hipGetLastError() == hipSuccess ? ORBG_OK : ORBG_EIO;
}

int launch_knn2(hipStream_t st, const uint8_t *q, int nq, const uint8_t *t, int nt, int32_t *out,
                void *prof)
{
    if (nt >= KNN_MAX_TRAIN) return ORBG_ENOTSUP;  // caller chunks the train set
    PL(prof, st, "knn2",
       hipLaunchKernelGGL(k_knn2_single,
                          dim3((nq + 255) / 256), dim3(256), 0, st, q, nq, t, nt, out));
    return hipGetLastError() == hipSuccess ? ORBG_OK : ORBG_EIO;
}

int launch_match_pairs(hipStream_t st, hipStream_t aux, hipEvent_t evf, hipEvent_t evj,
                       const uint8_t *desc, const orbg_keypoint *kps,
                       const int32_t *counts, int fc, const int32_t *d_f1, const int32_t *d_f2,
                       int npairs, orbg_bounds b, int window, float nnratio, int check_ori,
                       int32_t *knn, int32_t *m12, int32_t *nm, uint32_t *topk, int32_t *topk_n,
                       void *prof, int serial, int cap0)
{
    // cap0 = level-0 capacity: every index SearchForInitialization touches is below it
    if (fc > RESOLVE_N2_CAP || fc > (1 << 20) || cap0 > fc) return ORBG_ENOTSUP;
    PL(prof, st, "init_cands",
       // descriptors from global memory: at batch the staging measured +3% (r05ae)
       hipLaunchKernelGGL(k_init_cands_pairs<false>,
                          dim3((cap0 + 4 * INIT_QPW - 1) / (4 * INIT_QPW) * npairs), dim3(256),
                          init_cands_keys_bytes(cap0), st, kps, desc, counts, fc, d_f1, d_f2, b,
                          window, (unsigned long long *)topk, topk_n, cap0));
    // knn2 (VALU bound) on `aux` beside init_resolve (one sequential workgroup per pair);
    // serial == 1 (orbg_set_serial: isolated kernel timing) keeps it on `st`
    if (serial) aux = st;
    if (hipEventRecord(evf, st) != hipSuccess || hipStreamWaitEvent(aux, evf, 0) != hipSuccess)
        return ORBG_EIO;
    PL(prof, aux, "knn2",
       hipLaunchKernelGGL(k_knn2_pairs,
                          dim3((fc + 255) / 256 * npairs), dim3(256), 0, aux, desc, counts, fc,
                          d_f1, d_f2, knn));
    if (hipEventRecord(evj, aux) != hipSuccess) return ORBG_EIO;
    if (resolve_lds_bytes(cap0, resolve_nbuf(cap0, false)) > 65536) {
        static bool pattr = false;  // a preloaded batch resolver past 64 KB of dynamic LDS
        if (!pattr) {
            if (hipFuncSetAttribute((const void *)k_init_resolve_pairs,
                                    hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)resolve_lds_bytes(RESOLVE_PRELOAD_CAP,
                                                           resolve_nbuf(RESOLVE_PRELOAD_CAP, false))) !=
                hipSuccess)
                return ORBG_EIO;
            pattr = true;
        }
    }
    PL(prof, st, "init_resolve",
       hipLaunchKernelGGL(k_init_resolve_pairs, dim3(npairs), dim3(RESOLVE_T),
                          resolve_lds_bytes(cap0, resolve_nbuf(cap0, false)), st, kps, desc,
                          counts, fc, d_f1, d_f2, b,
                          window, nnratio, check_ori, (const unsigned long long *)topk, topk_n,
                          m12, nm, cap0));
    if (hipStreamWaitEvent(st, evj, 0) != hipSuccess) return ORBG_EIO;
    return hipGetLastError() == hipSuccess ? ORBG_OK : ORBG_EIO;
}

// cap: 1 + the last level-0 index of either frame (every query / candidate index the
// search can touch: it reads level-0 keypoints only, ORBmatcher.cc:509-512, 1 <= cap <=
// max(n1, n2)); queries past it get no candidates and vnMatches12 = -1
#ifdef ORBG_DEV_KNOBS
// developer builds: read (and with reset, clear) the resolver cycle counters
extern "C" int orbg_dev_resolve_prof(unsigned long long out[8], int reset)
{
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rprof), sizeof(g_rprof)) != hipSuccess) return -5;
    if (reset) {
        const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_rprof), z, sizeof(z)) != hipSuccess) return -5;
    }
    return 0;
}
#endif

int launch_init_match_single(hipStream_t st, const orbg_keypoint *k1, const uint8_t *d1, int n1,
                             const orbg_keypoint *k2, const uint8_t *d2, int n2, orbg_bounds b,
                             const float *prev, float *prev_out, int32_t *m12, int32_t *nm,
                             int window, float nnratio,
                             int check_ori, uint32_t *topk, int32_t *topk_n, void *prof, int cap)
{
    const int nq = std::min(n1, cap), n2c = std::min(n2, cap);  // indices below cap
    if (n1 > RESOLVE_N2_CAP || n2 > RESOLVE_N2_CAP || n2 > INIT_F2_CAP) return ORBG_ENOTSUP;
    static bool attr = false;  // > 64 KB of dynamic LDS at the 4608-keypoint bound
    if (!attr) {
        if (hipFuncSetAttribute((const void *)k_init_resolve_single,
                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)std::max(resolve_lds_bytes(RESOLVE_N2_CAP, 2),
                                              resolve_lds_bytes(RESOLVE_PRELOAD_CAP,
                                                                resolve_nbuf(RESOLVE_PRELOAD_CAP, true)))) !=
                hipSuccess)
            return ORBG_EIO;
        attr = true;
    }
    PL(prof, st, "init_cands",
       if (init_cands_lds(std::max(n2c, 1)))
           hipLaunchKernelGGL(k_init_cands_single<true>,
                              dim3((nq + 4 * INIT_QPW_SINGLE - 1) / (4 * INIT_QPW_SINGLE)), dim3(256),
                              init_cands_keys_bytes(std::max(n2c, 1)) + (size_t)std::max(n2c, 1) * 32,
                              st, k1, d1, nq, k2, d2, n2c, b, prev, window,
                              (unsigned long long *)topk, topk_n);
       else
           hipLaunchKernelGGL(k_init_cands_single<false>,
                              dim3((nq + 4 * INIT_QPW_SINGLE - 1) / (4 * INIT_QPW_SINGLE)), dim3(256),
                              init_cands_keys_bytes(std::max(n2c, 1)), st, k1, d1, nq, k2, d2, n2c,
                              b, prev, window, (unsigned long long *)topk, topk_n));
    PL(prof, st, "init_resolve",
       hipLaunchKernelGGL(k_init_resolve_single, dim3(1), dim3(RESOLVE_T),
                          resolve_lds_bytes(cap, resolve_nbuf(cap, true)), st, k1, d1, n1, k2, d2,
                          n2, b, prev, prev_out, window,
                          nnratio, check_ori, (const unsigned long long *)topk, topk_n, m12, nm,
                          cap));
    return hipGetLastError() == hipSuccess ? ORBG_OK : ORBG_EIO;
}

}  // namespace orbg
