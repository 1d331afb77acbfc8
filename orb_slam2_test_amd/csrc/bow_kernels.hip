// bow_kernels.hip -- DBoW2 TemplatedVocabulary::transform(features, BowVector, FeatureVector,
// levelsup) (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1126-1189, 1220-1259) for a batch
// of frames on gfx950, as Frame::ComputeBoW (src/Frame.cc:532-539) calls it.
//
//   k_bow_words<G>   G lanes per descriptor (G >= the widest node): each descent step lane j
//                    reads child j's 64-byte BowSlot, Hamming-distances it, and the group
//                    takes min(d << 8 | j) -- strict <, first child wins, as the reference's
//                    loop; the winner's record already holds the next children range, so a
//                    level costs one dependent load.  Writes word / FeatureVector node /
//                    weight per feature.
//   k_bow_vectors    one workgroup per frame: (word, feature) keys of the non-stopped
//                    features bitonic-sorted in LDS = std::map order with per-word feature
//                    order; segment sums (addWeight) or first (addIfNotExist) per word, then
//                    the norm summed by one lane in word order (BowVector::normalize) so the
//                    doubles are bit-identical; then (node, feature) keys sorted the same way
//                    give FeatureVector's node list and per-node feature lists.
#include <hip/hip_runtime.h>

#include <cmath>

#include "../../include/orbg.h"
#include "bow_args.h"

#pragma clang fp contract(off)

namespace orbg {

void prof_begin(void *prof, hipStream_t s, const char *n, hipEvent_t *a);
void prof_end(void *prof, hipStream_t s, const char *n, hipEvent_t a);

#define BOW_THREADS 256

template <int G>
__global__ __launch_bounds__(BOW_THREADS) void k_bow_words(BowArgs A)
{
    constexpr int GPB = BOW_THREADS / G;
    const int64_t gid = (int64_t)blockIdx.x * GPB + threadIdx.x / G;
    const int lane = threadIdx.x % G;
    const int f = (int)(gid / A.cap), i = (int)(gid - (int64_t)f * A.cap);
    if (f >= A.nframes || i >= A.counts[f]) return;  // uniform per group
    const size_t fi = (size_t)f * A.cap + i;
    if (A.empty) {
        if (lane == 0) {
            A.fword[fi] = -1;
            A.fnode[fi] = 0;
            A.fweight[fi] = 0.0;
        }
        return;
    }
    const uint4 *fd = (const uint4 *)(A.desc + fi * 32);
    const uint4 q0 = fd[0], q1 = fd[1];
    int c0 = A.root_c0, c1 = A.root_c1, level = 0;
    int nid = 0, word = 0;
    double w = 0.0;
    while (true) {
        ++level;
        unsigned key = 0xFFFFFFFFu;
        int sc0 = 0, sc1 = 0, snode = 0, sword = 0;
        double sw = 0.0;
        if (lane < c1 - c0) {
            const uint4 *s = (const uint4 *)(A.slots + c0 + lane);
            const uint4 a = s[0], b = s[1];
            const int4 m = *(const int4 *)(s + 2);
            sw = *(const double *)(s + 3);
            const unsigned d = __popc(a.x ^ q0.x) + __popc(a.y ^ q0.y) + __popc(a.z ^ q0.z) +
                               __popc(a.w ^ q0.w) + __popc(b.x ^ q1.x) + __popc(b.y ^ q1.y) +
                               __popc(b.z ^ q1.z) + __popc(b.w ^ q1.w);
            key = d << 8 | lane;
            sc0 = m.x;
            sc1 = m.y;
            snode = m.z;
            sword = m.w;
        }
#pragma unroll
        for (int o = G / 2; o > 0; o >>= 1) key = min(key, (unsigned)__shfl_xor((int)key, o, G));
        const int win = key & 0xFF;
        const int n0 = __shfl(sc0, win, G), n1 = __shfl(sc1, win, G);
        const int wnode = __shfl(snode, win, G);
        if (level == A.nid_level) nid = wnode;
        if (n0 == n1) {  // isLeaf(): no children
            if (level < A.nid_level) nid = wnode;  // leaf above nid_level (see bow_oracle.c)
            word = __shfl(sword, win, G);
            w = __shfl(sw, win, G);
            break;
        }
        c0 = n0;
        c1 = n1;
    }
    if (lane == 0) {
        A.fword[fi] = w > 0 ? word : -1;
        A.fnode[fi] = nid;
        A.fweight[fi] = w;
    }
}

__device__ __forceinline__ int wave_incl_scan(int v)
{
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    return v;
}

// exclusive prefix of v over the workgroup; *total = sum (all threads)
__device__ __forceinline__ int block_exscan(int v, int *tmp, int *total)
{
    const int inc = wave_incl_scan(v);
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 63) tmp[wv] = inc;
    __syncthreads();
    int base = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < BOW_THREADS / 64; k++) {
        if (k < wv) base += tmp[k];
        tot += tmp[k];
    }
    __syncthreads();
    *total = tot;
    return base + inc - v;
}

__device__ void bitonic_sort(uint64_t *keys, int P)
{
    for (int k = 2; k <= P; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int t = threadIdx.x; t < P / 2; t += BOW_THREADS) {
                const int i = 2 * t - (t & (j - 1)), l = i + j;
                const uint64_t a = keys[i], b = keys[l];
                const bool up = (i & k) == 0;
                if ((a > b) == up) {
                    keys[i] = b;
                    keys[l] = a;
                }
            }
            __syncthreads();
        }
}

size_t bow_vectors_lds(int cap)
{
    int P = 256;
    while (P < cap) P <<= 1;
    return (size_t)P * 16;
}

__global__ __launch_bounds__(BOW_THREADS) void k_bow_vectors(BowArgs A)
{
    extern __shared__ __align__(16) uint8_t lds[];
    __shared__ int tmp[BOW_THREADS / 64];
    __shared__ double s_norm;
    const int f = blockIdx.x, tid = threadIdx.x;
    const int n = A.counts[f];
    int P = 256;
    while (P < n) P <<= 1;
    uint64_t *keys = (uint64_t *)lds;
    double *val = (double *)(lds + (size_t)P * 8);
    const size_t fb = (size_t)f * A.cap;
    const int E = P / BOW_THREADS, i0 = tid * E;
    const bool tf = A.weighting == ORBG_TF_IDF || A.weighting == ORBG_TF;
    const bool must = A.scoring != ORBG_DOT_PRODUCT;

    // ---- BowVector ----
    int mloc = 0;
    for (int i = tid; i < P; i += BOW_THREADS) {
        uint64_t k = ~0ull;
        if (i < n) {
            const int wd = A.fword[fb + i];
            if (wd >= 0) {
                k = (uint64_t)(uint32_t)wd << 32 | (uint32_t)i;
                mloc++;
            }
        }
        keys[i] = k;
    }
    int m;
    block_exscan(mloc, tmp, &m);
    bitonic_sort(keys, P);
    int heads = 0;
    for (int i = i0; i < i0 + E; i++)
        if (i < m && (i == 0 || (keys[i] >> 32) != (keys[i - 1] >> 32))) heads++;
    int nb;
    int out = block_exscan(heads, tmp, &nb);
    for (int i = i0; i < i0 + E; i++) {
        if (!(i < m && (i == 0 || (keys[i] >> 32) != (keys[i - 1] >> 32)))) continue;
        const uint32_t wd = (uint32_t)(keys[i] >> 32);
        double s = A.fweight[fb + (uint32_t)keys[i]];
        if (tf)  // addWeight in feature order; IDF / BINARY keep the first (addIfNotExist)
            for (int j = i + 1; j < m && (uint32_t)(keys[j] >> 32) == wd; j++)
                s += A.fweight[fb + (uint32_t)keys[j]];
        A.bow_words[fb + out] = (int32_t)wd;
        val[out] = s;
        out++;
    }
    __syncthreads();
    if (tid == 0) {
        double norm = 1.0;
        if (must) {
            double acc = 0.0;
            int k = 0;
            if (A.scoring == ORBG_L2_NORM) {
                for (; k + 8 <= nb; k += 8) {
                    double v[8];
#pragma unroll
                    for (int u = 0; u < 8; u++) v[u] = val[k + u];
#pragma unroll
                    for (int u = 0; u < 8; u++) acc += v[u] * v[u];
                }
                for (; k < nb; k++) acc += val[k] * val[k];
                acc = sqrt(acc);
            } else {
                for (; k + 8 <= nb; k += 8) {
                    double v[8];
#pragma unroll
                    for (int u = 0; u < 8; u++) v[u] = val[k + u];
#pragma unroll
                    for (int u = 0; u < 8; u++) acc += fabs(v[u]);
                }
                for (; k < nb; k++) acc += fabs(val[k]);
            }
            norm = acc > 0.0 ? acc : 1.0;
        } else if (tf && nb > 0) {
            norm = (double)nb;
        }
        s_norm = norm;
        A.nbow[f] = nb;
    }
    __syncthreads();
    const double norm = s_norm;
    const bool divide = (must && norm != 1.0) || (!must && tf);
    for (int k = tid; k < nb; k += BOW_THREADS) A.bow_weights[fb + k] = divide ? val[k] / norm : val[k];
    __syncthreads();

    // ---- FeatureVector ----
    for (int i = tid; i < P; i += BOW_THREADS) {
        uint64_t k = ~0ull;
        if (i < n && A.fword[fb + i] >= 0) k = (uint64_t)(uint32_t)A.fnode[fb + i] << 32 | (uint32_t)i;
        keys[i] = k;
    }
    __syncthreads();
    bitonic_sort(keys, P);
    heads = 0;
    for (int i = i0; i < i0 + E; i++)
        if (i < m && (i == 0 || (keys[i] >> 32) != (keys[i - 1] >> 32))) heads++;
    int nf;
    out = block_exscan(heads, tmp, &nf);
    int32_t *fo = A.fv_off + (size_t)f * (A.cap + 1);
    for (int i = i0; i < i0 + E; i++) {
        if (i >= m) break;
        A.fv_feats[fb + i] = (int32_t)(uint32_t)keys[i];
        if (i == 0 || (keys[i] >> 32) != (keys[i - 1] >> 32)) {
            A.fv_nodes[fb + out] = (int32_t)(keys[i] >> 32);
            fo[out] = i;
            out++;
        }
    }
    if (tid == 0) {
        fo[nf] = m;
        A.nfv[f] = nf;
    }
}

int launch_bow(hipStream_t st, const BowArgs &A, void *prof)
{
    if (A.nframes <= 0) return ORBG_OK;
    hipEvent_t ev = nullptr;
    prof_begin(prof, st, "bow_words", &ev);
    const int64_t groups = (int64_t)A.nframes * A.cap;
    const dim3 blk(BOW_THREADS);
    if (A.group <= 16)
        hipLaunchKernelGGL(k_bow_words<16>, dim3((unsigned)((groups + 15) / 16)), blk, 0, st, A);
    else if (A.group <= 32)
        hipLaunchKernelGGL(k_bow_words<32>, dim3((unsigned)((groups + 7) / 8)), blk, 0, st, A);
    else
        hipLaunchKernelGGL(k_bow_words<64>, dim3((unsigned)((groups + 3) / 4)), blk, 0, st, A);
    prof_end(prof, st, "bow_words", ev);
    const size_t lds = bow_vectors_lds(A.cap);
    hipFuncSetAttribute((const void *)k_bow_vectors, hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)lds);
    prof_begin(prof, st, "bow_vectors", &ev);
    hipLaunchKernelGGL(k_bow_vectors, dim3(A.nframes), blk, lds, st, A);
    prof_end(prof, st, "bow_vectors", ev);
    return hipGetLastError() == hipSuccess ? ORBG_OK : ORBG_EIO;
}

}  // namespace orbg
