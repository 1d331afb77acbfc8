// bow_match_kernels.hip -- k_bow_match: ORBmatcher::SearchByBoW(KeyFrame *pKF, Frame &F,
// vector<MapPoint*> &vpMapPointMatches) (src/ORBmatcher.cc:195-348) for gfx950, one workgroup
// per (KF, F) pair; k_bow_match<true> is the KeyFrame-KeyFrame form SearchByBoW(pKF1, pKF2,
// vpMatches12) (:634-769: KF2's MapPoint flags, strict < TH_LOW, output at the KF1 index).  Callers: Tracking::TrackReferenceKeyFrame (Tracking.cc:1069) and
// Tracking::Relocalization (:2009), over the FeatureVectors DBoW2's transform builds
// (orbg_bow_transform_batch_device, bow_kernels.hip).
//
// The reference walks both FeatureVectors (std::map NodeId -> feature indices) in id order and
// matches features that share a node; a feature of F lives in exactly one node, so nodes are
// independent and only the order WITHIN a node matters (an F feature taken by an earlier KF
// feature of the node is skipped).  Here:
//   join     the KF node ids, 64 per wave, each lane binary-searching F's sorted node ids in
//            HBM; common (KF node, F node) pairs are appended to an LDS list (any order);
//   node     a wave per common node: lane l holds F candidate l (+ 64, + 128 ...) of the node,
//            its descriptor in registers and a "taken" bit; the node's KF features run in the
//            reference's order (a KF feature without a valid MapPoint skipped, wave-uniform),
//            the KF descriptor in scalar registers; per lane the Hamming distance (8 xor +
//            8 bcnt), then two wave-wide min reductions: (distance, position) for the best --
//            the first position wins ties, as the reference's strict < -- and the second best
//            (the winner's own second, everyone else's best).  TH_LOW and the float nnratio
//            test, then the winner lane marks its candidate taken, writes the match and adds
//            the rotation bin to an LDS histogram;
//   rotation ComputeThreeMaxima (ORBmatcher.cc:1800-1841) by one lane, then every match
//            outside the three bins dropped (its bin recomputed from the two angles).
#include <hip/hip_runtime.h>

#include "../../include/orbg.h"
#include "orbg_internal.h"
#include "orbg_device.h"

#pragma clang fp contract(off)

namespace orbg {

#define BM_HISTO 30
#define BM_TH_LOW 50
#define BM_LIST 1024  // common nodes per pass held in LDS (KeyFrame nodes joined BM_LIST at a time)
#define BM_MAX_NODE 4096  // Frame features per node the taken mask covers (64 chunks of 64)

struct BowMatchSide {
    const uint8_t *desc;
    const orbg_keypoint *kps;
    const int32_t *counts, *fv_nodes, *fv_off, *fv_feats, *nfv;
    const uint8_t *valid;
};

__device__ __forceinline__ unsigned wave_min_u32(unsigned v)
{
    // butterfly over the wave with DPP row ops and the 32-lane swap; result in every lane
    v = min(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0xb1, 0xf, 0xf, false));  // quad_perm 1,0,3,2
    v = min(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x4e, 0xf, 0xf, false));  // quad_perm 2,3,0,1
    v = min(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xf, 0xf, false)); // row_ror 4
    v = min(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xf, 0xf, false)); // row_ror 8
    const unsigned r0 = (unsigned)__builtin_amdgcn_readlane((int)v, 0);
    const unsigned r1 = (unsigned)__builtin_amdgcn_readlane((int)v, 16);
    const unsigned r2 = (unsigned)__builtin_amdgcn_readlane((int)v, 32);
    const unsigned r3 = (unsigned)__builtin_amdgcn_readlane((int)v, 48);
    return min(min(r0, r1), min(r2, r3));
}

__device__ __forceinline__ int bm_rot_bin(float a_kf, float a_f)
{
    // ORBmatcher.cc:291-297 (rot < 0.0 in double as the reference compares, then float)
    const float factor = 1.0f / BM_HISTO;
    float rot = a_kf - a_f;
    if (rot < 0.0) rot += 360.0f;
    int bin = (int)roundf(rot * factor);
    if (bin == BM_HISTO) bin = 0;
    return bin;
}

// KFKF: ORBmatcher::SearchByBoW(KeyFrame *pKF1, KeyFrame *pKF2, vpMatches12)
// (ORBmatcher.cc:634-769) -- K = pKF1, F = pKF2 with its MapPoint flags (F.valid), accepted on
// bestDist1 < TH_LOW (strict), the match written at the KF1 index (match[idx1] = idx2)
template <bool KFKF>
__global__ __launch_bounds__(256) void k_bow_match(BowMatchSide K, BowMatchSide F, int cap,
                                                   const int32_t *__restrict__ kf_index,
                                                   const int32_t *__restrict__ f_index,
                                                   float nnratio, int check_ori,
                                                   int32_t *__restrict__ match,
                                                   int32_t *__restrict__ nmatch)
{
    __shared__ int2 common[BM_LIST];
    __shared__ int ncommon, nm, removed, hist[BM_HISTO], ind[3];
    const int p = blockIdx.x;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int kf = kf_index[p], fr = f_index[p];
    const int nk_nodes = K.nfv[kf], nf_nodes = F.nfv[fr];
    const int n_f = F.counts[fr];
    const int n_out = KFKF ? K.counts[kf] : n_f;  // output rows: KF1 (KFKF) or F features
    const int32_t *kn = K.fv_nodes + (size_t)kf * cap, *ko = K.fv_off + (size_t)kf * (cap + 1),
                  *kfe = K.fv_feats + (size_t)kf * cap;
    const int32_t *fn = F.fv_nodes + (size_t)fr * cap, *fo = F.fv_off + (size_t)fr * (cap + 1),
                  *ffe = F.fv_feats + (size_t)fr * cap;
    const uint8_t *kdesc = K.desc + (size_t)kf * cap * 32, *fdesc = F.desc + (size_t)fr * cap * 32;
    const orbg_keypoint *kkp = K.kps + (size_t)kf * cap, *fkp = F.kps + (size_t)fr * cap;
    const uint8_t *kval = K.valid ? K.valid + (size_t)kf * cap : nullptr;
    const uint8_t *fval = (KFKF && F.valid) ? F.valid + (size_t)fr * cap : nullptr;
    int32_t *out = match + (size_t)p * cap;
    if (threadIdx.x == 0) {
        nm = 0;
        removed = 0;
    }
    if (threadIdx.x < BM_HISTO) hist[threadIdx.x] = 0;
    for (int i = threadIdx.x; i < n_out; i += blockDim.x) out[i] = -1;
    int wave_nm = 0;
    // Nodes are independent (a feature sits in one node of its FeatureVector, so two nodes
    // share no candidate and no KeyFrame feature): any node order gives the reference's
    // matches, and the KeyFrame nodes are joined BM_LIST at a time.
    for (int j0 = 0; j0 < nk_nodes; j0 += BM_LIST) {
    if (threadIdx.x == 0) ncommon = 0;
    __syncthreads();
    // ---- join: KF node j looks its id up in F's sorted node ids ----
    for (int j = j0 + (int)threadIdx.x; j < min(nk_nodes, j0 + BM_LIST); j += blockDim.x) {
        const int id = kn[j];
        int lo = 0, hi = nf_nodes;  // first F node with id >= kn[j]
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (fn[mid] < id)
                lo = mid + 1;
            else
                hi = mid;
        }
        if (lo < nf_nodes && fn[lo] == id) {
            const int k = atomicAdd(&ncommon, 1);
            common[k] = make_int2(j, lo);  // k < BM_LIST: at most BM_LIST KF nodes per pass
        }
    }
    __syncthreads();
    const int nc = ncommon;
    // ---- a wave per common node ----
    for (int c = wv; c < nc; c += (int)(blockDim.x >> 6)) {
        const int2 jb = common[c];
        const int k0 = ko[jb.x], k1 = ko[jb.x + 1];
        const int f0 = fo[jb.y], nF = fo[jb.y + 1] - f0;
        const int nchunk = (nF + 63) >> 6;
        uint32_t cd0[8], cd1[8];  // candidates lane and lane + 64 (larger nodes: re-read)
        int ci0 = -1, ci1 = -1;
        if (lane < nF) ci0 = ffe[f0 + lane];
        if (lane + 64 < nF) ci1 = ffe[f0 + lane + 64];
        // KFKF: a KF2 feature without a good MapPoint is no candidate (ORBmatcher.cc:695-699)
        const bool ok0 = !fval || (ci0 >= 0 && fval[ci0]), ok1 = !fval || (ci1 >= 0 && fval[ci1]);
#pragma unroll
        for (int w = 0; w < 8; w++) {
            cd0[w] = ci0 >= 0 ? ((const uint32_t *)(fdesc + (size_t)ci0 * 32))[w] : 0u;
            cd1[w] = ci1 >= 0 ? ((const uint32_t *)(fdesc + (size_t)ci1 * 32))[w] : 0u;
        }
        uint64_t taken = 0;  // bit k: candidate lane + 64 k already matched (nF <= BM_MAX_NODE)
        // the node's KF features, 64 at a time: lane l loads feature ib + l (index, MapPoint
        // flag, descriptor) so the in-order walk broadcasts them by readlane instead of
        // waiting on dependent global loads per feature
        for (int ib = k0; ib < k1; ib += 64) {
        const int cn = min(64, k1 - ib);
        int my_rk = 0, my_ok = 0;
        uint32_t my_kd[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (lane < cn) {
            my_rk = kfe[ib + lane];
            my_ok = !kval || kval[my_rk];  // pMP NULL or bad: skipped
            const uint4 *dp = (const uint4 *)(kdesc + (size_t)my_rk * 32);
            const uint4 qa = dp[0], qb = dp[1];
            my_kd[0] = qa.x; my_kd[1] = qa.y; my_kd[2] = qa.z; my_kd[3] = qa.w;
            my_kd[4] = qb.x; my_kd[5] = qb.y; my_kd[6] = qb.z; my_kd[7] = qb.w;
        }
        const unsigned long long okm = __ballot(lane < cn && my_ok);
        for (int t = 0; t < cn; t++) {
            if (!((okm >> t) & 1ull)) continue;  // wave-uniform skip
            const int rk = __builtin_amdgcn_readlane(my_rk, t);
            uint32_t kd[8];
#pragma unroll
            for (int w = 0; w < 8; w++) kd[w] = (uint32_t)__builtin_amdgcn_readlane((int)my_kd[w], t);
            unsigned b1 = 256, b2 = 256, pos1 = 0xFFFF;
            for (int ch = 0; ch < nchunk; ch++) {  // in position order: strict < keeps the first
                const int pos = ch * 64 + lane;
                if (pos >= nF || (taken >> ch & 1u)) continue;
                if (KFKF && fval && !(ch == 0 ? ok0 : ch == 1 ? ok1 : fval[ffe[f0 + pos]] != 0))
                    continue;
                unsigned d = 0;
                if (ch == 0) {
#pragma unroll
                    for (int w = 0; w < 8; w++) d += __popc(kd[w] ^ cd0[w]);
                } else if (ch == 1) {
#pragma unroll
                    for (int w = 0; w < 8; w++) d += __popc(kd[w] ^ cd1[w]);
                } else {
                    const uint32_t *q = (const uint32_t *)(fdesc + (size_t)ffe[f0 + pos] * 32);
#pragma unroll
                    for (int w = 0; w < 8; w++) d += __popc(kd[w] ^ q[w]);
                }
                if (d < b1) {
                    b2 = b1;
                    b1 = d;
                    pos1 = (unsigned)pos;
                } else if (d < b2) {
                    b2 = d;
                }
            }
            const unsigned key = b1 << 16 | pos1;
            const unsigned best = wave_min_u32(key);
            const unsigned best1 = best >> 16, bpos = best & 0xFFFFu;
            const bool winner = key == best && best1 < 256;
            const unsigned best2 = wave_min_u32(winner ? b2 : b1);
            if ((KFKF ? best1 < BM_TH_LOW : best1 <= BM_TH_LOW) &&
                (float)best1 < nnratio * (float)best2) {
                wave_nm++;
                if (winner) {
                    taken |= 1ull << (bpos >> 6);
                    const int rf = ffe[f0 + (int)bpos];
                    if (KFKF)
                        out[rk] = rf;
                    else
                        out[rf] = rk;
                    if (check_ori) atomicAdd(&hist[bm_rot_bin(kkp[rk].angle, fkp[rf].angle)], 1);
                }
            }
        }
        }
    }
    __syncthreads();  // the common list is rebuilt by the next pass
    }
    if (lane == 0 && wave_nm) atomicAdd(&nm, wave_nm);
    __syncthreads();
    if (check_ori) {
        if (threadIdx.x == 0) {
            // ComputeThreeMaxima (ORBmatcher.cc:1800-1841)
            int max1 = 0, max2 = 0, max3 = 0, i1 = -1, i2 = -1, i3 = -1;
            for (int i = 0; i < BM_HISTO; i++) {
                const int s = hist[i];
                if (s > max1) {
                    max3 = max2;
                    max2 = max1;
                    max1 = s;
                    i3 = i2;
                    i2 = i1;
                    i1 = i;
                } else if (s > max2) {
                    max3 = max2;
                    max2 = s;
                    i3 = i2;
                    i2 = i;
                } else if (s > max3) {
                    max3 = s;
                    i3 = i;
                }
            }
            if (max2 < 0.1f * (float)max1) {
                i2 = -1;
                i3 = -1;
            } else if (max3 < 0.1f * (float)max1) {
                i3 = -1;
            }
            ind[0] = i1;
            ind[1] = i2;
            ind[2] = i3;
        }
        __syncthreads();
        int rm = 0;
        for (int i = threadIdx.x; i < n_out; i += blockDim.x) {
            const int m = out[i];
            if (m < 0) continue;
            const int bin = KFKF ? bm_rot_bin(kkp[i].angle, fkp[m].angle)
                                 : bm_rot_bin(kkp[m].angle, fkp[i].angle);
            if (bin != ind[0] && bin != ind[1] && bin != ind[2]) {
                out[i] = -1;
                rm++;
            }
        }
        if (rm) atomicAdd(&removed, rm);
        __syncthreads();
    }
    if (threadIdx.x == 0) nmatch[p] = nm - removed;
}

int launch_bow_match(hipStream_t st, const orbg_bow_frames &kf, const orbg_bow_frames &f, int cap,
                     const int32_t *kf_index, const int32_t *f_index, int npairs, float nnratio,
                     int check_ori, int32_t *match, int32_t *nmatch, bool kfkf)
{
    if (npairs <= 0) return 0;
    if (cap > BM_MAX_NODE) return -95;  // ORBG_ENOTSUP: a node could exceed the taken mask
    const BowMatchSide K{kf.desc, kf.kps, kf.counts, kf.fv_nodes, kf.fv_off, kf.fv_feats, kf.nfv,
                         kf.valid};
    const BowMatchSide F{f.desc, f.kps, f.counts, f.fv_nodes, f.fv_off, f.fv_feats, f.nfv,
                         kfkf ? f.valid : nullptr};
    if (kfkf)
        hipLaunchKernelGGL(k_bow_match<true>, dim3(npairs), dim3(256), 0, st, K, F, cap, kf_index,
                           f_index, nnratio, check_ori, match, nmatch);
    else
        hipLaunchKernelGGL(k_bow_match<false>, dim3(npairs), dim3(256), 0, st, K, F, cap, kf_index,
                           f_index, nnratio, check_ori, match, nmatch);
    return hipGetLastError() == hipSuccess ? 0 : -5;
}

}  // namespace orbg
