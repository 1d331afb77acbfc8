// schur_args.h -- launch arguments of the LBA Schur solve (schur_kernels.hip), shared with
// the host entry points (orbg_api.hip): orbg_ba_schur_solve (host arrays) and
// orbg_ba_graph_schur_solve (an orbg_ba_graph's device blocks), both on one device plan.
#pragma once

#include <hip/hip_runtime.h>

#include <vector>

#include "../../include/orbg.h"

namespace orbg {

// The solve's structure, built once on the host per (graph, fixed set, active set) -- the
// graph is fixed across LM iterations -- and uploaded (device pointers below).
//   free poses: pidx[pose] = free index or -1 (g2o fixes them: no Schur block);
//   points: their active edges to any pose, ascending pose (CSR pt_off / pt_edges);
//   upper Schur blocks (i1 <= i2): every diagonal block + every free-pose pair sharing a
//     landmark, with its (slot of e1, e2) pairs in landmark order (blk_off / blk_pairs; a
//     slot is a position in pt_edges: the k_schur_points records are stored by slot);
//   free poses' active edges' slots in landmark order (pose_off / pose_slots);
//   segments: contiguous free-index ranges closed under the landmark coupling, solved as
//     independent dense systems (one LBA window is one segment; independent windows
//     batched into one graph are several).  S is block diagonal across segments, so the
//     per-segment LDLT gives the same bits as one dense LDLT of the whole system.
struct SchurPlanHost {
    int npose = 0, npoint = 0, nfree = 0, nblk = 0, nseg = 0, max_seg = 0;
    std::vector<int32_t> pidx, free_pose, pt_off, pt_edges, slot_point, slot_fidx, edge_pose,
        blk_off, blk_i1, blk_i2, blk_seg, blk_order, pose_off, pose_slots, seg_lo;
    std::vector<int2> blk_pairs;
    std::vector<int64_t> seg_soff;  // [nseg + 1] doubles before each segment's dense matrix
};

// epose / epoint / eactive: per edge; fixed: per pose
void build_schur_plan(int npose, int npoint, int nedge, const int32_t *epose,
                      const int32_t *epoint, const uint8_t *eactive, const uint8_t *fixed,
                      SchurPlanHost &P);

struct SchurArgs {
    int npose, npoint, nfree, nblk, nseg, max_seg;
    const int32_t *pidx;               // [npose] free-pose index or -1
    const int32_t *free_pose;          // [nfree] its pose
    const int32_t *pt_off, *pt_edges;  // active edges per point, ascending pose (CSR)
    const int32_t *slot_point;         // [nslot] the point of each slot of pt_edges
    const int32_t *slot_fidx;          // [nslot] free index of the slot's pose, or -1 (fixed)
    int nslot;                         // = pt_off[npoint]
    const int32_t *edge_pose;          // [nedge] pose of each edge
    const int32_t *blk_off;            // [nblk + 1] (slot1, e2) pairs per upper block, landmark order
    const int2 *blk_pairs;
    const int32_t *blk_i1, *blk_i2, *blk_seg;  // [nblk]
    const int32_t *blk_order;          // [nblk] k_schur_blocks' dispatch order (a permutation)
    const int32_t *pose_off, *pose_slots;      // active slots per free pose, landmark order
    const int32_t *seg_lo;             // [nseg + 1] free-index range of each segment
    const int64_t *seg_soff;           // [nseg + 1] offset (doubles) of its dense matrix in S
    const double *hpl;                 // H_pl of edge e: hpl[e * hpl_stride + 6 k + c] (3 x 6)
    int hpl_stride;
    const double *hpose, *bpose, *hpoint, *bpoint;
    double lambda;
    // scratch
    double *rec;                       // [nslot][24]: B D^-1 (row-major 6x3), B D^-1 b_l (6)
    double *S;                         // s_total doubles: the segments' dense systems
    int64_t s_total;                   // = seg_soff[nseg] (host copy)
    double *x;                         // [6 nfree]  b_schur, then x_p
    int32_t *ok;                       // 1 unless some segment hit a zero / non-finite pivot
    double *dx_pose, *dx_point;        // outputs [npose][6], [npoint][3]
};

int launch_schur(hipStream_t st, const SchurArgs &A, void *prof);

}  // namespace orbg
