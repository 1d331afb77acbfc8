// schur_args.h -- launch arguments of the LBA Schur solve (schur_kernels.hip), shared with
// the host entry point (orbg_api.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "../../include/orbg.h"

namespace orbg {

// host-built structure of one solve (device pointers)
struct SchurArgs {
    int npose, npoint, nfree, n;       // n = 6 nfree
    const int32_t *pidx;               // [npose] free-pose index or -1
    const int32_t *pt_off, *pt_edges;  // active edges per point, ascending pose (CSR)
    const int32_t *edge_pose;          // [nedge] pose of each edge
    const int32_t *blk_off;            // [nblk + 1] (e1, e2) pairs per upper block, landmark order
    const int2 *blk_pairs;
    const int32_t *blk_i1, *blk_i2;    // [nblk]
    int nblk;
    const int32_t *pose_off, *pose_edges;  // edges per free pose, landmark order
    const orbg_edge_out *eout;
    const double *hpose, *bpose, *hpoint, *bpoint;
    double lambda;
    // scratch
    double *dinv;                      // [npoint][9]
    double *bd;                        // [nedge][18]  B D^-1 (row-major 6x3)
    double *cf;                        // [nedge][6]   B D^-1 b_l
    double *S;                         // [n][n]
    double *x;                         // [n]  b_schur, then x_p
    int32_t *ok;
    double *dx_pose, *dx_point;        // outputs [npose][6], [npoint][3]
};

int launch_schur(hipStream_t st, const SchurArgs &A, void *prof);

}  // namespace orbg
