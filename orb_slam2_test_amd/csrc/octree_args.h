// octree_args.h -- launch dimensions of k_octree_lds (host + device).
#pragma once

#include <stdint.h>

// One k_octree_lds launch covers levels level0 .. level0 + gridDim.x - 1.  Dynamic LDS =
// kcap * 7 + uni_bytes + acap2 * 4 (octree_kernels.hip OctLdsView).
struct OctLdsDims {
    int32_t level0;
    int32_t kcap;       // candidates per level this launch can hold (multiple of 64)
    int32_t acap;       // quadtree list capacity: max over its levels of out_cap
    int32_t acap2;      // aux entries: max(acap, cells + 1)
    int32_t nbw;        // bucket counter words: 512 * max roots (two u16 counters per word)
    int32_t uni_bytes;  // max(nbw * 4, 3 * acap * 8)
    int32_t tile_sort;  // winners to slots in (32-row x 128-column tile) order (ORBG_OD_SORT)
    int32_t kmin;       // > 0: levels with <= kmin candidates are another launch's (untouched)
    int32_t first;      // first of a split pair: a level past kcap is the second launch's
                        // (flagged in err_flag[3])
    int32_t keep_cnt;   // 1: a level left to k_octree keeps its lvl_cnt entry (k_octree runs
                        // concurrently and owns it: ORBG_BIG_SIDE), 0: zeroed for a consumer
                        // that may run without k_octree
    int32_t tag;        // != 0: a level left to k_octree stores tag into err_flag[4] instead of
                        // setting err_flag[2] (the single-frame path's per-call flag: nothing
                        // to clear ahead of the launch)
};

// static LDS header of k_octree_lds
struct OctLdsHdr {
    int red[16];
    int rootlo[20];
    int s_alive, s_cur, s_seq, s_vbase, s_vend, s_err, s_nproc, s_phase2;
};

static inline size_t oct_lds_bytes(const OctLdsDims &d)
{
    return (size_t)d.kcap * 7 + (size_t)d.uni_bytes + (size_t)d.acap2 * 4;
}
