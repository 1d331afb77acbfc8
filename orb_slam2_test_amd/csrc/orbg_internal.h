// orbg_internal.h -- shared host/device definitions of liborbg (MI355X, gfx950).
//
// HBM layout for a batch of B frames (all per-frame regions contiguous, frame-major):
//   input images ........ caller's buffer (level 0 of the pyramid, pitch = caller's step)
//   pyramid levels 1..L-1  d_pyr   [B][pyr_frame_bytes], level l at lv[l].off, pitch lv[l].pitch
//   blurred levels 0..L-1  d_blur  [B][blur_frame_bytes]
//   FAST cell slots ...... d_cell_cnt [B][ncells], d_cell_kp [B][ncells][cell_cap] (packed u32)
//   octree scratch ....... d_keys/d_keynode [B][keys_frame]; d_nodes [B][nodes_frame] (int4)
//   octree output ........ d_lvl_kp [B][out_frame] (packed u32), d_lvl_cnt [B][L]
//   final outputs ........ d_kps [B][frame_cap] orbg_keypoint, d_desc [B][frame_cap][32],
//                          d_counts [B]
// Packed candidate/keypoint word: x | y << 12 | score << 24 (coordinates relative to
// minBorder = EDGE_THRESHOLD-3 = 16, exactly the vToDistributeKeys coordinates).
#pragma once

#include <stdint.h>

#define ORBG_EDGE_THRESHOLD 19
#define ORBG_MIN_BORDER 16
#define ORBG_HALF_PATCH 15
#define ORBG_PATCH 31
#define ORBG_CELL_W 30.0f
#define ORBG_MAX_WIN 72          // largest FAST window edge (wCell+6 < 66)
#define ORBG_OCT_ALIVE 2048      // max live quadtree nodes per (frame, level)
#define ORBG_OCT_THREADS 256
#define ORBG_GRID_COLS 64        // Frame.h:38
#define ORBG_GRID_ROWS 48        // Frame.h:37
#define ORBG_MATCH_TOPK 8
#ifndef ORBG_FC2_BITMAP
#define ORBG_FC2_BITMAP 0  // 1: k_fast2 marks corner units in an LDS bitmap while scoring (no pass over every unit); measured +0.07 ms, profiles/r05o_fast_bitmap_ab.txt
#endif
// sticky device error word, bit 16: a device matcher read a per-frame / per-pair count past
// its capacity (clamped; orbg_check_errors reports it).  Bits 0..9: the quadtree's flags.
#define ORBG_DEVFLAG_COUNT (1 << 16)
// orbg_ba_graph's packed LBA edge (24 B instead of orbg_edge's 104): flags bit 0 stereo,
// 1 robust, 2 active, bits 8..15 camera index, 16..31 (information, Huber) index; the
// observations are f32 (ORB-SLAM2's are cv::KeyPoint floats: exact)
struct BaPackedEdge {
    int32_t point, pose;
    uint32_t flags;
    float obs[3];
};
struct BaCam {
    double fx, fy, cx, cy, bf;
};
struct BaInfo {
    double inv_sigma2, huber_delta;
};
// an orbg_ba_graph's device-side structure (ba_kernels.hip launch_ba_graph), built once at
// orbg_ba_graph_create: special = the points whose k_ba_edges slots span two workgroups or
// that have no edge; the pose slices of ORBG_BA_SLICE edges and their partial sums
#define ORBG_BA_SLICE 64
#define ORBG_BA_EDGES_TPB 256
struct BaGraphDev {
    const int32_t *special;   // special points (above)
    int32_t nspecial;
    const int32_t *slice_off, *slice_pose;  // pose p owns slices slice_off[p] .. [p+1]-1
    int32_t nslice;
    double *part;             // [nslice][42] pose-block partials
};
#define ORBG_BA_MAX_CAMS 256
#define ORBG_BA_MAX_INFOS 65536

#ifndef ORBG_RZ_NT
#define ORBG_RZ_NT 1             // k_resize: 16-row output tiles per workgroup (more: the prefetched chunks cost occupancy, measured slower)
#endif
#ifndef ORBG_RZ_FILL
#define ORBG_RZ_FILL 5           // k_resize: staged 16-byte chunks per thread
#endif
#ifndef ORBG_OD_KPW
#define ORBG_OD_KPW 10           // k_orient_desc: quadtree output slots per wave (8: +1.6% orient, 12: a tie, profiles/r06aj_od_kpw_ab.txt)
#endif
#define ORBG_OD_TABW 93          // k_orient_desc: IC_Angle lanes (31 rows x 3 chunks)
#define OCT_KEY_CAP 16384        // k_octree_lds handles levels with <= this many candidates

struct OrbgLevel {
    int32_t w, h, pitch;
    int32_t max_bx, max_by;       // maxBorderX/Y = w-16 / h-16
    int32_t ncols, nrows, wcell, hcell;
    int32_t cell_base, ncells;
    int32_t nfeat;                // mnFeaturesPerLevel
    int32_t nini;                 // quadtree roots
    float hx;                     // root width (float, DistributeOctTree :680)
    int32_t key_off, key_cap;     // candidate scratch (u32 words) within a frame
    int32_t node_off, node_cap;   // int4 node records within a frame
    int32_t out_off, out_cap;     // octree output words within a frame
    int32_t bulk_end;             // resize: first column using the scalar vertical pass
    int32_t xtab_off, ytab_off;   // resize coefficient tables (int2 per column / row)
    int32_t xs_off, ys_off;       // quadtree path-code tables (u32 per rel. column / row)
    int32_t rz_pitch, rz_rows;    // k_resize LDS staging: bytes per source row, rows per tile
    int64_t pyr_off;              // byte offset of the level in a frame's pyramid (l >= 1)
    int64_t blur_off;             // byte offset in a frame's blurred pyramid
    float scale;                  // mvScaleFactor[l]
    int32_t patch_size;           // int(PATCH_SIZE * scale)
    int32_t oct_kcap, oct_acap2;  // this level's k_octree_lds launch: candidate / cell caps
    // GaussianBlur fused into k_fast2 (G.fast_blur): the FAST cells blur the rectangle
    // [bx0, bx1) x [by0, by1) (their detection regions, from the first dword boundary at or
    // after the regions' left edge 19 to the first after their right edge) from their window
    // tiles; k_blur_border the rest of the level, bt_cnt tasks (4 columns x 8 rows) from
    // bt_off on in a frame's task list
    int32_t bx0, by0, bx1, by1, bt_off, bt_cnt;
};

struct OrbgGeom {
    int32_t L;
    int32_t w, h;
    int32_t ncells;               // all levels
    int32_t cell_cap;             // max packed candidates per cell
    int32_t keys_frame;           // u32 words per frame of candidate scratch
    int32_t nodes_frame;          // int4 per frame
    int32_t out_frame;            // octree output words per frame
    int32_t frame_cap;            // max keypoints per frame (final)
    int32_t ini_th, min_th;
    int32_t brief_fma;
    int32_t sincos_mode;          // rBRIEF cos/sin: 0 glibc cosf/sinf restated, 1 pinned double
    int32_t dbg;                  // developer timing knob (ORBG_DBG env), 0 in production
    int32_t fc2_p4;               // k_fast2 LDS row pitch (dwords, a template instance)
    int32_t fc2_wave_bytes;       // k_fast2 LDS bytes per wave
    int32_t fc2_sc_off, fc2_list_off;  // k_fast2 regions within a wave's LDS
    int32_t fc2_list_cap;         // k_fast2 pretest list entries per wave
    int32_t fast_blur;            // 1: k_fast2 blurs its cells' regions (OrbgLevel bx1 / by1)
    int32_t bt_total;             // k_blur_border tasks per frame (all levels)
    int32_t blur_tiled;           // 1: the blurred levels are 16 x 8-px tiles (blur2_tile TILED)
    int32_t gk[7];
    int64_t pyr_frame;            // bytes per frame of d_pyr
    int64_t blur_frame;
    int32_t umax[16];
    OrbgLevel lv[16];
};

// cell table entry
struct OrbgCell {
    int16_t level, pad;
    int16_t x0, y0;   // window top-left (level coords)
    int16_t w, h;     // window size
    int16_t ci, cj;   // cell row / col (for pt += j*wCell, i*hCell)
};

// k_fast_rows strip: up to 8 consecutive cells of one cell row of one level (host plan)
struct OrbgFastTile {
    int16_t level, ncell;
    int32_t c0;       // global index of the first cell (a cell row's cells are consecutive)
    int16_t x0, y0;   // window top-left of the first cell (level coords)
    int16_t h, tw;    // window rows (region rows + 6), region width (sum of the cells')
};

static inline __host__ __device__ uint32_t orbg_pack(int x, int y, int s)
{
    return (uint32_t)x | ((uint32_t)y << 12) | ((uint32_t)s << 24);
}
static inline __host__ __device__ int orbg_px(uint32_t v) { return (int)(v & 0xFFFu); }
static inline __host__ __device__ int orbg_py(uint32_t v) { return (int)((v >> 12) & 0xFFFu); }
static inline __host__ __device__ int orbg_ps(uint32_t v) { return (int)(v >> 24); }
