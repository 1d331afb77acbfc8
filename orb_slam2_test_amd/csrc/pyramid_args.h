// pyramid_args.h -- k_pyramid launch arguments (host plan <-> pyramid_kernels.hip).
#pragma once

#include <stdint.h>

#define PYR_ROWS 8   // output rows per work item (one lane)
#define PYR_COLS 8   // output columns per work item
#define PYR_NS 11    // max source rows per item: floor(7 * 1.2) + 1 + 2 (host checks)
#ifndef PYR_BLUR_SEG
#define PYR_BLUR_SEG 16  // k_pyramid's fused GaussianBlur: output rows per wave tile
#endif
#ifndef PYR_PF
#define PYR_PF 4     // source rows in flight ahead of the one being summed
#endif

// per output column octet: 5 x uint4
//   [0] {sx0 = source column of the octet's first output column, scalar-column mask, 0, 0}
//   [1], [2]  v_perm selectors of columns 0-3 (window bytes 0-7) and 4-7 (window bytes 4-11):
//             {rel(sx), 0, rel(sx + 1 clamped), 0} as u16 lanes of the 12-byte window that
//             starts at source byte sx0
//   [3], [4]  horizontal coefficients {a0 << 4 | a1 << 4 << 16} (v_dot2_u32_u16 gives h << 4)
// per output row: int4 {sy0 | sy1 << 16, b0 << 8, b1 << 8, b0 | b1 << 16}
struct PyrLevelArgs {
    int32_t sw, sh, dw, dh;
    int32_t spitch, dpitch;       // spitch unused for level 1 (the caller's pitch)
    int64_t src_off, dst_off;     // byte offsets in a frame's d_pyr (src_off: level l-1 >= 1)
    int32_t noct;                 // output column octets
    int32_t ptab_off;             // uint4 index of the level's octet records
    int32_t ytab_off;             // int4 index of the level's row records
    int32_t fix_oct;              // first octet with a FixedPtCast column or past the width
    int32_t clamp_row;            // first output row with sy0 == sy1 (dh if none)
    int32_t guard_row;            // level 1: first output row reading the caller's last row
    int32_t pad;
    int64_t blur_off;             // byte offset of the level in a frame's blurred pyramid
};

// bands[b * L + l] = {first, end} rows of level l (l >= 1) band b computes (its own rows, the
// rows its higher levels read and, with fuse_blur, the +-3 rows its own blurred rows read),
// {own first, own end} rows of level l whose GaussianBlur band b writes (level 0 too)
struct PyrArgs {
    int32_t L, nband;
    int64_t pyr_frame;
    int32_t fuse_blur;            // GaussianBlur in the same launch: 1 every level, 2 levels >= 1
    int32_t w0, h0, bpitch0;      // level 0 size and its blurred row pitch
    int64_t blur_frame, blur_off0;
    PyrLevelArgs lv[16];
};
