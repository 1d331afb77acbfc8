// blur_kernels.hip -- k_blur2: GaussianBlur(7x7, sigma 2, BORDER_REFLECT_101) of every pyramid
// level (ORBextractor.cc:1375-1377, cv::GaussianBlur 8U bit-exact fixed point:
// out = sat((sum_v k_v * sum_h k_h * p + 2^15) >> 16)), without LDS and without workgroup
// barriers.  Levels are >= 62 px wide (the plan refuses a level narrower than one 30-px cell
// plus the borders), so the row-end permutes always have the 8 bytes they assume.
//
// One wave owns a 244-column x SEG-row output tile of one (frame, level); lane j owns columns
// gx .. gx+3 (gx = tile x + 4j; lanes 61..63 only supply data) and walks the SEG + 6 source
// rows top to bottom:
//   load       one dword per lane and row (column gx - 4 of the row's 4-byte-aligned start,
//              bounds-checked buffer load: past the level's last byte it reads 0), the next
//              three dwords from lanes j+1 .. j+3 by DPP wave shifts, v_alignbyte by the row's
//              (wave-uniform) byte shift: the 12 window bytes gx-4 .. gx+7;
//   row ends   REFLECT_101 by byte permutes of that window, in the first / last tile of a level
//              row only (wave-uniform branches): the left lane rebuilds window dword 0, the
//              right lanes (W - gx < 8) dwords 1 and 2 with per-lane v_perm selectors;
//   row pass   ten v_dot4_u32_u8 against byte-shifted weight words give the four row sums;
//   column     a register window of packed row-pair sums: output row o = dot2(P[o], (k0,k1)) +
//              dot2(P[o+2], (k2,k3)) + dot2(P[o+4], (k4,k5)) + k6 * s[o+6], the rounding term
//              2^15 as the chain's start value;
//   store      with weights summing to 256 the output is byte 2 of the sum: four pixels packed by
//              two v_perm, one dword store (legacy 257-sum weights saturate instead).
#include <hip/hip_runtime.h>

#include "orbg_internal.h"
#include "orbg_device.h"
#include "blur_device.h"

#pragma clang fp contract(off)

namespace orbg {

template <int SEG>
__global__ __launch_bounds__(256) void k_blur2(
    const OrbgGeom *__restrict__ g, const int32_t *__restrict__ task_base,
    const uint8_t *__restrict__ img0, int64_t img_fs, int img_pitch,
    const uint8_t *__restrict__ pyr, uint8_t *__restrict__ blur, int t_begin, int t_count,
    int nframes)
{
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int wid = __builtin_amdgcn_readfirstlane(xcd_remap(blockIdx.x, gridDim.x) * 4 + wv);
    if (wid >= t_count * nframes) return;  // wave-uniform; no barrier below
    const Blur2Weights k(g);
    // frame-major, then the tiles [t_begin, t_begin + t_count) in level order
    const int f = wid / t_count, t = t_begin + wid - f * t_count;
    int l = 0;
    while (l + 1 < g->L && t >= task_base[l + 1]) l++;
    const int tt = t - task_base[l];
    const OrbgLevel &lv = g->lv[l];
    const int W = lv.w, H = lv.h;
    const int ntx = (W + BLUR2_TW - 1) / BLUR2_TW;
    const int ty = tt / ntx, tx = tt - ty * ntx;
    const uint8_t *src = l == 0 ? img0 + f * img_fs : pyr + f * g->pyr_frame + lv.pyr_off;
    const int pitch = l == 0 ? img_pitch : lv.pitch;
    uint8_t *dst = blur + f * g->blur_frame + lv.blur_off;
    blur2_tile<SEG>(k, src, pitch, W, H, dst, lv.pitch, tx, ty * SEG, H, lane);
}

int blur2_seg() { return ORBG_BLUR2_SEG; }
int blur2_tw() { return BLUR2_TW; }

// tiles [t_begin, t_begin + t_count) of every frame
hipError_t launch_blur2(hipStream_t st, const OrbgGeom *g, const int32_t *task_base,
                        const uint8_t *img0, int64_t img_fs, int img_pitch, const uint8_t *pyr,
                        uint8_t *blur, int t_begin, int t_count, int nframes)
{
    const int waves = t_count * nframes;
    if (waves <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_blur2<ORBG_BLUR2_SEG>, dim3((waves + 3) / 4), dim3(256), 0, st, g,
                       task_base, img0, img_fs, img_pitch, pyr, blur, t_begin, t_count, nframes);
    return hipGetLastError();
}

}  // namespace orbg
