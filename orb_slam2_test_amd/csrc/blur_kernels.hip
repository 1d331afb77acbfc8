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
//              two v_perm, one dword store (legacy 257-sum weights saturate instead); with
//              tiled output (G.blur_tiled, the default) the wave is 240 columns (15 tiles of
//              16 x 8 px) wide and every 8 output rows go through the wave's LDS stage and
//              leave as two dwordx4 stores of whole tile rows (blur_device.h blur2_tile).
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
    const int TW = g->blur_tiled ? BLUR2_TW_T : BLUR2_TW;
    const int ntx = (W + TW - 1) / TW;
    const int ty = tt / ntx, tx = tt - ty * ntx;
    const uint8_t *src = l == 0 ? img0 + f * img_fs : pyr + f * g->pyr_frame + lv.pyr_off;
    const int pitch = l == 0 ? img_pitch : lv.pitch;
    uint8_t *dst = blur + f * g->blur_frame + lv.blur_off;
    __shared__ uint32_t rows[4][8 * BLUR2_LDS_ROW];  // tiled output: each wave's 8 staged rows
    if (g->blur_tiled)  // uniform
        blur2_tile<SEG, true>(k, src, pitch, W, H, dst, lv.pitch, tx, ty * SEG, H, lane, rows[wv]);
    else
        blur2_tile<SEG, false>(k, src, pitch, W, H, dst, lv.pitch, tx, ty * SEG, H, lane);
}

// k_blur_border: the GaussianBlur of every pixel the fused FAST cells do not blur (k_fast2
// with G.fast_blur: the rectangle [bx0, bx1) x [by0, by1) of each level, bx0 = 20, by0 = 19):
// the top rows [0, by0), the bottom rows [by1, H), and beside the rectangle the columns
// [0, bx0) and [bx1, W).  A thread per task (4 output columns x 8 output rows, the output columns' dword):
// tasks of a level in the order top | bottom | left | right, consecutive tasks in x.  The row
// and column arithmetic is k_blur2's (blur2_column); source rows and columns past the level
// are REFLECT_101 (rows by the row index, columns by per-byte loads in the few tasks that
// need them).
#define BLUR_BSEG 8
__global__ __launch_bounds__(256) void k_blur_border(
    const OrbgGeom *__restrict__ g, const uint8_t *__restrict__ img0, int64_t img_fs,
    int img_pitch, const uint8_t *__restrict__ pyr, uint8_t *__restrict__ blur, int l0, int l1,
    int nframes)
{
    const int tpf = g->lv[l1 - 1].bt_off + g->lv[l1 - 1].bt_cnt - g->lv[l0].bt_off;
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (int64_t)tpf * nframes) return;
    const int f = (int)(idx / tpf);
    int t = (int)(idx - (int64_t)f * tpf) + g->lv[l0].bt_off;
    int l = l0;
    while (l + 1 < l1 && t >= g->lv[l + 1].bt_off) l++;
    const OrbgLevel &lv = g->lv[l];
    t -= lv.bt_off;
    const int W = lv.w, H = lv.h, nqw = (W + 3) >> 2;
    const int segm = (lv.by1 - lv.by0 + BLUR_BSEG - 1) / BLUR_BSEG;
    const int nleft = lv.bx0 >> 2, nright = nqw - (lv.bx1 >> 2);
    const int ttop = ((lv.by0 + BLUR_BSEG - 1) / BLUR_BSEG) * nqw,
              tbot = ((H - lv.by1 + BLUR_BSEG - 1) / BLUR_BSEG) * nqw, tleft = segm * nleft;
    int q, y0, yend;
    if (t < ttop) {
        const int sg = t / nqw;
        q = t - sg * nqw;
        y0 = BLUR_BSEG * sg;
        yend = lv.by0;
    } else if ((t -= ttop) < tbot) {
        const int sg = t / nqw;
        q = t - sg * nqw;
        y0 = lv.by1 + BLUR_BSEG * sg;
        yend = H;
    } else if ((t -= tbot) < tleft) {
        const int sg = t / nleft;
        q = t - sg * nleft;
        y0 = lv.by0 + BLUR_BSEG * sg;
        yend = lv.by1;
    } else {
        t -= tleft;
        const int sg = t / nright;
        q = (lv.bx1 >> 2) + t - sg * nright;
        y0 = lv.by0 + BLUR_BSEG * sg;
        yend = lv.by1;
    }
    const uint8_t *src = l == 0 ? img0 + f * img_fs : pyr + f * g->pyr_frame + lv.pyr_off;
    const int pitch = l == 0 ? img_pitch : lv.pitch;
    uint8_t *dst = blur + f * g->blur_frame + lv.blur_off;
    // the source range starts at the dword holding the level's first byte (blur2_tile: a batch
    // frame may start at any byte); offsets below are src-relative, the loads add sh0
    const int nrec = (H - 1) * pitch + W;
    const int sh0 = (int)((uintptr_t)src & 3);
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void *)(src - sh0), (short)0, nrec + sh0, 0x00020000);
    const __amdgpu_buffer_rsrc_t drsrc = __builtin_amdgcn_make_buffer_rsrc((void *)dst, (short)0, H * lv.pitch, 0x00020000);
    const int gx = 4 * q;
    // window bytes gx - 4 .. gx + 7 inside the level with a dword of slack: aligned loads
    const bool inside = gx - 4 >= 0 && gx + 11 < W;
    const Blur2Weights k(g);
    auto loader = [&](int i, uint32_t &w0, uint32_t &w1, uint32_t &w2) {
        int y = b2_reflect101(min(y0 - 3 + i, H + 2), H);
        y = min(max(y, 0), H - 1);  // rows feeding no stored output only
        const int ro = y * pitch;
        if (inside) {
            const int a = ro + gx - 4;
            const int sh = (int)(((uintptr_t)src + a) & 3);
            const int aa = a - sh + sh0;  // the range's offset of the aligned dword
            const uint32_t d0 = __builtin_amdgcn_raw_buffer_load_b32(rsrc, aa, 0, 0);
            const uint32_t d1 = __builtin_amdgcn_raw_buffer_load_b32(rsrc, aa + 4, 0, 0);
            const uint32_t d2 = __builtin_amdgcn_raw_buffer_load_b32(rsrc, aa + 8, 0, 0);
            const uint32_t d3 = __builtin_amdgcn_raw_buffer_load_b32(rsrc, aa + 12, 0, 0);
            w0 = __builtin_amdgcn_alignbyte(d1, d0, sh);
            w1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
            w2 = __builtin_amdgcn_alignbyte(d3, d2, sh);
        } else {
            uint32_t w[3] = {0, 0, 0};
#pragma unroll
            for (int b = 0; b < 12; b++) {
                const int x = min(max(b2_reflect101(gx - 4 + b, W), 0), W - 1);
                w[b >> 2] |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rsrc, ro + x + sh0, 0, 0) << (8 * (b & 3));
            }
            w0 = w[0];
            w1 = w[1];
            w2 = w[2];
        }
    };
    auto store = [&](int o, uint32_t word) {
        const int y = y0 + o;
        __builtin_amdgcn_raw_buffer_store_b32(word, drsrc, y < yend ? y * lv.pitch + gx : (1 << 30), 0, 0);
    };
    if (k.norm256)
        blur2_column<BLUR_BSEG, true>(k, loader, store);
    else
        blur2_column<BLUR_BSEG, false>(k, loader, store);
}

hipError_t launch_blur_border(hipStream_t st, const OrbgGeom *g, int tasks_per_frame,
                              const uint8_t *img0, int64_t img_fs, int img_pitch,
                              const uint8_t *pyr, uint8_t *blur, int l0, int l1, int nframes)
{
    const int64_t n = (int64_t)tasks_per_frame * nframes;
    if (n <= 0 || l1 <= l0) return hipSuccess;
    hipLaunchKernelGGL(k_blur_border, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, g,
                       img0, img_fs, img_pitch, pyr, blur, l0, l1, nframes);
    return hipGetLastError();
}

int blur2_seg() { return ORBG_BLUR2_SEG; }
int blur2_tw(bool tiled) { return tiled ? BLUR2_TW_T : BLUR2_TW; }

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
