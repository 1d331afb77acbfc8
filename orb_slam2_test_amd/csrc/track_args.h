// track_args.h -- launch arguments of the tracking matchers (track_kernels.hip), shared
// with the host entry points (orbg_api.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "../../include/orbg.h"

namespace orbg {

// one batch of frames: F = CurrentFrame / F, queries = LastFrame points / local map points
struct TrackArgs {
    const orbg_keypoint *kps;   // [B][fc]  mvKeysUn (x, y, angle, octave)
    const uint8_t *desc;        // [B][fc][32]
    const float *uright;        // [B][fc]  mvuRight, or null (monocular)
    const uint8_t *taken0;      // [B][fc]  initial mvpMapPoints[i] && Observations() > 0, or null
    const int32_t *counts;      // [B]      N
    const orbg_bounds *bounds;  // [B]      mnMinX .. mnMaxY
    int fc;
    const void *q;              // [B][qc]  orbg_lastframe_point / orbg_map_projection
    const uint8_t *qdesc;       // [B][qc][32]
    const int32_t *qcounts;     // [B]
    int qc;
    const orbg_track_camera *cams;  // [B] (last-frame search)
    float scale[ORBG_MAX_LEVELS];   // mvScaleFactors
    float th, nnratio;
    int check_ori;
    unsigned long long *topk;   // [B][qc][K]  (scratch)
    int32_t *topn;              // [B][qc]  candidates (-1: query skipped before the search)
    int32_t *match;             // [B][fc]  query index per keypoint, -1
    int32_t *nmatches;          // [B]
    const orbg_frustum_camera *fcams;  // [B] (relocalization / loop searches)
    int orb_dist;               // relocalization: ORBdist
};

enum { TRK_LASTFRAME = 0, TRK_LOCAL = 1, TRK_RELOC = 2, TRK_LOOP = 3 };

int launch_track(hipStream_t st, int mode, const TrackArgs &A, int nframes, void *prof);

}  // namespace orbg
