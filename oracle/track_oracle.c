/*
 * oracle/track_oracle.c -- TEST INFRASTRUCTURE ONLY (see orb_oracle.h).
 *
 * Plain-C restatement of the per-frame tracking matchers:
 *   ORBmatcher::SearchByProjection(CurrentFrame, LastFrame, th, bMono)
 *       src/ORBmatcher.cc:1503-1667 (motion-model tracking, Tracking.cc TrackWithMotionModel)
 *   ORBmatcher::SearchByProjection(F, vpMapPoints, th)
 *       src/ORBmatcher.cc:59-146 with RadiusByViewingCos :148-154 (local-map tracking)
 * over the Frame grid (Frame.cc:292-307, 421-504; match_oracle.c).
 *
 * MapPoint / Frame state enters as flat records (orb_oracle.h: orc_lf_point,
 * orc_map_proj): what the two loops read of pMP (world position or projection,
 * descriptor, Observations() > 0) and of the frames.  The outputs are the loops' writes:
 * CurrentFrame.mvpMapPoints as a query index per keypoint (-1 = untouched / NULL) and
 * nmatches.
 *
 * cv::Mat float pins (OpenCV is not in the image): Rcw*x3Dw+tcw and the pose algebra of
 * :1511-1519 go through cv::gemm's small-matrix path, restated with a double work type
 * and one rounding to float per element (orc_gemm3).  Scalar float expressions keep the
 * reference's evaluation order with no FMA contraction (-ffp-contract=off).
 */
#include "orc_grid.h"

#include <limits.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define TH_HIGH 100  /* ORBmatcher.cc:37 */

void orc_gemm3(const float *R, int transR, const float *x, float alpha, const float *c,
               float *out)
{
    for (int r = 0; r < 3; r++) {
        double t = 0.0;
        for (int k = 0; k < 3; k++) {
            const float a = transR ? R[4 * k + r] : R[4 * r + k];
            t += (double)a * (double)x[k];
        }
        t *= (double)alpha;
        if (c)
            t += (double)c[r];
        out[r] = (float)t;
    }
}

void orc_track_direction(const orc_track_cam *cam, int *forward, int *backward)
{
    /* ORBmatcher.cc:1511-1522; R/t are the 3x3 / 3x1 blocks of the 3x4 row-major poses */
    const float tcw[3] = {cam->Tcw[3], cam->Tcw[7], cam->Tcw[11]};
    const float tlw[3] = {cam->Tlw[3], cam->Tlw[7], cam->Tlw[11]};
    float twc[3], tlc[3];
    orc_gemm3(cam->Tcw, 1, tcw, -1.0f, NULL, twc);  /* twc = -Rcw.t()*tcw */
    orc_gemm3(cam->Tlw, 0, twc, 1.0f, tlw, tlc);    /* tlc = Rlw*twc+tlw */
    *forward = tlc[2] > cam->b && !cam->mono;
    *backward = -tlc[2] > cam->b && !cam->mono;
}

static int rot_bin(float a1, float a2)
{
    /* ORBmatcher.cc:1635-1641 */
    const float factor = 1.0f / HISTO_LENGTH;
    float rot = a1 - a2;
    if (rot < 0.0)
        rot += 360.0f;
    int bin = (int)roundf(rot * factor);
    if (bin == HISTO_LENGTH)
        bin = 0;
    return bin;
}

int orc_search_by_projection_lastframe(const orc_keypoint *kps, const uint8_t *desc,
                                       const float *uright, int n, const uint8_t *taken0,
                                       const orc_bounds *b, const float *scale_factors,
                                       const orc_lf_point *pts, const uint8_t *pdesc, int np,
                                       const orc_track_cam *cam, float th, int check_ori,
                                       int32_t *match)
{
    int nmatches = 0;
    ogrid g;
    orc_grid_build(&g, kps, n, b);
    /* taken[i2]: CurrentFrame.mvpMapPoints[i2] && ->Observations() > 0 */
    uint8_t *taken = (uint8_t *)calloc(n > 0 ? n : 1, 1);
    for (int i = 0; i < n; i++) {
        match[i] = -1;
        taken[i] = taken0 ? taken0[i] : 0;
    }
    int fwd, bwd;
    orc_track_direction(cam, &fwd, &bwd);
    const float tcw[3] = {cam->Tcw[3], cam->Tcw[7], cam->Tcw[11]};
    int *cand = (int *)malloc(sizeof(int) * (n > 0 ? n : 1));
    /* rotHist[bin] as (bin, i2) pushes in push order */
    int *push_bin = (int *)malloc(sizeof(int) * (np > 0 ? np : 1));
    int *push_idx = (int *)malloc(sizeof(int) * (np > 0 ? np : 1));
    int npush = 0, hsize[HISTO_LENGTH];
    memset(hsize, 0, sizeof(hsize));

    for (int i = 0; i < np; i++) {
        const orc_lf_point *P = &pts[i];
        if (!(P->flags & ORC_MP_VALID))
            continue;
        const float x3Dw[3] = {P->x, P->y, P->z};
        float x3Dc[3];
        orc_gemm3(cam->Tcw, 0, x3Dw, 1.0f, tcw, x3Dc);
        const float xc = x3Dc[0], yc = x3Dc[1];
        const float invzc = (float)(1.0 / (double)x3Dc[2]);
        if (invzc < 0)
            continue;
        const float u = cam->fx * xc * invzc + cam->cx;
        const float v = cam->fy * yc * invzc + cam->cy;
        if (u < b->min_x || u > b->max_x)
            continue;
        if (v < b->min_y || v > b->max_y)
            continue;
        const int nLastOctave = P->octave;
        const float radius = th * scale_factors[nLastOctave];
        int nc;
        if (fwd)
            nc = orc_features_in_area(&g, kps, u, v, radius, nLastOctave, -1, cand);
        else if (bwd)
            nc = orc_features_in_area(&g, kps, u, v, radius, 0, nLastOctave, cand);
        else
            nc = orc_features_in_area(&g, kps, u, v, radius, nLastOctave - 1, nLastOctave + 1,
                                      cand);
        if (nc == 0)
            continue;
        int bestDist = 256, bestIdx2 = -1;
        for (int k = 0; k < nc; k++) {
            const int i2 = cand[k];
            if (taken[i2])
                continue;
            if (uright && uright[i2] > 0) {
                const float ur = u - cam->bf * invzc;
                const float er = fabsf(ur - uright[i2]);
                if (er > radius)
                    continue;
            }
            const int dist = orc_descriptor_distance(pdesc + (size_t)i * 32, desc + (size_t)i2 * 32);
            if (dist < bestDist) {
                bestDist = dist;
                bestIdx2 = i2;
            }
        }
        if (bestDist <= TH_HIGH) {
            match[bestIdx2] = i;
            taken[bestIdx2] = (P->flags & ORC_MP_HAS_OBS) ? 1 : 0;
            nmatches++;
            if (check_ori) {
                const int bin = rot_bin(P->angle, kps[bestIdx2].angle);
                push_bin[npush] = bin;
                push_idx[npush++] = bestIdx2;
                hsize[bin]++;
            }
        }
    }
    if (check_ori) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        orc_three_maxima(hsize, &ind1, &ind2, &ind3);
        /* :1651-1663: every push in a dropped bin sets its slot to NULL and decrements */
        for (int k = 0; k < npush; k++) {
            const int bn = push_bin[k];
            if (bn != ind1 && bn != ind2 && bn != ind3) {
                match[push_idx[k]] = -2; /* NULLed by the rotation filter */
                nmatches--;
            }
        }
    }
    free(cand);
    free(push_bin);
    free(push_idx);
    free(taken);
    orc_grid_free(&g);
    return nmatches;
}

int orc_search_by_projection_local(const orc_keypoint *kps, const uint8_t *desc,
                                   const float *uright, int n, const uint8_t *taken0,
                                   const orc_bounds *b, const float *scale_factors,
                                   const orc_map_proj *mps, const uint8_t *mdesc, int nm,
                                   float th, float nnratio, int32_t *match)
{
    int nmatches = 0;
    ogrid g;
    orc_grid_build(&g, kps, n, b);
    uint8_t *taken = (uint8_t *)calloc(n > 0 ? n : 1, 1);
    for (int i = 0; i < n; i++) {
        match[i] = -1;
        taken[i] = taken0 ? taken0[i] : 0;
    }
    int *cand = (int *)malloc(sizeof(int) * (n > 0 ? n : 1));
    const int bFactor = th != 1.0;
    for (int iMP = 0; iMP < nm; iMP++) {
        const orc_map_proj *M = &mps[iMP];
        if (!(M->flags & ORC_MP_VALID))
            continue;
        const int nPredictedLevel = M->level;
        /* RadiusByViewingCos, ORBmatcher.cc:148-154 */
        float r = M->view_cos > 0.998 ? 2.5f : 4.0f;
        if (bFactor)
            r *= th;
        const float rs = r * scale_factors[nPredictedLevel];
        const int nc = orc_features_in_area(&g, kps, M->u, M->v, rs, nPredictedLevel - 1,
                                            nPredictedLevel, cand);
        if (nc == 0)
            continue;
        int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
        for (int k = 0; k < nc; k++) {
            const int idx = cand[k];
            if (taken[idx])
                continue;
            if (uright && uright[idx] > 0) {
                const float er = fabsf(M->ur - uright[idx]);
                if (er > r * scale_factors[nPredictedLevel])
                    continue;
            }
            const int dist = orc_descriptor_distance(mdesc + (size_t)iMP * 32, desc + (size_t)idx * 32);
            if (dist < bestDist) {
                bestDist2 = bestDist;
                bestDist = dist;
                bestLevel2 = bestLevel;
                bestLevel = kps[idx].octave;
                bestIdx = idx;
            } else if (dist < bestDist2) {
                bestLevel2 = kps[idx].octave;
                bestDist2 = dist;
            }
        }
        if (bestDist <= TH_HIGH) {
            if (bestLevel == bestLevel2 && bestDist > nnratio * bestDist2)
                continue;
            match[bestIdx] = iMP;
            taken[bestIdx] = (M->flags & ORC_MP_HAS_OBS) ? 1 : 0;
            nmatches++;
        }
    }
    free(cand);
    free(taken);
    orc_grid_free(&g);
    return nmatches;
}
