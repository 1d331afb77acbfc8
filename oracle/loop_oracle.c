/*
 * oracle/loop_oracle.c -- TEST INFRASTRUCTURE ONLY (see orb_oracle.h).
 *
 * Plain-C restatement of the two remaining projection matchers:
 *   ORBmatcher::SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist)
 *       src/ORBmatcher.cc:1670-1798 (Tracking::Relocalization, Tracking.cc:2120, 2141)
 *   ORBmatcher::SearchByProjection(pKF, Scw, vpPoints, vpMatched, th)
 *       src/ORBmatcher.cc:353-470 (LoopClosing::ComputeSim3, LoopClosing.cc:669)
 * over the Frame / KeyFrame grid (orc_grid.h).  Both loops write into a keypoint-indexed
 * array (CurrentFrame.mvpMapPoints / vpMatched) and skip keypoints already written, so the
 * outputs are that array as a query index per keypoint (-1 untouched, -2 NULLed by the
 * rotation filter) and nmatches.  The pins are track_oracle.c's (cv::gemm with a double work
 * type, norm / dot in double) and mapping_oracle.c's Sim3 decomposition.
 */
#include "orc_grid.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* MapPoint::PredictScale (MapPoint.cc:575-590 / the Frame overload :592-607) */
static int predict_scale(float max_dist, float dist, float log_sf, int nlevels)
{
    const float ratio = max_dist / dist;
    int n = (int)ceil(log((double)ratio) / (double)log_sf);
    if (n < 0)
        n = 0;
    else if (n >= nlevels)
        n = nlevels - 1;
    return n;
}

static float norm3(const float *p)
{
    double s = 0.0;
    for (int k = 0; k < 3; k++)
        s += (double)p[k] * (double)p[k];
    return (float)sqrt(s);
}

int orc_search_by_projection_reloc(const orc_keypoint *kps, const uint8_t *desc, int n,
                                   const uint8_t *taken0, const orc_frustum_cam *cam,
                                   const float *scale_factors, const orc_reloc_point *pts,
                                   const uint8_t *pdesc, int np, float th, int orb_dist,
                                   int check_ori, int32_t *match)
{
    int nmatches = 0;
    ogrid g;
    orc_grid_build(&g, kps, n, &cam->bounds);
    const orc_bounds *b = &cam->bounds;
    /* taken[i2] = CurrentFrame.mvpMapPoints[i2] != NULL */
    uint8_t *taken = (uint8_t *)calloc(n > 0 ? n : 1, 1);
    for (int i = 0; i < n; i++) {
        match[i] = -1;
        taken[i] = taken0 ? taken0[i] : 0;
    }
    const float tcw[3] = {cam->Tcw[3], cam->Tcw[7], cam->Tcw[11]};
    float Ow[3];
    orc_gemm3(cam->Tcw, 1, tcw, -1.0f, NULL, Ow); /* -Rcw.t()*tcw */
    int *cand = (int *)malloc(sizeof(int) * (n > 0 ? n : 1));
    int *push_bin = (int *)malloc(sizeof(int) * (np > 0 ? np : 1));
    int *push_idx = (int *)malloc(sizeof(int) * (np > 0 ? np : 1));
    int npush = 0, hsize[HISTO_LENGTH];
    memset(hsize, 0, sizeof(hsize));
    const float factor = 1.0f / HISTO_LENGTH;
    for (int i = 0; i < np; i++) {
        const orc_reloc_point *P = &pts[i];
        if (!(P->flags & ORC_MP_VALID)) /* pMP && !isBad() && !sAlreadyFound.count(pMP) */
            continue;
        const float x3Dw[3] = {P->x, P->y, P->z};
        float x3Dc[3];
        orc_gemm3(cam->Tcw, 0, x3Dw, 1.0f, tcw, x3Dc);
        const float xc = x3Dc[0], yc = x3Dc[1];
        const float invzc = (float)(1.0 / (double)x3Dc[2]);
        const float u = cam->fx * xc * invzc + cam->cx;
        const float v = cam->fy * yc * invzc + cam->cy;
        if (u < b->min_x || u > b->max_x)
            continue;
        if (v < b->min_y || v > b->max_y)
            continue;
        const float PO[3] = {x3Dw[0] - Ow[0], x3Dw[1] - Ow[1], x3Dw[2] - Ow[2]};
        const float dist3D = norm3(PO);
        const float maxDistance = 1.2f * P->max_dist;
        const float minDistance = 0.8f * P->min_dist;
        if (dist3D < minDistance || dist3D > maxDistance)
            continue;
        const int nPredictedLevel =
            predict_scale(P->max_dist, dist3D, cam->log_scale_factor, cam->nlevels);
        const float radius = th * scale_factors[nPredictedLevel];
        const int nc = orc_features_in_area(&g, kps, u, v, radius, nPredictedLevel - 1,
                                            nPredictedLevel + 1, cand);
        if (nc == 0)
            continue;
        int bestDist = 256, bestIdx2 = -1;
        for (int k = 0; k < nc; k++) {
            const int i2 = cand[k];
            if (taken[i2])
                continue;
            const int dist = orc_descriptor_distance(pdesc + (size_t)i * 32, desc + (size_t)i2 * 32);
            if (dist < bestDist) {
                bestDist = dist;
                bestIdx2 = i2;
            }
        }
        if (bestDist <= orb_dist) {
            match[bestIdx2] = i;
            taken[bestIdx2] = 1;
            nmatches++;
            if (check_ori) {
                float rot = P->angle - kps[bestIdx2].angle;
                if (rot < 0.0)
                    rot += 360.0f;
                int bin = (int)roundf(rot * factor);
                if (bin == HISTO_LENGTH)
                    bin = 0;
                push_bin[npush] = bin;
                push_idx[npush++] = bestIdx2;
                hsize[bin]++;
            }
        }
    }
    if (check_ori) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        orc_three_maxima(hsize, &ind1, &ind2, &ind3);
        for (int k = 0; k < npush; k++) {
            const int bn = push_bin[k];
            if (bn != ind1 && bn != ind2 && bn != ind3) {
                match[push_idx[k]] = -2;
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

int orc_search_by_projection_sim3(const orc_keypoint *kps, const uint8_t *desc, int n,
                                  const uint8_t *taken0, const orc_frustum_cam *cam,
                                  const float *scale_factors, const orc_map_point *mps,
                                  const uint8_t *mdesc, int nm, int th, int32_t *match)
{
    int nmatches = 0;
    /* the KeyFrame's grid is the Frame's; IsInImage and GetFeaturesInArea's cell range use
     * its int bounds (KeyFrame.h:288-291), as in Fuse (mapping_oracle.c) */
    ogrid g;
    orc_grid_build(&g, kps, n, &cam->bounds);
    ogrid gk = g;
    const float kminx = (float)(int)cam->bounds.min_x, kmaxx = (float)(int)cam->bounds.max_x;
    const float kminy = (float)(int)cam->bounds.min_y, kmaxy = (float)(int)cam->bounds.max_y;
    gk.b.min_x = kminx;
    gk.b.min_y = kminy;
    /* taken[idx] = vpMatched[idx] != NULL */
    uint8_t *taken = (uint8_t *)calloc(n > 0 ? n : 1, 1);
    for (int i = 0; i < n; i++) {
        match[i] = -1;
        taken[i] = taken0 ? taken0[i] : 0;
    }
    float Tcw[12];
    orc_sim3_decompose(cam->Tcw, Tcw);
    const float tcw[3] = {Tcw[3], Tcw[7], Tcw[11]};
    float Ow[3];
    orc_gemm3(Tcw, 1, tcw, -1.0f, NULL, Ow);
    int *cand = (int *)malloc(sizeof(int) * (n > 0 ? n : 1));
    for (int i = 0; i < nm; i++) {
        const orc_map_point *mp = &mps[i];
        if (!(mp->flags & ORC_MP_VALID)) /* !isBad() && !spAlreadyFound.count(pMP) */
            continue;
        const float P[3] = {mp->x, mp->y, mp->z};
        float Pc[3];
        orc_gemm3(Tcw, 0, P, 1.0f, tcw, Pc);
        if (Pc[2] < 0.0)
            continue;
        const float invz = 1 / Pc[2];
        const float x = Pc[0] * invz;
        const float y = Pc[1] * invz;
        const float u = cam->fx * x + cam->cx;
        const float v = cam->fy * y + cam->cy;
        if (!(u >= kminx && u < kmaxx && v >= kminy && v < kmaxy)) /* KeyFrame::IsInImage */
            continue;
        const float maxDistance = 1.2f * mp->max_dist;
        const float minDistance = 0.8f * mp->min_dist;
        const float PO[3] = {P[0] - Ow[0], P[1] - Ow[1], P[2] - Ow[2]};
        const float dist = norm3(PO);
        if (dist < minDistance || dist > maxDistance)
            continue;
        double dot = 0.0;
        dot += (double)PO[0] * (double)mp->nx;
        dot += (double)PO[1] * (double)mp->ny;
        dot += (double)PO[2] * (double)mp->nz;
        if (dot < 0.5 * (double)dist)
            continue;
        const int nPredictedLevel =
            predict_scale(mp->max_dist, dist, cam->log_scale_factor, cam->nlevels);
        const float radius = th * scale_factors[nPredictedLevel];
        /* KeyFrame::GetFeaturesInArea(u, v, radius): no level test */
        const int nc = orc_features_in_area(&gk, kps, u, v, radius, -1, -1, cand);
        if (nc == 0)
            continue;
        int bestDist = 256, bestIdx = -1;
        for (int k = 0; k < nc; k++) {
            const int idx = cand[k];
            if (taken[idx])
                continue;
            const int kpLevel = kps[idx].octave;
            if (kpLevel < nPredictedLevel - 1 || kpLevel > nPredictedLevel)
                continue;
            const int d = orc_descriptor_distance(mdesc + (size_t)i * 32, desc + (size_t)idx * 32);
            if (d < bestDist) {
                bestDist = d;
                bestIdx = idx;
            }
        }
        if (bestDist <= 50) { /* TH_LOW */
            match[bestIdx] = i;
            taken[bestIdx] = 1;
            nmatches++;
        }
    }
    free(cand);
    free(taken);
    orc_grid_free(&g);
    return nmatches;
}

/* one direction of SearchBySim3 (ORBmatcher.cc:1293-1365 / 1366-1440): the source
 * KeyFrame's points through its pose (Tsw) and M | tm (sR21 | t21 or sR12 | t12) into the
 * target KeyFrame; vn[i] = the target index of the least distance (TH_HIGH), -1 */
static void sim3_direction(const orc_keypoint *tk, const uint8_t *tdesc, int nt,
                           const orc_map_point *mps, const uint8_t *mdesc, const uint8_t *am,
                           int ns, const float *Tsw, const float *M, const float *tm,
                           const orc_sim3_pair *g, float th, const float *scale_factors, int *vn)
{
    ogrid gr;
    orc_grid_build(&gr, tk, nt, &g->bounds);
    ogrid gk = gr;
    const float kminx = (float)(int)g->bounds.min_x, kmaxx = (float)(int)g->bounds.max_x;
    const float kminy = (float)(int)g->bounds.min_y, kmaxy = (float)(int)g->bounds.max_y;
    gk.b.min_x = kminx;
    gk.b.min_y = kminy;
    const float ts[3] = {Tsw[3], Tsw[7], Tsw[11]};
    float M4[12]; /* M as a 3x4 for orc_gemm3 */
    for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++)
            M4[4 * r + c] = M[3 * r + c];
        M4[4 * r + 3] = 0.f;
    }
    int *cand = (int *)malloc(sizeof(int) * (nt > 0 ? nt : 1));
    for (int i = 0; i < ns; i++) {
        vn[i] = -1;
        const orc_map_point *mp = &mps[i];
        if (!(mp->flags & ORC_MP_VALID) || (am && am[i]))
            continue;
        const float P[3] = {mp->x, mp->y, mp->z};
        float Pcs[3], Pc[3];
        orc_gemm3(Tsw, 0, P, 1.0f, ts, Pcs);
        orc_gemm3(M4, 0, Pcs, 1.0f, tm, Pc);
        if (Pc[2] < 0.0)
            continue;
        const float invz = (float)(1.0 / (double)Pc[2]);
        const float x = Pc[0] * invz;
        const float y = Pc[1] * invz;
        const float u = g->fx * x + g->cx;
        const float v = g->fy * y + g->cy;
        if (!(u >= kminx && u < kmaxx && v >= kminy && v < kmaxy))
            continue;
        const float maxDistance = 1.2f * mp->max_dist;
        const float minDistance = 0.8f * mp->min_dist;
        const float dist3D = norm3(Pc);
        if (dist3D < minDistance || dist3D > maxDistance)
            continue;
        const int lvl = predict_scale(mp->max_dist, dist3D, g->log_scale_factor, g->nlevels);
        const float radius = th * scale_factors[lvl];
        const int nc = orc_features_in_area(&gk, tk, u, v, radius, -1, -1, cand);
        int bestDist = 1 << 30, bestIdx = -1;
        for (int k = 0; k < nc; k++) {
            const int idx = cand[k];
            const int o = tk[idx].octave;
            if (o < lvl - 1 || o > lvl)
                continue;
            const int d = orc_descriptor_distance(mdesc + (size_t)i * 32, tdesc + (size_t)idx * 32);
            if (d < bestDist) {
                bestDist = d;
                bestIdx = idx;
            }
        }
        if (bestDist <= 100) /* TH_HIGH */
            vn[i] = bestIdx;
    }
    free(cand);
    orc_grid_free(&gr);
}

int orc_search_by_sim3(const orc_keypoint *k1, const uint8_t *d1, int n1, const orc_map_point *mp1,
                       const uint8_t *md1, const uint8_t *matched1, const orc_keypoint *k2,
                       const uint8_t *d2, int n2, const orc_map_point *mp2, const uint8_t *md2,
                       const uint8_t *matched2, const orc_sim3_pair *g, float th,
                       const float *scale_factors, int32_t *matches12)
{
    /* sR12 = s12*R12, sR21 = (1.0/s12)*R12.t(): Mat * scalar = convertTo with the float
     * alpha (one rounding per element); t21 = -sR21*t12 by gemm (ORBmatcher.cc:1275-1279) */
    float sR12[9], sR21[9], t21[3];
    const float a = (float)(1.0 / (double)g->s12);
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) {
            sR12[3 * r + c] = g->R12[3 * r + c] * g->s12 + 0.0f;
            sR21[3 * r + c] = g->R12[3 * c + r] * a + 0.0f;
        }
    for (int r = 0; r < 3; r++) {
        double t = 0.0;
        for (int k = 0; k < 3; k++)
            t += (double)sR21[3 * r + k] * (double)g->t12[k];
        t21[r] = (float)(t * -1.0);
    }
    int *vn1 = (int *)malloc(sizeof(int) * (n1 > 0 ? n1 : 1));
    int *vn2 = (int *)malloc(sizeof(int) * (n2 > 0 ? n2 : 1));
    sim3_direction(k2, d2, n2, mp1, md1, matched1, n1, g->T1w, sR21, t21, g, th, scale_factors, vn1);
    sim3_direction(k1, d1, n1, mp2, md2, matched2, n2, g->T2w, sR12, g->t12, g, th, scale_factors,
                   vn2);
    int nFound = 0;
    for (int i1 = 0; i1 < n1; i1++) {
        matches12[i1] = -1;
        const int idx2 = vn1[i1];
        if (idx2 >= 0 && vn2[idx2] == i1) {
            matches12[i1] = idx2;
            nFound++;
        }
    }
    free(vn1);
    free(vn2);
    return nFound;
}
