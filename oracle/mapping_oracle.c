/*
 * oracle/mapping_oracle.c -- TEST INFRASTRUCTURE ONLY (see orb_oracle.h).
 *
 * Plain-C restatement of LocalMapping's per-keyframe Hamming matchers:
 *   ORBmatcher::SearchForTriangulation(pKF1, pKF2, F12, vMatchedPairs, bOnlyStereo)
 *       src/ORBmatcher.cc:779-957 with CheckDistEpipolarLine :165-182 and ComputeThreeMaxima
 *       :1800-1841 (caller LocalMapping::CreateNewMapPoints, LocalMapping.cc:305-378)
 *   ORBmatcher::Fuse(pKF, vpMapPoints, th) -- the per-MapPoint search
 *       src/ORBmatcher.cc:968-1107 over KeyFrame::GetFeaturesInArea / IsInImage
 *       (caller LocalMapping::SearchInNeighbors, LocalMapping.cc:622-690)
 *
 * KeyFrame state enters as flat arrays: mvKeysUn, mDescriptors, mvuRight (< 0: monocular
 * observation), has_mp[i] = (GetMapPoint(i) != NULL) and the FeatureVector (node ids
 * ascending, feature lists in order), as orc_search_by_bow takes it.
 *
 * Notes on the reference's semantics kept here:
 *   - vbMatched2 is never set (ORBmatcher.cc:810, 898-904): one KF2 feature can be the match
 *     of several KF1 features;
 *   - a candidate replaces the best on dist <= bestDist (`dist>bestDist` skips, :872) once it
 *     passes the epipole and epipolar tests, so the LAST passing candidate of the least
 *     distance wins, starting from bestDist = TH_LOW;
 *   - CheckDistEpipolarLine compares the float dsqr against 3.84 * sigma2 in double.
 *   - Fuse: the search (projection, gates, GetFeaturesInArea order, strict dist < bestDist)
 *     reads only the KeyFrame's keypoints and the MapPoint's position / normal / distances /
 *     descriptor; what the reference then does with the match (Replace, AddObservation) is
 *     the caller's sequential map update, so the restatement returns bestIdx per MapPoint.
 */
#include "orc_grid.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#define TRI_TH_LOW 50

static int tri_rot_bin(float a1, float a2)
{
    const float factor = 1.0f / HISTO_LENGTH;
    float rot = a1 - a2;
    if (rot < 0.0)
        rot += 360.0f;
    int bin = (int)roundf(rot * factor);
    if (bin == HISTO_LENGTH)
        bin = 0;
    return bin;
}

/* CheckDistEpipolarLine (ORBmatcher.cc:165-182) */
static int tri_epipolar_ok(const orc_keypoint *kp1, const orc_keypoint *kp2, const float F[9],
                           const float *sigma2)
{
    const float a = kp1->x * F[0] + kp1->y * F[3] + F[6];
    const float b = kp1->x * F[1] + kp1->y * F[4] + F[7];
    const float c = kp1->x * F[2] + kp1->y * F[5] + F[8];
    const float num = a * kp2->x + b * kp2->y + c;
    const float den = a * a + b * b;
    if (den == 0)
        return 0;
    const float dsqr = num * num / den;
    return (double)dsqr < 3.84 * (double)sigma2[kp2->octave];
}

int orc_search_for_triangulation(const orc_tri_kf *kf1, const orc_tri_kf *kf2,
                                 const orc_tri_geom *g, const float *scale_factors,
                                 const float *sigma2, int only_stereo, int check_ori,
                                 int32_t *matches12)
{
    /* epipole of KF1's centre in KF2 (:800-806): C2 = R2w*Cw+t2w (cv::gemm pin) */
    const float t2w[3] = {g->Tcw2[3], g->Tcw2[7], g->Tcw2[11]};
    float C2[3];
    orc_gemm3(g->Tcw2, 0, g->Cw1, 1.0f, t2w, C2);
    const float invz = 1.0f / C2[2];
    const float ex = g->fx2 * C2[0] * invz + g->cx2;
    const float ey = g->fy2 * C2[1] * invz + g->cy2;

    for (int i = 0; i < kf1->n; i++)
        matches12[i] = -1;
    int *bins = (int *)malloc(sizeof(int) * (kf1->n > 0 ? kf1->n : 1));
    int hsize[HISTO_LENGTH];
    memset(hsize, 0, sizeof(hsize));
    int nmatches = 0;
    int a = 0, b = 0;
    while (a < kf1->nfv && b < kf2->nfv) {
        if (kf1->fv_nodes[a] == kf2->fv_nodes[b]) {
            for (int i1 = kf1->fv_off[a]; i1 < kf1->fv_off[a + 1]; i1++) {
                const int idx1 = kf1->fv_feats[i1];
                if (kf1->has_mp[idx1])
                    continue;
                const int bStereo1 = kf1->uright[idx1] >= 0;
                if (only_stereo && !bStereo1)
                    continue;
                const orc_keypoint *kp1 = &kf1->kps[idx1];
                const uint8_t *d1 = kf1->desc + (size_t)idx1 * 32;
                int bestDist = TRI_TH_LOW, bestIdx2 = -1;
                for (int i2 = kf2->fv_off[b]; i2 < kf2->fv_off[b + 1]; i2++) {
                    const int idx2 = kf2->fv_feats[i2];
                    if (kf2->has_mp[idx2])  /* vbMatched2[idx2] is never set */
                        continue;
                    const int bStereo2 = kf2->uright[idx2] >= 0;
                    if (only_stereo && !bStereo2)
                        continue;
                    const int dist = orc_descriptor_distance(d1, kf2->desc + (size_t)idx2 * 32);
                    if (dist > TRI_TH_LOW || dist > bestDist)
                        continue;
                    const orc_keypoint *kp2 = &kf2->kps[idx2];
                    if (!bStereo1 && !bStereo2) {
                        const float distex = ex - kp2->x;
                        const float distey = ey - kp2->y;
                        if (distex * distex + distey * distey < 100 * scale_factors[kp2->octave])
                            continue;
                    }
                    if (tri_epipolar_ok(kp1, kp2, g->F12, sigma2)) {
                        bestIdx2 = idx2;
                        bestDist = dist;
                    }
                }
                if (bestIdx2 >= 0) {
                    matches12[idx1] = bestIdx2;
                    nmatches++;
                    if (check_ori) {
                        const int bin = tri_rot_bin(kp1->angle, kf2->kps[bestIdx2].angle);
                        bins[idx1] = bin;
                        hsize[bin]++;
                    }
                }
            }
            a++;
            b++;
        } else if (kf1->fv_nodes[a] < kf2->fv_nodes[b]) {
            a++;
        } else {
            b++;
        }
    }
    if (check_ori) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        orc_three_maxima(hsize, &ind1, &ind2, &ind3);
        for (int i = 0; i < kf1->n; i++)
            if (matches12[i] >= 0 && bins[i] != ind1 && bins[i] != ind2 && bins[i] != ind3) {
                matches12[i] = -1;
                nmatches--;
            }
    }
    free(bins);
    return nmatches;
}

/* The Sim3 decomposition at the top of ORBmatcher::Fuse(pKF, Scw, ...) (ORBmatcher.cc:
 * 1143-1148): scw = sqrt(sRcw.row(0).dot(sRcw.row(0))) -- Mat::dot of floats sums double
 * products (the dot pin of isInFrustum) and the float scw is the double root rounded; Rcw =
 * sRcw / scw and tcw = t / scw are Mat / double, i.e. convertTo with the float alpha
 * (float)(1 / scw) and shift 0: each element x * alpha rounded once (+ 0.0f). */
void orc_sim3_decompose(const float *Scw, float *Tcw)
{
    double d = 0.0;
    for (int k = 0; k < 3; k++)
        d += (double)Scw[k] * (double)Scw[k];
    const float scw = (float)sqrt(d);
    const float a = (float)(1.0 / (double)scw);
    for (int k = 0; k < 12; k++)
        Tcw[k] = Scw[k] * a + 0.0f;
}

static int fuse_search(const orc_tri_kf *kf, const orc_frustum_cam *cam0, const orc_map_point *mps,
                       const uint8_t *mdesc, int nmp, float th, const float *scale_factors,
                       const float *inv_sigma2, int sim3, int32_t *best_idx, int32_t *best_dist)
{
    orc_frustum_cam camd = *cam0;
    const orc_frustum_cam *cam = &camd;
    if (sim3)
        orc_sim3_decompose(cam0->Tcw, camd.Tcw);
    /* the KeyFrame's grid is the Frame's (mGrid and mfGridElementWidthInv copied from the
     * Frame, float bounds), its mnMinX .. mnMaxY are ints (KeyFrame.h:288-291, the Frame's
     * truncated, KeyFrame.cc:51): IsInImage and GetFeaturesInArea's cell range use those */
    ogrid g;
    orc_grid_build(&g, kf->kps, kf->n, &cam->bounds);
    ogrid gk = g;
    const float kminx = (float)(int)cam->bounds.min_x, kmaxx = (float)(int)cam->bounds.max_x;
    const float kminy = (float)(int)cam->bounds.min_y, kmaxy = (float)(int)cam->bounds.max_y;
    gk.b.min_x = kminx;
    gk.b.min_y = kminy;
    int *cand = (int *)malloc(sizeof(int) * (kf->n > 0 ? kf->n : 1));
    const float tcw[3] = {cam->Tcw[3], cam->Tcw[7], cam->Tcw[11]};
    float Ow[3];
    orc_gemm3(cam->Tcw, 1, tcw, -1.0f, NULL, Ow); /* KeyFrame::GetCameraCenter */
    int nfused = 0;
    for (int i = 0; i < nmp; i++) {
        best_idx[i] = -1;
        best_dist[i] = 256;
        const orc_map_point *mp = &mps[i];
        if (!(mp->flags & ORC_MP_VALID)) /* !pMP, isBad() or IsInKeyFrame(pKF) */
            continue;
        const float P[3] = {mp->x, mp->y, mp->z};
        float Pc[3];
        orc_gemm3(cam->Tcw, 0, P, 1.0f, tcw, Pc); /* Rcw*p3Dw + tcw */
        if (Pc[2] < 0.0f)
            continue;
        const float invz = 1 / Pc[2];
        const float x = Pc[0] * invz;
        const float y = Pc[1] * invz;
        const float u = cam->fx * x + cam->cx;
        const float v = cam->fy * y + cam->cy;
        /* KeyFrame::IsInImage (KeyFrame.cc:792-795) */
        if (!(u >= kminx && u < kmaxx && v >= kminy && v < kmaxy))
            continue;
        const float ur = u - cam->bf * invz;
        const float maxDistance = 1.2f * mp->max_dist;
        const float minDistance = 0.8f * mp->min_dist;
        const float PO[3] = {P[0] - Ow[0], P[1] - Ow[1], P[2] - Ow[2]};
        double s = 0.0;
        for (int k = 0; k < 3; k++)
            s += (double)PO[k] * (double)PO[k];
        const float dist3D = (float)sqrt(s);
        if (dist3D < minDistance || dist3D > maxDistance)
            continue;
        double dot = 0.0;
        dot += (double)PO[0] * (double)mp->nx;
        dot += (double)PO[1] * (double)mp->ny;
        dot += (double)PO[2] * (double)mp->nz;
        if (dot < 0.5 * (double)dist3D)
            continue;
        const float ratio = mp->max_dist / dist3D;
        int nPredictedLevel = (int)ceil(log((double)ratio) / (double)cam->log_scale_factor);
        if (nPredictedLevel < 0)
            nPredictedLevel = 0;
        else if (nPredictedLevel >= cam->nlevels)
            nPredictedLevel = cam->nlevels - 1;
        const float radius = th * scale_factors[nPredictedLevel];
        /* KeyFrame::GetFeaturesInArea(u, v, radius): Frame's with no level test */
        const int nc = orc_features_in_area(&gk, kf->kps, u, v, radius, -1, -1, cand);
        if (nc == 0)
            continue;
        const uint8_t *dMP = mdesc + (size_t)i * 32;
        int bestDist = 256, bestIdx = -1;
        for (int k = 0; k < nc; k++) {
            const int idx = cand[k];
            const orc_keypoint *kp = &kf->kps[idx];
            const int kpLevel = kp->octave;
            if (kpLevel < nPredictedLevel - 1 || kpLevel > nPredictedLevel)
                continue;
            if (sim3) {
                /* the Sim3 variant has no reprojection gate (ORBmatcher.cc:1218-1236) */
            } else if (kf->uright[idx] >= 0) {
                const float ex = u - kp->x, ey = v - kp->y, er = ur - kf->uright[idx];
                const float e2 = ex * ex + ey * ey + er * er;
                if ((double)(e2 * inv_sigma2[kpLevel]) > 7.8)
                    continue;
            } else {
                const float ex = u - kp->x, ey = v - kp->y;
                const float e2 = ex * ex + ey * ey;
                if ((double)(e2 * inv_sigma2[kpLevel]) > 5.99)
                    continue;
            }
            const int dist = orc_descriptor_distance(dMP, kf->desc + (size_t)idx * 32);
            if (dist < bestDist) {
                bestDist = dist;
                bestIdx = idx;
            }
        }
        best_dist[i] = bestDist;
        if (bestDist <= TRI_TH_LOW) {
            best_idx[i] = bestIdx;
            nfused++;
        }
    }
    free(cand);
    orc_grid_free(&g);
    return nfused;
}

/* ORBmatcher::Fuse(pKF, vpMapPoints, th), the per-MapPoint search (ORBmatcher.cc:968-1069):
 * best_idx[i] = bestIdx when bestDist <= TH_LOW (the reference then fuses), else -1;
 * best_dist[i] = bestDist (256: no candidate passed or the point was skipped). */
int orc_fuse_search(const orc_tri_kf *kf, const orc_frustum_cam *cam, const orc_map_point *mps,
                    const uint8_t *mdesc, int nmp, float th, const float *scale_factors,
                    const float *inv_sigma2, int32_t *best_idx, int32_t *best_dist)
{
    return fuse_search(kf, cam, mps, mdesc, nmp, th, scale_factors, inv_sigma2, 0, best_idx,
                       best_dist);
}

/* ORBmatcher::Fuse(pKF, Scw, vpPoints, th, vpReplacePoint)'s search (ORBmatcher.cc:1133-1238,
 * LoopClosing::SearchAndFuse): cam->Tcw holds Scw's rows 0..2 (sR | t), decomposed as above;
 * the projection, IsInImage, distance, angle and scale gates are Fuse's, the candidates are
 * ranked by descriptor distance alone (no reprojection gate, mvuRight unused).  Same outputs;
 * the replace / add update (:1239-1254) is the caller's, in vpPoints order. */
int orc_fuse_sim3_search(const orc_tri_kf *kf, const orc_frustum_cam *cam,
                         const orc_map_point *mps, const uint8_t *mdesc, int nmp, float th,
                         const float *scale_factors, int32_t *best_idx, int32_t *best_dist)
{
    return fuse_search(kf, cam, mps, mdesc, nmp, th, scale_factors, NULL, 1, best_idx, best_dist);
}
