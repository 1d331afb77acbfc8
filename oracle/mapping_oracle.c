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

/* ===================================================================================
 * LocalMapping::CreateNewMapPoints' per-pair geometry and per-match triangulation
 * (src/LocalMapping.cc:293-560) and LocalMapping::ComputeF12 (:690-707).
 *
 * cv::Mat float arithmetic as OpenCV 3.4 evaluates it (recalled, unpinned against a real
 * build, like the other cv:: pins of this oracle):
 *   - gemm (A*B, A*B+C, alpha): double work type, one rounding per element (orc_gemm3);
 *   - Mat::dot / cv::norm of float vectors: double accumulation in order;
 *   - A.inv()*B with DECOMP_LU and B of more than one column is solve(A, B): the float LU
 *     with partial pivoting of hal::LU32f (LUImpl: d = -1/A[i][i], alpha = A[j][i]*d,
 *     A[j][k] += alpha*A[i][k], b likewise, then back substitution with the stored 1/A[i][i]);
 *   - B*A.inv(): invert()'s closed form for a 3x3 float (det3 and the cofactors in double,
 *     times 1/det, rounded);
 *   - Mat / double: convertTo with a float alpha (one rounding);
 *   - scalar*Mat - Mat: addWeighted in float, r2*a + r0*(-1) (+0).
 * cos(2*atan2(mb/2, depth)) takes float arguments: glibc's atan2f (flt-32 e_atan2f.c /
 * s_atanf.c, fdlibm's algorithm, restated in orc_atan2f and pinned against the host libm by
 * tests/test_oracle_mapping.py) and cosf (orc_sinf_cosf).  cv::SVD::compute of the 4x4
 * linear-triangulation system is replaced by the null vector of A^T A from a cyclic Jacobi
 * eigen-decomposition in double (fixed rotation order, at most 12 sweeps): the same vector up
 * to scale and float rounding, not OpenCV's float one-sided Jacobi bits (parity unpinned).
 * =================================================================================== */

/* glibc / fdlibm atanf (s_atanf.c) for |x| < 2^26 and atan2f (e_atan2f.c), float
 * arithmetic, no FMA (-ffp-contract=off) */
static const float orc_atanhi[4] = {4.6364760399e-01f, 7.8539812565e-01f, 9.8279368877e-01f,
                                    1.5707962513e+00f};
static const float orc_atanlo[4] = {5.0121582440e-09f, 3.7748947079e-08f, 3.4473217170e-08f,
                                    7.5497894159e-08f};
static const float orc_aT[11] = {3.3333334327e-01f,  -2.0000000298e-01f, 1.4285714924e-01f,
                                 -1.1111110449e-01f, 9.0908870101e-02f,  -7.6918758452e-02f,
                                 6.6610731184e-02f,  -5.8335702866e-02f, 4.9768779427e-02f,
                                 -3.6531571299e-02f, 1.6285819933e-02f};

static uint32_t orc_fbits(float f)
{
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
}

static float orc_atanf(float x)
{
    const int32_t hx = (int32_t)orc_fbits(x), ix = hx & 0x7fffffff;
    int id;
    if (ix >= 0x4c000000) { /* |x| >= 2^25 (glibc's bound; fdlibm's is 2^26) */
        if (ix > 0x7f800000)
            return x + x;
        return hx > 0 ? orc_atanhi[3] + orc_atanlo[3] : -orc_atanhi[3] - orc_atanlo[3];
    }
    if (ix < 0x3ee00000) {     /* |x| < 0.4375 */
        if (ix < 0x31000000) /* |x| < 2^-29 */
            return x;
        id = -1;
    } else {
        x = fabsf(x);
        if (ix < 0x3f980000) {     /* |x| < 1.1875 */
            if (ix < 0x3f300000) { /* 7/16 <= |x| < 11/16 */
                id = 0;
                x = (2.0f * x - 1.0f) / (2.0f + x);
            } else { /* 11/16 <= |x| < 19/16 */
                id = 1;
                x = (x - 1.0f) / (x + 1.0f);
            }
        } else {
            if (ix < 0x401c0000) { /* |x| < 2.4375 */
                id = 2;
                x = (x - 1.5f) / (1.0f + 1.5f * x);
            } else { /* 2.4375 <= |x| < 2^26 */
                id = 3;
                x = -1.0f / x;
            }
        }
    }
    const float z = x * x, w = z * z;
    const float s1 = z * (orc_aT[0] + w * (orc_aT[2] + w * (orc_aT[4] + w * (orc_aT[6] + w * (orc_aT[8] + w * orc_aT[10])))));
    const float s2 = w * (orc_aT[1] + w * (orc_aT[3] + w * (orc_aT[5] + w * (orc_aT[7] + w * orc_aT[9]))));
    if (id < 0)
        return x - x * (s1 + s2);
    const float r = orc_atanhi[id] - ((x * (s1 + s2) - orc_atanlo[id]) - x);
    return hx < 0 ? -r : r;
}

float orc_atan2f(float y, float x)
{
    static const float tiny = 1.0e-30f, pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f,
                       pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f;
    const int32_t hx = (int32_t)orc_fbits(x), ix = hx & 0x7fffffff;
    const int32_t hy = (int32_t)orc_fbits(y), iy = hy & 0x7fffffff;
    if (ix > 0x7f800000 || iy > 0x7f800000)
        return x + y;
    if (hx == 0x3f800000)
        return orc_atanf(y);
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
    if (iy == 0) {
        switch (m) {
        case 0:
        case 1:
            return y;
        case 2:
            return pi + tiny;
        default:
            return -pi - tiny;
        }
    }
    if (ix == 0)
        return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    if (ix == 0x7f800000) {
        if (iy == 0x7f800000) {
            switch (m) {
            case 0:
                return pi_o_4 + tiny;
            case 1:
                return -pi_o_4 - tiny;
            case 2:
                return 3.0f * pi_o_4 + tiny;
            default:
                return -3.0f * pi_o_4 - tiny;
            }
        }
        switch (m) {
        case 0:
            return 0.0f;
        case 1:
            return -0.0f;
        case 2:
            return pi + tiny;
        default:
            return -pi - tiny;
        }
    }
    if (iy == 0x7f800000)
        return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    const int k = (iy - ix) >> 23;
    float z;
    if (k > 60)
        z = pi_o_2 + 0.5f * pi_lo;
    else if (hx < 0 && k < -60)
        z = 0.0f;
    else
        z = orc_atanf(fabsf(y / x));
    switch (m) {
    case 0:
        return z;
    case 1: {
        const uint32_t u = orc_fbits(z) ^ 0x80000000u;
        memcpy(&z, &u, 4);
        return z;
    }
    case 2:
        return pi - (z - pi_lo);
    default:
        return (z - pi_lo) - pi;
    }
}

/* 3x3 float matrices, row-major: C = A * B (gemm, double work, one rounding) */
static void orc_mm3(const float *A, const float *B, float *C)
{
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double t = 0.0;
            for (int k = 0; k < 3; k++)
                t += (double)A[3 * i + k] * (double)B[3 * k + j];
            C[3 * i + j] = (float)t;
        }
}

/* solve(A, B) for 3x3 float A, B (hal::LU32f, LUImpl, eps = 10 FLT_EPSILON): X into B;
 * returns 0 when singular (X then 0, as cv::solve leaves dst zeroed) */
static int orc_solve3_lu(const float *A0, float *B)
{
    float A[9];
    memcpy(A, A0, sizeof(A));
    const float eps = 10.0f * 1.19209290e-07f;
    for (int i = 0; i < 3; i++) {
        int k = i;
        for (int j = i + 1; j < 3; j++)
            if (fabsf(A[3 * j + i]) > fabsf(A[3 * k + i]))
                k = j;
        if (fabsf(A[3 * k + i]) < eps) {
            memset(B, 0, 9 * sizeof(float));
            return 0;
        }
        if (k != i) {
            for (int j = i; j < 3; j++) {
                const float t = A[3 * i + j];
                A[3 * i + j] = A[3 * k + j];
                A[3 * k + j] = t;
            }
            for (int j = 0; j < 3; j++) {
                const float t = B[3 * i + j];
                B[3 * i + j] = B[3 * k + j];
                B[3 * k + j] = t;
            }
        }
        const float d = -1.0f / A[3 * i + i];
        for (int j = i + 1; j < 3; j++) {
            const float alpha = A[3 * j + i] * d;
            for (int c = i + 1; c < 3; c++)
                A[3 * j + c] += alpha * A[3 * i + c];
            for (int c = 0; c < 3; c++)
                B[3 * j + c] += alpha * B[3 * i + c];
        }
        A[3 * i + i] = -d;
    }
    for (int i = 2; i >= 0; i--)
        for (int j = 0; j < 3; j++) {
            float s = B[3 * i + j];
            for (int c = i + 1; c < 3; c++)
                s -= A[3 * i + c] * B[3 * c + j];
            B[3 * i + j] = s * A[3 * i + i];
        }
    return 1;
}

/* invert() of a 3x3 float (closed form: det3 and cofactors in double) */
static void orc_inv3f(const float *S, float *D)
{
#define Sf(y, x) ((double)S[3 * (y) + (x)])
    double d = Sf(0, 0) * (Sf(1, 1) * Sf(2, 2) - Sf(1, 2) * Sf(2, 1)) -
               Sf(0, 1) * (Sf(1, 0) * Sf(2, 2) - Sf(1, 2) * Sf(2, 0)) +
               Sf(0, 2) * (Sf(1, 0) * Sf(2, 1) - Sf(1, 1) * Sf(2, 0));
    if (d == 0.0) {
        memset(D, 0, 9 * sizeof(float));
        return;
    }
    d = 1.0 / d;
    D[0] = (float)((Sf(1, 1) * Sf(2, 2) - Sf(1, 2) * Sf(2, 1)) * d);
    D[1] = (float)((Sf(0, 2) * Sf(2, 1) - Sf(0, 1) * Sf(2, 2)) * d);
    D[2] = (float)((Sf(0, 1) * Sf(1, 2) - Sf(0, 2) * Sf(1, 1)) * d);
    D[3] = (float)((Sf(1, 2) * Sf(2, 0) - Sf(1, 0) * Sf(2, 2)) * d);
    D[4] = (float)((Sf(0, 0) * Sf(2, 2) - Sf(0, 2) * Sf(2, 0)) * d);
    D[5] = (float)((Sf(0, 2) * Sf(1, 0) - Sf(0, 0) * Sf(1, 2)) * d);
    D[6] = (float)((Sf(1, 0) * Sf(2, 1) - Sf(1, 1) * Sf(2, 0)) * d);
    D[7] = (float)((Sf(0, 1) * Sf(2, 0) - Sf(0, 0) * Sf(2, 1)) * d);
    D[8] = (float)((Sf(0, 0) * Sf(1, 1) - Sf(0, 1) * Sf(1, 0)) * d);
#undef Sf
}

/* KeyFrame::SetPose: Ow = -Rcw.t()*tcw (gemm, alpha -1) */
static void orc_kf_center(const float *Tcw, float *Ow)
{
    const float t[3] = {Tcw[3], Tcw[7], Tcw[11]};
    orc_gemm3(Tcw, 1, t, -1.0f, NULL, Ow);
}

void orc_tri_geometry(const orc_kf_cam *c1, const orc_kf_cam *c2, orc_tri_geom *g)
{
    /* ComputeF12: R12 = R1w*R2w.t(); t12 = -R1w*R2w.t()*t2w+t1w (the -R12 product evaluated,
     * then one gemm with C); F12 = solve(K1^T, [t12]x) * R12 * inv(K2) */
    const float *T1 = c1->Tcw, *T2 = c2->Tcw;
    float R12[9], nR12[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double t = 0.0;
            for (int k = 0; k < 3; k++)
                t += (double)T1[4 * i + k] * (double)T2[4 * j + k];
            R12[3 * i + j] = (float)t;
            nR12[3 * i + j] = (float)(t * -1.0);
        }
    float t12[3];
    for (int i = 0; i < 3; i++) {
        double t = 0.0;
        for (int k = 0; k < 3; k++)
            t += (double)nR12[3 * i + k] * (double)T2[4 * k + 3];
        t += (double)T1[4 * i + 3];
        t12[i] = (float)t;
    }
    float X[9] = {0.0f, -t12[2], t12[1], t12[2], 0.0f, -t12[0], -t12[1], t12[0], 0.0f};
    const float K1t[9] = {c1->fx, 0.0f, 0.0f, 0.0f, c1->fy, 0.0f, c1->cx, c1->cy, 1.0f};
    const float K2[9] = {c2->fx, 0.0f, c2->cx, 0.0f, c2->fy, c2->cy, 0.0f, 0.0f, 1.0f};
    orc_solve3_lu(K1t, X);
    float Y[9], K2i[9];
    orc_mm3(X, R12, Y);
    orc_inv3f(K2, K2i);
    orc_mm3(Y, K2i, g->F12);
    orc_kf_center(T1, g->Cw1);
    memcpy(g->Tcw2, T2, sizeof(g->Tcw2));
    g->fx2 = c2->fx;
    g->fy2 = c2->fy;
    g->cx2 = c2->cx;
    g->cy2 = c2->cy;
}

/* the null vector of the 4x4 A (row-major float) in double: cyclic Jacobi on B = A^T A */
void orc_tri_nullvec(const float *A, double *v)
{
    double B[16], V[16];
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
            double t = 0.0;
            for (int k = 0; k < 4; k++)
                t += (double)A[4 * k + i] * (double)A[4 * k + j];
            B[4 * i + j] = t;
            V[4 * i + j] = i == j ? 1.0 : 0.0;
        }
    for (int sweep = 0; sweep < 12; sweep++) {
        double off = 0.0;
        for (int p = 0; p < 3; p++)
            for (int q = p + 1; q < 4; q++)
                off += fabs(B[4 * p + q]);
        if (off == 0.0)
            break;
        for (int p = 0; p < 3; p++)
            for (int q = p + 1; q < 4; q++) {
                const double apq = B[4 * p + q];
                if (apq == 0.0)
                    continue;
                const double theta = (B[4 * q + q] - B[4 * p + p]) / (2.0 * apq);
                double t = 1.0 / (fabs(theta) + sqrt(theta * theta + 1.0));
                if (theta < 0.0)
                    t = -t;
                const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
                for (int k = 0; k < 4; k++) { /* B = J^T B J: columns, then rows */
                    const double bkp = B[4 * k + p], bkq = B[4 * k + q];
                    B[4 * k + p] = c * bkp - s * bkq;
                    B[4 * k + q] = s * bkp + c * bkq;
                }
                for (int k = 0; k < 4; k++) {
                    const double bpk = B[4 * p + k], bqk = B[4 * q + k];
                    B[4 * p + k] = c * bpk - s * bqk;
                    B[4 * q + k] = s * bpk + c * bqk;
                }
                for (int k = 0; k < 4; k++) {
                    const double vkp = V[4 * k + p], vkq = V[4 * k + q];
                    V[4 * k + p] = c * vkp - s * vkq;
                    V[4 * k + q] = s * vkp + c * vkq;
                }
            }
    }
    int m = 0;
    for (int i = 1; i < 4; i++)
        if (B[4 * i + i] < B[4 * m + m])
            m = i;
    for (int k = 0; k < 4; k++)
        v[k] = V[4 * k + m];
}

/* Mat::dot / cv::norm of float 3-vectors */
static double orc_dot3f(const float *a, const float *b)
{
    double s = 0.0;
    for (int k = 0; k < 3; k++)
        s += (double)a[k] * (double)b[k];
    return s;
}

/* one match of CreateNewMapPoints (LocalMapping.cc:395-560): the status, X = x3D */
static int orc_triangulate_one(const orc_kf_tri *k1, const orc_kf_tri *k2, const orc_kf_cam *c1,
                               const orc_kf_cam *c2, int idx1, int idx2, const float *Ow1,
                               const float *Ow2, const float *scale_factors, const float *sigma2,
                               float ratioFactor, float *X)
{
    const float *T1 = c1->Tcw, *T2 = c2->Tcw;
    const orc_keypoint *kp1 = &k1->kps[idx1], *kp2 = &k2->kps[idx2];
    const float kp1_ur = k1->uright ? k1->uright[idx1] : -1.0f;
    const float kp2_ur = k2->uright ? k2->uright[idx2] : -1.0f;
    const int bStereo1 = kp1_ur >= 0, bStereo2 = kp2_ur >= 0;
    const float xn1[3] = {(kp1->x - c1->cx) * c1->invfx, (kp1->y - c1->cy) * c1->invfy, 1.0f};
    const float xn2[3] = {(kp2->x - c2->cx) * c2->invfx, (kp2->y - c2->cy) * c2->invfy, 1.0f};
    float ray1[3], ray2[3];
    orc_gemm3(T1, 1, xn1, 1.0f, NULL, ray1); /* Rwc1*xn1 */
    orc_gemm3(T2, 1, xn2, 1.0f, NULL, ray2);
    const float cosParallaxRays =
        (float)(orc_dot3f(ray1, ray2) / (sqrt(orc_dot3f(ray1, ray1)) * sqrt(orc_dot3f(ray2, ray2))));
    float cosParallaxStereo = cosParallaxRays + 1;
    float cosParallaxStereo1 = cosParallaxStereo, cosParallaxStereo2 = cosParallaxStereo;
    if (bStereo1)
        cosParallaxStereo1 = orc_glibc_cosf(2 * orc_atan2f(c1->mb / 2, k1->depth[idx1]));
    else if (bStereo2)
        cosParallaxStereo2 = orc_glibc_cosf(2 * orc_atan2f(c2->mb / 2, k2->depth[idx2]));
    cosParallaxStereo = cosParallaxStereo2 < cosParallaxStereo1 ? cosParallaxStereo2 : cosParallaxStereo1;
    float x3D[3];
    if (cosParallaxRays < cosParallaxStereo && cosParallaxRays > 0 &&
        (bStereo1 || bStereo2 || cosParallaxRays < 0.9998)) {
        /* A.row(r) = xn*Tcw.row(2) - Tcw.row(k): addWeighted in float */
        float A[16];
        for (int k = 0; k < 4; k++) {
            A[k] = (T1[8 + k] * xn1[0] + T1[k] * -1.0f) + 0.0f;
            A[4 + k] = (T1[8 + k] * xn1[1] + T1[4 + k] * -1.0f) + 0.0f;
            A[8 + k] = (T2[8 + k] * xn2[0] + T2[k] * -1.0f) + 0.0f;
            A[12 + k] = (T2[8 + k] * xn2[1] + T2[4 + k] * -1.0f) + 0.0f;
        }
        double v[4];
        orc_tri_nullvec(A, v);
        const float vf[4] = {(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
        if (vf[3] == 0)
            return ORC_TRI_W0;
        const float a = (float)(1.0 / (double)vf[3]); /* Mat / double: convertTo, float alpha */
        for (int k = 0; k < 3; k++)
            x3D[k] = vf[k] * a + 0.0f;
    } else if (bStereo1 && cosParallaxStereo1 < cosParallaxStereo2) {
        /* KeyFrame::UnprojectStereo (KeyFrame.cc:798-814): mvKeys, not mvKeysUn */
        const float z = k1->depth[idx1];
        if (!(z > 0))
            return ORC_TRI_PARALLAX; /* the reference would use an empty Mat */
        const orc_keypoint *kr = k1->kps_raw ? &k1->kps_raw[idx1] : kp1;
        const float xc[3] = {(kr->x - c1->cx) * z * c1->invfx, (kr->y - c1->cy) * z * c1->invfy, z};
        orc_gemm3(T1, 1, xc, 1.0f, Ow1, x3D);
    } else if (bStereo2 && cosParallaxStereo2 < cosParallaxStereo1) {
        const float z = k2->depth[idx2];
        if (!(z > 0))
            return ORC_TRI_PARALLAX;
        const orc_keypoint *kr = k2->kps_raw ? &k2->kps_raw[idx2] : kp2;
        const float xc[3] = {(kr->x - c2->cx) * z * c2->invfx, (kr->y - c2->cy) * z * c2->invfy, z};
        orc_gemm3(T2, 1, xc, 1.0f, Ow2, x3D);
    } else {
        return ORC_TRI_PARALLAX; /* no stereo and very low parallax */
    }
    /* in front of both cameras (Mat::dot in double + the float translation) */
    const float z1 = (float)(orc_dot3f(&T1[8], x3D) + (double)T1[11]);
    if (z1 <= 0)
        return ORC_TRI_Z1;
    const float z2 = (float)(orc_dot3f(&T2[8], x3D) + (double)T2[11]);
    if (z2 <= 0)
        return ORC_TRI_Z2;
    /* reprojection error in the first keyframe */
    const float sigmaSquare1 = sigma2[kp1->octave];
    const float x1 = (float)(orc_dot3f(&T1[0], x3D) + (double)T1[3]);
    const float y1 = (float)(orc_dot3f(&T1[4], x3D) + (double)T1[7]);
    const float invz1 = (float)(1.0 / (double)z1);
    {
        const float u1 = c1->fx * x1 * invz1 + c1->cx;
        const float v1 = c1->fy * y1 * invz1 + c1->cy;
        const float errX1 = u1 - kp1->x, errY1 = v1 - kp1->y;
        if (!bStereo1) {
            if ((double)(errX1 * errX1 + errY1 * errY1) > 5.991 * (double)sigmaSquare1)
                return ORC_TRI_REPROJ1;
        } else {
            const float u1_r = u1 - c1->mbf * invz1;
            const float errX1_r = u1_r - kp1_ur;
            if ((double)(errX1 * errX1 + errY1 * errY1 + errX1_r * errX1_r) > 7.8 * (double)sigmaSquare1)
                return ORC_TRI_REPROJ1;
        }
    }
    /* ... and in the second (its stereo term uses the CURRENT keyframe's mbf, :528) */
    const float sigmaSquare2 = sigma2[kp2->octave];
    const float x2 = (float)(orc_dot3f(&T2[0], x3D) + (double)T2[3]);
    const float y2 = (float)(orc_dot3f(&T2[4], x3D) + (double)T2[7]);
    const float invz2 = (float)(1.0 / (double)z2);
    {
        const float u2 = c2->fx * x2 * invz2 + c2->cx;
        const float v2 = c2->fy * y2 * invz2 + c2->cy;
        const float errX2 = u2 - kp2->x, errY2 = v2 - kp2->y;
        if (!bStereo2) {
            if ((double)(errX2 * errX2 + errY2 * errY2) > 5.991 * (double)sigmaSquare2)
                return ORC_TRI_REPROJ2;
        } else {
            const float u2_r = u2 - c1->mbf * invz2;
            const float errX2_r = u2_r - kp2_ur;
            if ((double)(errX2 * errX2 + errY2 * errY2 + errX2_r * errX2_r) > 7.8 * (double)sigmaSquare2)
                return ORC_TRI_REPROJ2;
        }
    }
    /* scale consistency */
    const float n1[3] = {x3D[0] - Ow1[0], x3D[1] - Ow1[1], x3D[2] - Ow1[2]};
    const float n2[3] = {x3D[0] - Ow2[0], x3D[1] - Ow2[1], x3D[2] - Ow2[2]};
    const float dist1 = (float)sqrt(orc_dot3f(n1, n1)), dist2 = (float)sqrt(orc_dot3f(n2, n2));
    if (dist1 == 0 || dist2 == 0)
        return ORC_TRI_DIST0;
    const float ratioDist = dist2 / dist1;
    const float ratioOctave = scale_factors[kp1->octave] / scale_factors[kp2->octave];
    if (ratioDist * ratioFactor < ratioOctave || ratioDist > ratioOctave * ratioFactor)
        return ORC_TRI_SCALE;
    X[0] = x3D[0];
    X[1] = x3D[1];
    X[2] = x3D[2];
    return ORC_TRI_NEW;
}

int orc_triangulate(const orc_kf_tri *k1, const orc_kf_tri *k2, const orc_kf_cam *c1,
                    const orc_kf_cam *c2, const int32_t *matches12, const float *scale_factors,
                    const float *sigma2, float scale_factor, float *x3d, int8_t *status)
{
    const float *T1 = c1->Tcw, *T2 = c2->Tcw;
    float Ow1[3], Ow2[3];
    orc_kf_center(T1, Ow1);
    orc_kf_center(T2, Ow2);
    const float ratioFactor = 1.5f * scale_factor;
    int nnew = 0;
    for (int i = 0; i < k1->n; i++) {
        float *X = x3d + 3 * (size_t)i;
        X[0] = X[1] = X[2] = 0.0f;
        const int idx2 = matches12[i];
        if (idx2 < 0) {
            status[i] = ORC_TRI_NONE;
            continue;
        }
        status[i] = orc_triangulate_one(k1, k2, c1, c2, i, idx2, Ow1, Ow2, scale_factors,
                                        sigma2, ratioFactor, X);
        nnew += status[i] == ORC_TRI_NEW;
    }
    return nnew;
}

/* orc_atan2f against the host libm's atan2f over n pseudo-random (y, x) pairs (a xorshift
 * stream of float bit patterns biased to the depth / baseline range, plus the full float range
 * every 4th pair): the number of bit mismatches */
long orc_atan2f_check(uint32_t seed, long n)
{
    long bad = 0;
    uint32_t s = seed ? seed : 0x9e3779b9u;
    for (long i = 0; i < n; i++) {
        uint32_t w[2];
        for (int k = 0; k < 2; k++) {
            s ^= s << 13;
            s ^= s >> 17;
            s ^= s << 5;
            w[k] = s;
        }
        if (i & 3) /* |v| in [2^-8, 2^8), either sign */
            for (int k = 0; k < 2; k++)
                w[k] = (w[k] & 0x807fffffu) | ((119u + (w[k] >> 23) % 16u) << 23);
        float y, x;
        memcpy(&y, &w[0], 4);
        memcpy(&x, &w[1], 4);
        const float a = atan2f(y, x), b = orc_atan2f(y, x);
        bad += memcmp(&a, &b, 4) != 0 && !(a != a && b != b);
    }
    return bad;
}
