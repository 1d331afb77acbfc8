/*
 * oracle/frame_oracle.c -- TEST INFRASTRUCTURE ONLY (see orb_oracle.h).
 *
 * Plain-C restatement of the per-frame / per-MapPoint geometry around the matchers:
 *   Frame::UndistortKeyPoints ............ src/Frame.cc:542-572 (cv::undistortPoints pin below)
 *   Frame::ComputeImageBounds ............ src/Frame.cc:575-611
 *   Frame::isInFrustum ................... src/Frame.cc:342-409, MapPoint::PredictScale
 *                                          src/MapPoint.cc:575-590, Get{Min,Max}Distance-
 *                                          Invariance :520-530 (caller: Tracking::
 *                                          SearchLocalPoints, Tracking.cc:1676-1691)
 *   MapPoint::ComputeDistinctiveDescriptors src/MapPoint.cc:342-420
 *
 * OpenCV pins (OpenCV is not in the image; recalled from 3.4's modules/imgproc/src/
 * undistort.cpp, cvUndistortPointsInternal):
 *   - cv::undistortPoints(src, dst, K, D, noArray(), K) with the default criteria
 *     TermCriteria(COUNT, 5, 0.01): the distortion is inverted by exactly 5 fixed-point
 *     iterations in double (no EPS test, so no reprojection error is computed);
 *     K and D (CV_32F) are converted to double first, ifx = 1./fx, ify = 1./fy;
 *     the tilt matrices are the identity (k[12] = k[13] = 0): x0 = x exactly; the
 *     rational and thin-prism terms are zero but kept in the expressions in the library's
 *     order (a + b + 0*r2 + 0*r2*r2 rounds like a + b);
 *     RR = P * I = K, so u = fx*x + cx, v = fy*y + cy (0*y / 0*x terms add +0), w = 1;
 *     the result is rounded to float.  No FMA contraction (-ffp-contract=off; the library
 *     is built for the SSE baseline).
 *   - cv::gemm's small-matrix path for Rcw*P+tcw / -Rcw.t()*tcw (orc_gemm3, track_oracle.c).
 *   - cv::norm(PO) of a 3x1 float Mat: double sum of squares in order, sqrt in double,
 *     assigned to float; PO.dot(Pn): double sum of (double) products in order, divided by
 *     the float dist in double, assigned to float.
 *   - MapPoint::PredictScale's log(ratio) and Frame's mfLogScaleFactor = log(mfScaleFactor):
 *     unqualified log() of a float inside namespace ORB_SLAM2 with no `using namespace std`
 *     (Frame.cc:103, MapPoint.cc:583): the C library's double log; pinned as
 *     log((double)x) (ratio / mfLogScaleFactor in double, ceil).
 */
#include "orb_oracle.h"

#include <limits.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

/* one point of cvUndistortPointsInternal (P = K, R = I, COUNT 5) */
static void undistort_one(const orc_camera *c, float uf, float vf, float *xo, float *yo)
{
    const double fx = c->fx, fy = c->fy, cx = c->cx, cy = c->cy;
    const double ifx = 1. / fx, ify = 1. / fy;
    double k[14];
    memset(k, 0, sizeof(k));
    k[0] = c->k1;
    k[1] = c->k2;
    k[2] = c->p1;
    k[3] = c->p2;
    k[4] = c->k3;
    double x = uf, y = vf;
    x = (x - cx) * ifx;
    y = (y - cy) * ify;
    const double x0 = x, y0 = y;
    for (int j = 0; j < 5; j++) {
        const double r2 = x * x + y * y;
        const double icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) /
                              (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
        const double deltaX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x) + k[8] * r2 +
                              k[9] * r2 * r2;
        const double deltaY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y + k[10] * r2 +
                              k[11] * r2 * r2;
        x = (x0 - deltaX) * icdist;
        y = (y0 - deltaY) * icdist;
    }
    /* RR = K: xx = fx*x + 0*y + cx, yy = 0*x + fy*y + cy, ww = 1/(0*x + 0*y + 1) */
    const double xx = fx * x + 0.0 * y + cx;
    const double yy = 0.0 * x + fy * y + cy;
    const double ww = 1. / (0.0 * x + 0.0 * y + 1.0);
    *xo = (float)(xx * ww);
    *yo = (float)(yy * ww);
}

void orc_undistort_points(const orc_camera *cam, const float *xy, int n, float *out)
{
    for (int i = 0; i < n; i++)
        undistort_one(cam, xy[2 * i], xy[2 * i + 1], &out[2 * i], &out[2 * i + 1]);
}

void orc_undistort_keypoints(const orc_camera *cam, const orc_keypoint *kps, int n,
                             orc_keypoint *out)
{
    /* Frame.cc:544-548: k1 == 0 -> mvKeysUn = mvKeys (whatever the other coefficients) */
    for (int i = 0; i < n; i++) {
        out[i] = kps[i];
        if (cam->k1 != 0.0f)
            undistort_one(cam, kps[i].x, kps[i].y, &out[i].x, &out[i].y);
    }
}

void orc_image_bounds(const orc_camera *cam, int w, int h, orc_bounds *b)
{
    if (cam->k1 != 0.0f) {
        /* Frame.cc:579-600: the four corners (0,0), (cols,0), (0,rows), (cols,rows) */
        const float in[8] = {0.0f, 0.0f, (float)w, 0.0f, 0.0f, (float)h, (float)w, (float)h};
        float o[8];
        orc_undistort_points(cam, in, 4, o);
        b->min_x = o[4] < o[0] ? o[4] : o[0];  /* std::min(a, b) = b < a ? b : a */
        b->max_x = o[2] < o[6] ? o[6] : o[2];  /* std::max(a, b): a < b ? b : a */
        b->min_y = o[3] < o[1] ? o[3] : o[1];
        b->max_y = o[5] < o[7] ? o[7] : o[5];
    } else {
        b->min_x = 0.0f;
        b->max_x = (float)w;
        b->min_y = 0.0f;
        b->max_y = (float)h;
    }
}

float orc_log_scale_factor(float scale_factor) { return (float)log((double)scale_factor); }

int orc_is_in_frustum(const orc_frustum_cam *cam, const orc_map_point *mp,
                      float viewing_cos_limit, orc_map_proj *out)
{
    /* Frame.cc:350: mbTrackInView = false (the other mTrack* members keep their values);
     * Observations() > 0 passes through for SearchByProjection */
    out->flags = mp->flags & ORC_MP_HAS_OBS;
    if (!(mp->flags & ORC_MP_VALID))  /* SearchLocalPoints: bad, or seen this frame */
        return 0;
    const float P[3] = {mp->x, mp->y, mp->z};
    const float tcw[3] = {cam->Tcw[3], cam->Tcw[7], cam->Tcw[11]};
    float Pc[3];
    orc_gemm3(cam->Tcw, 0, P, 1.0f, tcw, Pc); /* mRcw*P+mtcw */
    const float PcX = Pc[0], PcY = Pc[1], PcZ = Pc[2];
    if (PcZ < 0.0f)
        return 0;
    const float invz = 1.0f / PcZ;
    const float u = cam->fx * PcX * invz + cam->cx;
    const float v = cam->fy * PcY * invz + cam->cy;
    if (u < cam->bounds.min_x || u > cam->bounds.max_x)
        return 0;
    if (v < cam->bounds.min_y || v > cam->bounds.max_y)
        return 0;
    const float maxDistance = 1.2f * mp->max_dist; /* GetMaxDistanceInvariance */
    const float minDistance = 0.8f * mp->min_dist; /* GetMinDistanceInvariance */
    /* mOw = -mRcw.t()*mtcw (Frame::UpdatePoseMatrices, Frame.cc:334) */
    float Ow[3];
    orc_gemm3(cam->Tcw, 1, tcw, -1.0f, NULL, Ow);
    const float PO[3] = {P[0] - Ow[0], P[1] - Ow[1], P[2] - Ow[2]};
    double s = 0.0;
    for (int i = 0; i < 3; i++)
        s += (double)PO[i] * (double)PO[i];
    const float dist = (float)sqrt(s);
    if (dist < minDistance || dist > maxDistance)
        return 0;
    const float Pn[3] = {mp->nx, mp->ny, mp->nz};
    double dot = 0.0;
    for (int i = 0; i < 3; i++)
        dot += (double)PO[i] * (double)Pn[i];
    const float viewCos = (float)(dot / (double)dist);
    if (viewCos < viewing_cos_limit)
        return 0;
    /* MapPoint::PredictScale(dist, this) */
    const float ratio = mp->max_dist / dist;
    int nScale = (int)ceil(log((double)ratio) / (double)cam->log_scale_factor);
    if (nScale < 0)
        nScale = 0;
    else if (nScale >= cam->nlevels)
        nScale = cam->nlevels - 1;
    out->flags |= ORC_MP_VALID;
    out->u = u;
    out->ur = u - cam->bf * invz;
    out->v = v;
    out->level = nScale;
    out->view_cos = viewCos;
    return 1;
}

int orc_distinctive_descriptor(const uint8_t *desc, int n)
{
    /* MapPoint.cc:386-419: all-pairs DescriptorDistance, the row with the least median
     * (vDists[0.5*(N-1)] of the sorted row, the first such row on ties) */
    if (n <= 0)
        return -1;
    int *D = (int *)malloc(sizeof(int) * (size_t)n * (size_t)n);
    for (int i = 0; i < n; i++) {
        D[(size_t)i * n + i] = 0;
        for (int j = i + 1; j < n; j++) {
            const int d = orc_descriptor_distance(desc + (size_t)i * 32, desc + (size_t)j * 32);
            D[(size_t)i * n + j] = d;
            D[(size_t)j * n + i] = d;
        }
    }
    int best_median = INT_MAX, best = 0;
    const size_t k = (size_t)(0.5 * (double)(n - 1));
    for (int i = 0; i < n; i++) {
        /* counting sort of the row (values 0..256) = std::sort */
        int cnt[257];
        memset(cnt, 0, sizeof(cnt));
        for (int j = 0; j < n; j++)
            cnt[D[(size_t)i * n + j]]++;
        size_t seen = 0;
        int median = 0;
        for (int v = 0; v <= 256; v++) {
            seen += (size_t)cnt[v];
            if (seen > k) {
                median = v;
                break;
            }
        }
        if (median < best_median) {
            best_median = median;
            best = i;
        }
    }
    free(D);
    return best;
}

int orc_is_in_frustum_n(const orc_frustum_cam *cam, const orc_map_point *mps, int n,
                        float viewing_cos_limit, orc_map_proj *out)
{
    int nvis = 0;
    for (int i = 0; i < n; i++)
        nvis += orc_is_in_frustum(cam, &mps[i], viewing_cos_limit, &out[i]);
    return nvis;
}

void orc_distinctive_descriptors_n(const uint8_t *pool, const int32_t *rows, const int32_t *off,
                                   int npoints, int32_t *best)
{
    uint8_t *buf = NULL;
    int bcap = 0;
    for (int p = 0; p < npoints; p++) {
        const int n = off[p + 1] - off[p];
        if (n > bcap) {
            free(buf);
            bcap = n;
            buf = (uint8_t *)malloc((size_t)bcap * 32);
        }
        for (int i = 0; i < n; i++)
            memcpy(buf + (size_t)i * 32, pool + (size_t)rows[off[p] + i] * 32, 32);
        best[p] = orc_distinctive_descriptor(buf, n);
    }
    free(buf);
}

/* Frame::ComputeStereoFromRGBD (Frame.cc:837-858) after Tracking::GrabImageRGBD's
 * imDepth.convertTo(CV_32F, mDepthMapFactor) (Tracking.cc:233-234): the depth of a pixel is
 * raw * factor in float (convertTo's float alpha, shift 0), or the float itself when the image
 * is CV_32F and |factor - 1| <= 1e-5; imDepth.at<float>(v, u) truncates the keypoint's
 * position.  u16: 1 = raw uint16 image, 0 = float. */
void orc_rgbd_stereo(const void *depth, int u16, float factor, int w, int h, size_t pitch,
                     const orc_keypoint *kps, const orc_keypoint *kps_un, int n, float mbf,
                     float *uright, float *depth_out)
{
    const int scale = u16 || fabsf(factor - 1.0f) > 1e-5;
    for (int i = 0; i < n; i++) {
        uright[i] = -1.0f;
        depth_out[i] = -1.0f;
        const int u = (int)kps[i].x, v = (int)kps[i].y;
        if (u < 0 || u >= w || v < 0 || v >= h)
            continue;
        const uint8_t *row = (const uint8_t *)depth + (size_t)v * pitch;
        const float raw = u16 ? (float)((const uint16_t *)row)[u] : ((const float *)row)[u];
        const float d = scale ? raw * factor : raw;
        if (d > 0) {
            depth_out[i] = d;
            uright[i] = kps_un[i].x - mbf / d;
        }
    }
}
