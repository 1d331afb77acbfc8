// frame_device.h -- cv::undistortPoints(src, dst, K, D, noArray(), K) for one point, shared by
// k_undistort (frame_kernels.hip) and the host-side Frame::ComputeImageBounds (orbg_api.hip)
// so both run the same expression tree.  OpenCV 3.4's cvUndistortPointsInternal
// (modules/imgproc/src/undistort.cpp) with the default criteria TermCriteria(COUNT, 5, 0.01):
// five fixed-point iterations in double, no EPS test; K, D converted from CV_32F to double;
// identity tilt (x0 = x), zero rational / thin-prism terms kept in the library's order;
// RR = K * I = K, so u = fx*x + 0*y + cx, v = 0*x + fy*y + cy, w = 1 / (0*x + 0*y + 1); the
// result rounded to float.  No FMA contraction (fp contract off here and -ffp-contract=off).
#pragma once

#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include "../../include/orbg.h"

namespace orbg {

__host__ __device__ inline void undistort_point(const orbg_camera &c, float uf, float vf,
                                                float *xo, float *yo)
{
    const double fx = c.fx, fy = c.fy, cx = c.cx, cy = c.cy;
    const double ifx = 1. / fx, ify = 1. / fy;
    const double k0 = c.k1, k1 = c.k2, k2 = c.p1, k3 = c.p2, k4 = c.k3;
    const double z = 0.0;  // k[5..11]: rational and thin-prism coefficients (absent)
    double x = uf, y = vf;
    x = (x - cx) * ifx;
    y = (y - cy) * ify;
    const double x0 = x, y0 = y;
    for (int j = 0; j < 5; j++) {
        const double r2 = x * x + y * y;
        const double icdist = (1 + ((z * r2 + z) * r2 + z) * r2) / (1 + ((k4 * r2 + k1) * r2 + k0) * r2);
        const double deltaX = 2 * k2 * x * y + k3 * (r2 + 2 * x * x) + z * r2 + z * r2 * r2;
        const double deltaY = k2 * (r2 + 2 * y * y) + 2 * k3 * x * y + z * r2 + z * r2 * r2;
        x = (x0 - deltaX) * icdist;
        y = (y0 - deltaY) * icdist;
    }
    const double xx = fx * x + 0.0 * y + cx;
    const double yy = 0.0 * x + fy * y + cy;
    const double ww = 1. / (0.0 * x + 0.0 * y + 1.0);
    *xo = (float)(xx * ww);
    *yo = (float)(yy * ww);
}

// Fuse(pKF, Scw, ...) / SearchByProjection(pKF, Scw, ...)'s decomposition (ORBmatcher.cc:
// 1143-1148, 362-366): scw = the double root of row 0's double dot product, rounded to float;
// Rcw | tcw = Scw * (float)(1 / scw), rounded once per element (Mat / double is convertTo
// with a float alpha and shift 0; built with -ffp-contract=off)
__host__ __device__ inline void sim3_decompose(const float *S, float *T)
{
    double d = 0.0;
    for (int k = 0; k < 3; k++) d += (double)S[k] * (double)S[k];
    const float scw = (float)sqrt(d);
    const float a = (float)(1.0 / (double)scw);
    for (int k = 0; k < 12; k++) T[k] = S[k] * a + 0.0f;
}

// MapPoint::PredictScale (MapPoint.cc:575-607): ceil(log(ratio) / mfLogScaleFactor) in double.
// Fast path: the float quotient (logf within ~1 ulp, then one division: a few float ulps of q,
// i.e. about 1e-5 absolute near |q| = 64, where the ulp is 3.8e-6) decides the ceiling whenever
// it is more than 1e-3 away from an integer -- the double quotient is then inside the same
// open interval; near an integer, or non-finite, the reference's double expression is
// evaluated.  Same result, a fraction of the FP64 issue (pinned on ratios up to |q| ~ 64 by
// tests/test_oracle_frame.py).
__host__ __device__ inline int predict_scale(float max_dist, float dist, float log_sf, int nlevels)
{
    const float ratio = max_dist / dist;
    const float qf = logf(ratio) / log_sf;
    const float fl = floorf(qf);
    int n;
    if (fabsf(qf) < 64.0f && qf - fl > 1e-3f && qf - fl < 0.999f)
        n = (int)fl + 1;
    else
        n = (int)ceil(log((double)ratio) / (double)log_sf);
    if (n < 0)
        n = 0;
    else if (n >= nlevels)
        n = nlevels - 1;
    return n;
}

}  // namespace orbg
