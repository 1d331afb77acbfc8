// se3_device.h -- g2o's SE3Quat arithmetic on the device (q = x, y, z, w; Eigen's formulas,
// see oracle/pose_oracle.c): the LM's cube, quaternion rotate / product / normalise, the
// quaternion of a rotation matrix, and VertexSE3Expmap::oplusImpl.  Shared by
// PoseOptimization (pose_kernels.hip) and the LocalBundleAdjustment update (lm_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "orbg_device.h"

#pragma clang fp contract(off)

namespace orbg {

// ---- SE3Quat (q = x, y, z, w), Eigen's formulas (see oracle/pose_oracle.c) ----
// g2o's pow(2 rho - 1, 3) (optimization_algorithm_levenberg.cpp:135, libm pow): the exact
// cube as a double-double, rounded once (oracle/pose_oracle.c orc_lm_cube, same expression)
__device__ __forceinline__ double lm_cube(double t)
{
    const double h = t * t;
    const double l = __builtin_fma(t, t, -h);
    const double ph = h * t;
    const double pl = __builtin_fma(h, t, -ph);
    return ph + (pl + l * t);
}

__device__ __forceinline__ void q_rotate(const double q[4], const double v[3], double out[3])
{
    double uv[3] = {q[1] * v[2] - q[2] * v[1], q[2] * v[0] - q[0] * v[2],
                    q[0] * v[1] - q[1] * v[0]};
    uv[0] += uv[0];
    uv[1] += uv[1];
    uv[2] += uv[2];
    const double c[3] = {q[1] * uv[2] - q[2] * uv[1], q[2] * uv[0] - q[0] * uv[2],
                         q[0] * uv[1] - q[1] * uv[0]};
    out[0] = v[0] + q[3] * uv[0] + c[0];
    out[1] = v[1] + q[3] * uv[1] + c[1];
    out[2] = v[2] + q[3] * uv[2] + c[2];
}

__device__ __forceinline__ void q_mul(const double a[4], const double b[4], double o[4])
{
    o[3] = a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2];
    o[0] = a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1];
    o[1] = a[3] * b[1] + a[1] * b[3] + a[2] * b[0] - a[0] * b[2];
    o[2] = a[3] * b[2] + a[2] * b[3] + a[0] * b[1] - a[1] * b[0];
}

__device__ __forceinline__ void q_normalize(double q[4])
{
    if (q[3] < 0) {
        q[0] = -q[0];
        q[1] = -q[1];
        q[2] = -q[2];
        q[3] = -q[3];
    }
    const double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    q[0] /= n;
    q[1] /= n;
    q[2] /= n;
    q[3] /= n;
}

__device__ inline void q_from_rot(const double R[3][3], double q[4])
{
    const double t = R[0][0] + R[1][1] + R[2][2];
    if (t > 0) {
        double s = sqrt(t + 1.0);
        q[3] = 0.5 * s;
        s = 0.5 / s;
        q[0] = (R[2][1] - R[1][2]) * s;
        q[1] = (R[0][2] - R[2][0]) * s;
        q[2] = (R[1][0] - R[0][1]) * s;
    } else {
        int i = 0;
        if (R[1][1] > R[0][0]) i = 1;
        if (R[2][2] > R[i][i]) i = 2;
        const int j = (i + 1) % 3, k = (j + 1) % 3;
        double s = sqrt(R[i][i] - R[j][j] - R[k][k] + 1.0);
        q[i] = 0.5 * s;
        s = 0.5 / s;
        q[3] = (R[k][j] - R[j][k]) * s;
        q[j] = (R[j][i] + R[i][j]) * s;
        q[k] = (R[k][i] + R[i][k]) * s;
    }
}

// VertexSE3Expmap::oplusImpl: estimate = SE3Quat::exp(update) * estimate
__device__ inline void se3_oplus(double q[4], double t[3], const double upd[6])
{
    const double w[3] = {upd[0], upd[1], upd[2]}, u[3] = {upd[3], upd[4], upd[5]};
    const double theta = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    const double O[3][3] = {{0, -w[2], w[1]}, {w[2], 0, -w[0]}, {-w[1], w[0], 0}};
    double O2[3][3], R[3][3], V[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            O2[i][j] = O[i][0] * O[0][j] + O[i][1] * O[1][j] + O[i][2] * O[2][j];
    if (theta < 0.00001) {
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) {
                R[i][j] = ((i == j ? 1.0 : 0.0) + O[i][j]) + O2[i][j];
                V[i][j] = R[i][j];
            }
    } else {
        double s, c;
        pinned_sincos(theta, &s, &c);
        const double a = s / theta, b = (1 - c) / (theta * theta);
        const double cc = (theta - s) / (theta * theta * theta);
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) {
                const double I = i == j ? 1.0 : 0.0;
                R[i][j] = (I + a * O[i][j]) + b * O2[i][j];
                V[i][j] = (I + b * O[i][j]) + cc * O2[i][j];
            }
    }
    double dq[4], dt[3];
    q_from_rot(R, dq);
    for (int i = 0; i < 3; i++) dt[i] = V[i][0] * u[0] + V[i][1] * u[1] + V[i][2] * u[2];
    q_normalize(dq);
    double rt[3], nq[4];
    q_rotate(dq, t, rt);
    for (int i = 0; i < 3; i++) t[i] = dt[i] + rt[i];
    q_mul(dq, q, nq);
    q_normalize(nq);
    for (int i = 0; i < 4; i++) q[i] = nq[i];
}

}  // namespace orbg
