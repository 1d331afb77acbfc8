/*
 * oracle/pose_oracle.c -- TEST INFRASTRUCTURE ONLY (see orb_oracle.h).
 *
 * Double-precision restatement of Optimizer::PoseOptimization (src/Optimizer.cc:356-631):
 * one VertexSE3Expmap, unary EdgeSE3ProjectXYZOnlyPose / EdgeStereoSE3ProjectXYZOnlyPose
 * (types_six_dof_expmap.h:147-203, .cpp:266-364), Huber kernels (robust_kernel_impl.cpp:
 * 78-91), four rounds of optimize(10) with outlier re-classification, and g2o's
 * Levenberg-Marquardt step control (core/optimization_algorithm_levenberg.cpp:61-185) over
 * BlockSolver_6_3 + LinearSolverDense (Eigen LDLT, solvers/linear_solver_dense.h:64-110).
 *
 * Fixed-order pins (Eigen is not in the image; its vectorised reductions cannot be
 * reproduced, so these define the arithmetic the HIP kernel matches bit for bit -- parity
 * with the reference binary itself is unpinned):
 *   - sums over edges (activeRobustChi2, H, b): edge e goes to partial t = e mod 256 in
 *     increasing e; partials of 64 consecutive t are combined by the butterfly tree
 *     (pairs t, t^32, then t^16, ...), the four results as (w0 + w1) + (w2 + w3);
 *   - per-edge H = J^T (rho' Omega) J and b = -rho' J^T Omega e in BA's order
 *     (ba_oracle.c): H_rc = sum_k (J_kr * w) * J_kc, lower triangle used;
 *   - LDLT: Eigen's algorithm (largest remaining diagonal as pivot, first index on ties,
 *     lower triangle, zero pivots left unscaled, D^-1 skipped below DBL_MIN) with
 *     sequential inner products; solves forward / diagonal / backward in index order;
 *   - SE3Quat::exp uses a pinned sin/cos (orb_oracle.c pinned_sincos) and theta^3 as
 *     theta*theta*theta; LM's pow(2 rho - 1, 3) (optimization_algorithm_levenberg.cpp:135,
 *     libm pow under C++11) as the rounded exact cube orc_lm_cube;
 *   - Quaterniond(R) is Eigen's matrix-to-quaternion (trace branch, else largest diagonal).
 */
#include "orb_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>

/* g2o's pow(2 rho - 1, 3) (optimization_algorithm_levenberg.cpp:135): glibc's pow is
 * correctly rounded on all but astronomically rare inputs, and t*t*t is not (two roundings,
 * up to ~1 ulp off), so the cube is formed exactly as a double-double and rounded once:
 * t^2 = h + l (fma), h t = ph + pl (fma), t^3 = ph + (pl + l t).  The kernel
 * (pose_kernels.hip) evaluates the same expression; tests/test_oracle_kats.py checks it
 * against the host libm's pow(t, 3.0). */
double orc_lm_cube(double t)
{
    const double h = t * t;
    const double l = fma(t, t, -h);
    const double ph = h * t;
    const double pl = fma(h, t, -ph);
    return ph + (pl + l * t);
}
#include <string.h>

void orc_pinned_sincos_d(double x, double *s, double *c);

/* ---- SE3Quat (q = x, y, z, w) ---- */
static void q_rotate(const double q[4], const double v[3], double out[3])
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

/* Eigen Quaternion product a * b */
static void q_mul(const double a[4], const double b[4], double o[4])
{
    o[3] = a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2];
    o[0] = a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1];
    o[1] = a[3] * b[1] + a[1] * b[3] + a[2] * b[0] - a[0] * b[2];
    o[2] = a[3] * b[2] + a[2] * b[3] + a[0] * b[1] - a[1] * b[0];
}

/* SE3Quat::normalizeRotation (se3quat.h:280-285) */
static void q_normalize(double q[4])
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

/* Eigen quaternionbase_assign_impl<Matrix3>: rotation matrix -> quaternion */
static void q_from_rot(const double R[3][3], double q[4])
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
        if (R[1][1] > R[0][0])
            i = 1;
        if (R[2][2] > R[i][i])
            i = 2;
        const int j = (i + 1) % 3, k = (j + 1) % 3;
        double s = sqrt(R[i][i] - R[j][j] - R[k][k] + 1.0);
        q[i] = 0.5 * s;
        s = 0.5 / s;
        q[3] = (R[k][j] - R[j][k]) * s;
        q[j] = (R[j][i] + R[i][j]) * s;
        q[k] = (R[k][i] + R[i][k]) * s;
    }
}

/* VertexSE3Expmap::oplusImpl: estimate = SE3Quat::exp(update) * estimate (se3quat.h:223-257) */
void orc_se3_oplus(double q[4], double t[3], const double upd[6])
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
        orc_pinned_sincos_d(theta, &s, &c);
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
    for (int i = 0; i < 3; i++)
        dt[i] = V[i][0] * u[0] + V[i][1] * u[1] + V[i][2] * u[2];
    q_normalize(dq); /* SE3Quat(Quaterniond(R), V*upsilon) */
    /* exp * estimate: t = dt + dq * t; q = dq * q; normalizeRotation */
    double rt[3], nq[4];
    q_rotate(dq, t, rt);
    for (int i = 0; i < 3; i++)
        t[i] = dt[i] + rt[i];
    q_mul(dq, q, nq);
    q_normalize(nq);
    memcpy(q, nq, sizeof(nq));
}

/* ---- the unary edges ---- */
/* error, chi2 at pose (q, t); returns D */
static int pedge_error(const double q[4], const double t[3], const orc_pose_edge *e,
                       const orc_pose_cam *cam, double err[3], double xc[3])
{
    const double X[3] = {e->xw[0], e->xw[1], e->xw[2]};
    q_rotate(q, X, xc);
    xc[0] += t[0];
    xc[1] += t[1];
    xc[2] += t[2];
    const double fx = cam->fx, fy = cam->fy, cx = cam->cx, cy = cam->cy;
    if (!e->stereo) {
        /* EdgeSE3ProjectXYZOnlyPose::cam_project: project2d, then * f + c */
        const double px = xc[0] / xc[2], py = xc[1] / xc[2];
        err[0] = (double)e->obs[0] - (px * fx + cx);
        err[1] = (double)e->obs[1] - (py * fy + cy);
        err[2] = 0;
        return 2;
    }
    /* EdgeStereoSE3ProjectXYZOnlyPose::cam_project (.cpp:305-313): float invz */
    const float invz = (float)(1.0f / xc[2]);
    const double u = xc[0] * invz * fx + cx;
    const double v = xc[1] * invz * fy + cy;
    err[0] = (double)e->obs[0] - u;
    err[1] = (double)e->obs[1] - v;
    err[2] = (double)e->obs[2] - (u - (double)cam->bf * invz);
    return 3;
}

static double pedge_chi2(const double err[3], int D, double info)
{
    double chi2 = 0;
    for (int k = 0; k < D; k++)
        chi2 += err[k] * (info * err[k]);
    return chi2;
}

/* robustify's rho[0] / rho[1] (dsqr is a float member) */
static double huber_rho0(double chi2, double delta, double *rho1)
{
    const float dsqr = (float)(delta * delta);
    if (chi2 <= dsqr) {
        *rho1 = 1.0;
        return chi2;
    }
    const double sq = sqrt(chi2);
    *rho1 = delta / sq;
    return 2 * sq * delta - dsqr;
}

static void pedge_jac(const double xc[3], const orc_pose_edge *e, const orc_pose_cam *cam,
                      double J[3][6])
{
    const double x = xc[0], y = xc[1];
    const double invz = 1.0 / xc[2], invz_2 = invz * invz;
    const double fx = cam->fx, fy = cam->fy, bf = cam->bf;
    J[0][0] = x * y * invz_2 * fx;
    J[0][1] = -(1 + (x * x * invz_2)) * fx;
    J[0][2] = y * invz * fx;
    J[0][3] = -invz * fx;
    J[0][4] = 0;
    J[0][5] = x * invz_2 * fx;
    J[1][0] = (1 + y * y * invz_2) * fy;
    J[1][1] = -x * y * invz_2 * fy;
    J[1][2] = -x * invz * fy;
    J[1][3] = 0;
    J[1][4] = -invz * fy;
    J[1][5] = y * invz_2 * fy;
    if (e->stereo) {
        J[2][0] = J[0][0] - bf * y * invz_2;
        J[2][1] = J[0][1] + bf * x * invz_2;
        J[2][2] = J[0][2];
        J[2][3] = J[0][3];
        J[2][4] = 0;
        J[2][5] = J[0][5] - bf * invz_2;
    } else {
        memset(J[2], 0, sizeof(J[2]));
    }
}

/* the pinned 256-partial / butterfly reduction of v[e] over edges */
#define PO_T 256
static void po_reduce(const double *part, int nv, double *out)
{
    /* part[t * nv + j], t < 256 */
    double w[4][64];
    for (int j = 0; j < nv; j++) {
        for (int wv = 0; wv < 4; wv++) {
            for (int l = 0; l < 64; l++)
                w[wv][l] = part[(wv * 64 + l) * nv + j];
            for (int o = 32; o > 0; o >>= 1)
                for (int l = 0; l < o; l++)
                    w[wv][l] = w[wv][l] + w[wv][l + o];
        }
        out[j] = (w[0][0] + w[1][0]) + (w[2][0] + w[3][0]);
    }
}

/* one pass over the active edges at (q, t): robust chi2 and, when want_sys, H (lower
 * triangle, 21 entries row-major r >= c) and b */
#define PO_NV 28 /* chi2 + 21 H + 6 b */
int orc_pose_passes; /* edge passes of the last orc_pose_optimization (diagnostics) */
static double po_pass(const double q[4], const double t[3], const orc_pose_edge *edges, int n,
                      const uint8_t *active, int robust, const orc_pose_cam *cam, double H[6][6],
                      double b[6], double *part)
{
    memset(part, 0, sizeof(double) * PO_T * PO_NV);
    orc_pose_passes++;
    for (int e = 0; e < n; e++) {
        if (!active[e])
            continue;
        double *p = part + (e % PO_T) * PO_NV;
        const orc_pose_edge *E = &edges[e];
        double err[3], xc[3];
        const int D = pedge_error(q, t, E, cam, err, xc);
        const double info = E->inv_sigma2;
        const double chi2 = pedge_chi2(err, D, info);
        /* deltaMono / deltaStereo = (float)sqrt(5.991) / (float)sqrt(7.815) (:399-400) */
        const double delta = E->stereo ? (double)(float)sqrt(7.815) : (double)(float)sqrt(5.991);
        double rho1 = 1.0, rho0 = chi2;
        if (robust)
            rho0 = huber_rho0(chi2, delta, &rho1);
        p[0] += rho0;
        double J[3][6];
        pedge_jac(xc, E, cam, J);
        const double w = rho1 * info;
        double wr[3];
        for (int k = 0; k < D; k++)
            wr[k] = -info * err[k] * rho1;
        int hi = 1;
        for (int r = 0; r < 6; r++)
            for (int c = 0; c <= r; c++) {
                double a2 = 0;
                for (int k = 0; k < D; k++)
                    a2 += J[k][r] * w * J[k][c];
                p[hi++] += a2;
            }
        for (int r = 0; r < 6; r++) {
            double acc = 0;
            for (int k = 0; k < D; k++)
                acc += J[k][r] * wr[k];
            p[22 + r] += acc;
        }
    }
    double tot[PO_NV];
    po_reduce(part, PO_NV, tot);
    int hi = 1;
    for (int r = 0; r < 6; r++)
        for (int c = 0; c <= r; c++) {
            H[r][c] = tot[hi];
            H[c][r] = tot[hi];
            hi++;
        }
    for (int r = 0; r < 6; r++)
        b[r] = tot[22 + r];
    return tot[0];
}

/* Eigen LDLT (lower) + solve; returns isPositive() */
int orc_ldlt_solve6(const double Hin[6][6], const double b[6], double x[6])
{
    double m[6][6];
    memcpy(m, Hin, sizeof(m));
    int tr[6];
    int sign = 0; /* 0 zero, 1 positive semidef, 2 negative semidef, 3 indefinite */
    double temp[6];
    for (int k = 0; k < 6; k++) {
        int big = k;
        double bv = fabs(m[k][k]);
        for (int i = k + 1; i < 6; i++)
            if (fabs(m[i][i]) > bv) {
                bv = fabs(m[i][i]);
                big = i;
            }
        tr[k] = big;
        if (k != big) {
            for (int j = 0; j < k; j++) {
                const double s = m[k][j];
                m[k][j] = m[big][j];
                m[big][j] = s;
            }
            for (int i = big + 1; i < 6; i++) {
                const double s = m[i][k];
                m[i][k] = m[i][big];
                m[i][big] = s;
            }
            {
                const double s = m[k][k];
                m[k][k] = m[big][big];
                m[big][big] = s;
            }
            for (int i = k + 1; i < big; i++) {
                const double s = m[i][k];
                m[i][k] = m[big][i];
                m[big][i] = s;
            }
        }
        const int rs = 6 - k - 1;
        if (k > 0) {
            for (int j = 0; j < k; j++)
                temp[j] = m[j][j] * m[k][j];
            double dot = 0;
            for (int j = 0; j < k; j++)
                dot += m[k][j] * temp[j];
            m[k][k] -= dot;
            for (int i = k + 1; i < 6; i++) {
                double s = 0;
                for (int j = 0; j < k; j++)
                    s += m[i][j] * temp[j];
                m[i][k] -= s;
            }
        }
        const double akk = m[k][k];
        const int valid = fabs(akk) > 0.0;
        if (k == 0 && !valid) {
            sign = 0;
            for (int j = 0; j < 6; j++)
                tr[j] = j;
            for (int j = k; j < 6; j++)
                tr[j] = j;
            break;
        }
        if (rs > 0 && valid)
            for (int i = k + 1; i < 6; i++)
                m[i][k] /= akk;
        if (sign == 0 || sign == 1) {
            if (akk > 0)
                sign = 1;
            else if (akk < 0)
                sign = sign == 0 ? 2 : 3;
        } else if (sign == 2 && akk > 0) {
            sign = 3;
        }
    }
    if (!(sign == 1 || sign == 0))
        return 0;
    double d[6];
    for (int i = 0; i < 6; i++)
        d[i] = b[i];
    for (int k = 0; k < 6; k++) { /* P b */
        const double s = d[k];
        d[k] = d[tr[k]];
        d[tr[k]] = s;
    }
    for (int i = 0; i < 6; i++) { /* L^-1 */
        double s = 0;
        for (int j = 0; j < i; j++)
            s += m[i][j] * d[j];
        d[i] -= s;
    }
    for (int i = 0; i < 6; i++) /* D^-1 */
        d[i] = fabs(m[i][i]) > DBL_MIN ? d[i] / m[i][i] : 0.0;
    for (int i = 5; i >= 0; i--) { /* L^-T */
        double s = 0;
        for (int j = i + 1; j < 6; j++)
            s += m[j][i] * d[j];
        d[i] -= s;
    }
    for (int k = 5; k >= 0; k--) { /* P^-1 */
        const double s = d[k];
        d[k] = d[tr[k]];
        d[tr[k]] = s;
    }
    memcpy(x, d, sizeof(d));
    return 1;
}

/* SparseOptimizer::optimize(iterations) with OptimizationAlgorithmLevenberg on the single
 * pose vertex.  q/t: estimate (in/out).  last_q/last_t: where computeActiveErrors last
 * ran (the per-edge chi2() the caller reads afterwards).  Returns iterations run. */
static int po_optimize(double q[4], double t[3], const orc_pose_edge *edges, int n,
                       const uint8_t *active, int robust, const orc_pose_cam *cam, int iterations,
                       double last_q[4], double last_t[3], double *part)
{
    double H[6][6], b[6], x[6] = {0, 0, 0, 0, 0, 0};
    double lambda = 0, ni = 2;
    int nBad = 0;
    int it;
    for (it = 0; it < iterations; it++) {
        /* computeActiveErrors + buildSystem at the current estimate */
        double currentChi = po_pass(q, t, edges, n, active, robust, cam, H, b, part);
        memcpy(last_q, q, sizeof(double) * 4);
        memcpy(last_t, t, sizeof(double) * 3);
        const double iniChi = currentChi;
        if (it == 0) {
            double maxd = 0;
            for (int j = 0; j < 6; j++)
                maxd = fmax(fabs(H[j][j]), maxd);
            lambda = 1e-5 * maxd;
            ni = 2;
            nBad = 0;
        }
        double rho = 0;
        int qmax = 0;
        do {
            const double sq[4] = {q[0], q[1], q[2], q[3]}, st[3] = {t[0], t[1], t[2]};
            double Hd[6][6];
            memcpy(Hd, H, sizeof(Hd));
            for (int j = 0; j < 6; j++)
                Hd[j][j] += lambda;
            const int ok2 = orc_ldlt_solve6(Hd, b, x);
            orc_se3_oplus(q, t, x);
            double Hn[6][6], bn[6];  /* computeActiveErrors at the trial (the system is unused) */
            double tempChi = po_pass(q, t, edges, n, active, robust, cam, Hn, bn, part);
            memcpy(last_q, q, sizeof(double) * 4);
            memcpy(last_t, t, sizeof(double) * 3);
            if (!ok2)
                tempChi = DBL_MAX;
            rho = currentChi - tempChi;
            double scale = 0;
            for (int j = 0; j < 6; j++)
                scale += x[j] * (lambda * x[j] + b[j]);
            scale += 1e-3;
            rho /= scale;
            if (rho > 0 && isfinite(tempChi)) {
                double alpha = 1. - orc_lm_cube(2 * rho - 1);
                alpha = fmin(alpha, 2. / 3.);
                const double sf = fmax(1. / 3., alpha);
                lambda *= sf;
                ni = 2;
                currentChi = tempChi;
            } else {
                lambda *= ni;
                ni *= 2;
                memcpy(q, sq, sizeof(sq));
                memcpy(t, st, sizeof(st));
            }
            qmax++;
        } while (rho < 0 && qmax < 10);
        if (qmax == 10 || rho == 0)
            return it + 1; /* Terminate */
        if ((iniChi - currentChi) * 1e3 < iniChi)
            nBad++;
        else
            nBad = 0;
        if (nBad >= 3)
            return it + 1;
    }
    return it;
}

/* Converter::toSE3Quat (float cv::Mat -> SE3Quat(Matrix3d R, Vector3d t)) */
void orc_se3_from_tcw(const float Tcw[12], double q[4], double t[3])
{
    double R[3][3];
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++)
            R[i][j] = Tcw[4 * i + j];
        t[i] = Tcw[4 * i + 3];
    }
    q_from_rot(R, q);
    q_normalize(q);
}

/* Converter::toCvMat(SE3Quat): to_homogeneous_matrix, each element cast to float */
void orc_se3_to_tcw(const double q[4], const double t[3], float Tcw[12])
{
    const double tx = 2 * q[0], ty = 2 * q[1], tz = 2 * q[2];
    const double twx = tx * q[3], twy = ty * q[3], twz = tz * q[3];
    const double txx = tx * q[0], txy = ty * q[0], txz = tz * q[0];
    const double tyy = ty * q[1], tyz = tz * q[1], tzz = tz * q[2];
    const double R[3][3] = {{1 - (tyy + tzz), txy - twz, txz + twy},
                            {txy + twz, 1 - (txx + tzz), tyz - twx},
                            {txz - twy, tyz + twx, 1 - (txx + tyy)}};
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++)
            Tcw[4 * i + j] = (float)R[i][j];
        Tcw[4 * i + 3] = (float)t[i];
    }
}

int orc_pose_optimization(const orc_pose_edge *edges, int n, const orc_pose_cam *cam,
                          const float Tcw_in[12], double q_out[4], double t_out[3],
                          float Tcw_out[12], uint8_t *outlier)
{
    double q0[4], t0[3];
    orc_pose_passes = 0;
    orc_se3_from_tcw(Tcw_in, q0, t0);
    for (int i = 0; i < n; i++)
        outlier[i] = 0;
    if (n < 3) { /* Optimizer.cc:478-479: pose left as is */
        memcpy(q_out, q0, sizeof(q0));
        memcpy(t_out, t0, sizeof(t0));
        memcpy(Tcw_out, Tcw_in, sizeof(float) * 12);
        return 0;
    }
    double *part = (double *)malloc(sizeof(double) * PO_T * PO_NV);
    uint8_t *act = (uint8_t *)malloc((size_t)n);
    double q[4], t[3], lq[4] = {0, 0, 0, 1}, lt[3] = {0, 0, 0};
    const float chi2Mono = 5.991f, chi2Stereo = 7.815f;
    int nBad = 0, robust = 1;
    for (int it = 0; it < 4; it++) {
        memcpy(q, q0, sizeof(q));  /* vSE3->setEstimate(toSE3Quat(pFrame->mTcw)) */
        memcpy(t, t0, sizeof(t));
        int nact = 0;
        for (int i = 0; i < n; i++) {
            act[i] = !outlier[i];  /* initializeOptimization(0): level-0 edges */
            nact += act[i];
        }
        if (nact > 0)
            po_optimize(q, t, edges, n, act, robust, cam, 10, lq, lt, part);
        nBad = 0;
        for (int i = 0; i < n; i++) {
            const orc_pose_edge *E = &edges[i];
            double err[3], xc[3];
            /* active edges keep the error of the last computeActiveErrors; outliers get
             * computeError() at the current estimate (:531-535) */
            const int D = act[i] ? pedge_error(lq, lt, E, cam, err, xc)
                                 : pedge_error(q, t, E, cam, err, xc);
            const float chi2 = (float)pedge_chi2(err, D, E->inv_sigma2);
            if (chi2 > (E->stereo ? chi2Stereo : chi2Mono)) {
                outlier[i] = 1;
                nBad++;
            } else {
                outlier[i] = 0;
            }
        }
        if (it == 2)
            robust = 0;  /* e->setRobustKernel(0) */
        if (n < 10)      /* optimizer.edges().size() < 10 */
            break;
    }
    memcpy(q_out, q, sizeof(q));
    memcpy(t_out, t, sizeof(t));
    orc_se3_to_tcw(q, t, Tcw_out);
    free(part);
    free(act);
    return n - nBad;
}

/* The batched-sequence mode's per-frame pose (the "trajectory stub" of SURVEY.md 8e;
 * liborbg's orbg_match_pose_batch_device): Optimizer::PoseOptimization (Optimizer.cc:356-631)
 * of frame 2 with SearchForInitialization's vnMatches12 (m12[i] = j) as its map points.  F1
 * keypoint i matched to F2 keypoint j gives the mono edge obs = (x2_j, y2_j), Xw = F1 keypoint
 * i back-projected at `depth` in F1's camera ((x1 - cx) * z / fx, (y1 - cy) * z / fy, z, in
 * float), Omega = inv_sigma2[octave of j]; edges in F2 index order (PoseOptimization's loop
 * over pFrame's keypoints, Optimizer.cc:381); initial pose identity (F1 = world).  Returns
 * the inlier count; q / t = F2's pose relative to F1. */
int orc_match_pose(const orc_keypoint *k1, int n1, const orc_keypoint *k2, int n2,
                   const int32_t *m12, const orc_pose_cam *cam, float depth,
                   const float *inv_sigma2, double q[4], double t[3])
{
    int *inv = (int *)malloc(sizeof(int) * (size_t)(n2 > 0 ? n2 : 1));
    for (int j = 0; j < n2; j++)
        inv[j] = -1;
    for (int i = 0; i < n1; i++)
        if (m12[i] >= 0 && m12[i] < n2)
            inv[m12[i]] = i;
    orc_pose_edge *e = (orc_pose_edge *)malloc(sizeof(orc_pose_edge) * (size_t)(n2 > 0 ? n2 : 1));
    int n = 0;
    for (int j = 0; j < n2; j++) {
        const int i = inv[j];
        if (i < 0)
            continue;
        orc_pose_edge *E = &e[n++];
        E->obs[0] = k2[j].x;
        E->obs[1] = k2[j].y;
        E->obs[2] = -1.f;
        E->xw[0] = (k1[i].x - cam->cx) * depth / cam->fx;
        E->xw[1] = (k1[i].y - cam->cy) * depth / cam->fy;
        E->xw[2] = depth;
        E->inv_sigma2 = inv_sigma2[k2[j].octave];
        E->stereo = 0;
    }
    const float T0[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
    float To[12];
    uint8_t *out = (uint8_t *)malloc((size_t)(n > 0 ? n : 1));
    const int ninl = orc_pose_optimization(e, n, cam, T0, q, t, To, out);
    free(out);
    free(e);
    free(inv);
    return ninl;
}
