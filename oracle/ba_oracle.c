/*
 * oracle/ba_oracle.c -- TEST INFRASTRUCTURE ONLY (see orb_oracle.h).
 *
 * Double-precision restatement of the per-edge arithmetic g2o performs inside
 * Optimizer::LocalBundleAdjustment (src/Optimizer.cc:633-979):
 *   EdgeSE3ProjectXYZ::computeError / cam_project     types_six_dof_expmap.h:90-95, .cpp:141-147
 *   EdgeStereoSE3ProjectXYZ::computeError / cam_project  .h:122-127, .cpp:150-157 (float invz, float bf)
 *   linearizeOplus (mono, stereo)                     .cpp:103-139, 188-234
 *   SE3Quat::map (Eigen quaternion * vector)          se3quat.h:217-220
 *   chi2 / robustInformation                          core/base_edge.h:58-61, 96-102
 *   RobustKernelHuber::robustify (float dsqr)         core/robust_kernel_impl.cpp:65-91
 *   BaseBinaryEdge::constructQuadraticForm            core/base_binary_edge.hpp:55-120
 *   numeric linearizeOplus (central diff, 1e-9)       core/base_binary_edge.hpp:131-205
 *   SE3Quat::exp (oplus of VertexSE3Expmap)           se3quat.h:223-257, types_six_dof_expmap.h:73-76
 */
#include "orb_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

static void quat_rotate(const double q[4], const double v[3], double out[3])
{
    /* Eigen _transformVector: uv = 2 (q.vec x v); v + w uv + q.vec x uv */
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

static void quat_to_rot(const double q[4], double R[3][3])
{
    /* Eigen QuaternionBase::toRotationMatrix */
    const double tx = 2 * q[0], ty = 2 * q[1], tz = 2 * q[2];
    const double twx = tx * q[3], twy = ty * q[3], twz = tz * q[3];
    const double txx = tx * q[0], txy = ty * q[0], txz = tz * q[0];
    const double tyy = ty * q[1], tyz = tz * q[1], tzz = tz * q[2];
    R[0][0] = 1 - (tyy + tzz);
    R[0][1] = txy - twz;
    R[0][2] = txz + twy;
    R[1][0] = txy + twz;
    R[1][1] = 1 - (txx + tzz);
    R[1][2] = tyz - twx;
    R[2][0] = txz - twy;
    R[2][1] = tyz + twx;
    R[2][2] = 1 - (txx + tyy);
}

/* computeError with the pose given as (R, t) matrices (used by the numeric Jacobian) */
/* exact_invz: evaluate the stereo projection with a double 1/z.  The reference's
 * float invz (types_six_dof_expmap.cpp:151) makes the residual piecewise constant at
 * ~1e-7 relative, so a 1e-9 central difference of it is noise; the analytic stereo
 * Jacobian (:188-234) is the derivative of the double-precision model. */
static void edge_error_rt(const double R[3][3], const double t[3], const double X[3],
                          const orc_edge *e, double err[3], int exact_invz)
{
    double xc[3];
    for (int i = 0; i < 3; i++)
        xc[i] = R[i][0] * X[0] + R[i][1] * X[1] + R[i][2] * X[2] + t[i];
    if (!e->stereo) {
        err[0] = e->obs[0] - ((xc[0] / xc[2]) * e->fx + e->cx);
        err[1] = e->obs[1] - ((xc[1] / xc[2]) * e->fy + e->cy);
        err[2] = 0;
    } else if (exact_invz) {
        const double invz = 1.0 / xc[2];
        const double u = xc[0] * invz * e->fx + e->cx;
        const double v = xc[1] * invz * e->fy + e->cy;
        err[0] = e->obs[0] - u;
        err[1] = e->obs[1] - v;
        err[2] = e->obs[2] - (u - e->bf * invz);
    } else {
        const float invz = (float)(1.0f / xc[2]);
        const float bf = (float)e->bf;
        const double u = xc[0] * invz * e->fx + e->cx;
        const double v = xc[1] * invz * e->fy + e->cy;
        err[0] = e->obs[0] - u;
        err[1] = e->obs[1] - v;
        err[2] = e->obs[2] - (u - (double)(bf * invz));
    }
}

static void edge_error(const orc_pose *P, const double X[3], const orc_edge *e, double err[3],
                       double xc[3])
{
    quat_rotate(P->q, X, xc);
    xc[0] += P->t[0];
    xc[1] += P->t[1];
    xc[2] += P->t[2];
    if (!e->stereo) {
        /* project2d then *f + c */
        const double px = xc[0] / xc[2], py = xc[1] / xc[2];
        err[0] = e->obs[0] - (px * e->fx + e->cx);
        err[1] = e->obs[1] - (py * e->fy + e->cy);
        err[2] = 0;
    } else {
        const float invz = (float)(1.0f / xc[2]);
        const float bf = (float)e->bf; /* cam_project(const Vector3d&, const float &bf) */
        const double u = xc[0] * invz * e->fx + e->cx;
        const double v = xc[1] * invz * e->fy + e->cy;
        err[0] = e->obs[0] - u;
        err[1] = e->obs[1] - v;
        err[2] = e->obs[2] - (u - (double)(bf * invz));
    }
}

static void edge_jacobians(const orc_pose *P, const double xc[3], const orc_edge *e,
                           double jp[3][3], double jt[3][6])
{
    double R[3][3];
    quat_to_rot(P->q, R);
    const double x = xc[0], y = xc[1], z = xc[2], z_2 = z * z;
    const double fx = e->fx, fy = e->fy;
    memset(jp, 0, sizeof(double) * 9);
    memset(jt, 0, sizeof(double) * 18);
    if (!e->stereo) {
        const double tmp[2][3] = {{fx, 0, -x / z * fx}, {0, fy, -y / z * fy}};
        for (int r = 0; r < 2; r++)
            for (int c = 0; c < 3; c++) {
                double acc = 0;
                for (int k = 0; k < 3; k++)
                    acc += tmp[r][k] * R[k][c];
                jp[r][c] = -1. / z * acc;
            }
    } else {
        for (int c = 0; c < 3; c++) {
            jp[0][c] = -fx * R[0][c] / z + fx * x * R[2][c] / z_2;
            jp[1][c] = -fy * R[1][c] / z + fy * y * R[2][c] / z_2;
            jp[2][c] = jp[0][c] - e->bf * R[2][c] / z_2;
        }
    }
    jt[0][0] = x * y / z_2 * fx;
    jt[0][1] = -(1 + (x * x / z_2)) * fx;
    jt[0][2] = y / z * fx;
    jt[0][3] = -1. / z * fx;
    jt[0][4] = 0;
    jt[0][5] = x / z_2 * fx;
    jt[1][0] = (1 + y * y / z_2) * fy;
    jt[1][1] = -x * y / z_2 * fy;
    jt[1][2] = -x / z * fy;
    jt[1][3] = 0;
    jt[1][4] = -1. / z * fy;
    jt[1][5] = y / z_2 * fy;
    if (e->stereo) {
        jt[2][0] = jt[0][0] - e->bf * y / z_2;
        jt[2][1] = jt[0][1] + e->bf * x / z_2;
        jt[2][2] = jt[0][2];
        jt[2][3] = jt[0][3];
        jt[2][4] = 0;
        jt[2][5] = jt[0][5] - e->bf / z_2;
    }
}

void orc_ba_linearize(const orc_pose *poses, int npose, const double *points, int npoint,
                      const orc_edge *edges, int nedge, orc_edge_out *eout, double *hpose,
                      double *bpose, double *hpoint, double *bpoint)
{
    memset(hpose, 0, sizeof(double) * 36 * (size_t)npose);
    memset(bpose, 0, sizeof(double) * 6 * (size_t)npose);
    memset(hpoint, 0, sizeof(double) * 9 * (size_t)npoint);
    memset(bpoint, 0, sizeof(double) * 3 * (size_t)npoint);
    for (int i = 0; i < nedge; i++) {
        const orc_edge *e = &edges[i];
        orc_edge_out *o = &eout[i];
        memset(o, 0, sizeof(*o));
        if (!e->active)
            continue;
        const orc_pose *P = &poses[e->pose];
        const double *X = points + 3 * (size_t)e->point;
        double xc[3];
        edge_error(P, X, e, o->err, xc);
        edge_jacobians(P, xc, e, o->jp, o->jt);
        const int D = e->stereo ? 3 : 2;
        const double info = e->inv_sigma2;
        double chi2 = 0;
        for (int k = 0; k < D; k++)
            chi2 += o->err[k] * (info * o->err[k]);
        o->chi2 = chi2;
        double rho1 = 1.0;
        if (e->robust) {
            const float dsqr = (float)(e->huber_delta * e->huber_delta);
            if (!(chi2 <= dsqr))
                rho1 = e->huber_delta / sqrt(chi2);
        }
        o->rho1 = rho1;
        const double w = rho1 * info; /* weighted Omega = rho' * Omega (diagonal) */
        double wr[3];
        for (int k = 0; k < D; k++)
            wr[k] = -info * o->err[k] * rho1;
        /* from = point (never fixed in LBA), to = pose */
        double *hp = hpoint + 9 * (size_t)e->point, *bp = bpoint + 3 * (size_t)e->point;
        for (int r = 0; r < 3; r++) {
            double acc = 0;
            for (int k = 0; k < D; k++)
                acc += o->jp[k][r] * wr[k];
            bp[r] += acc;
            for (int c = 0; c < 3; c++) {
                double a2 = 0;
                for (int k = 0; k < D; k++)
                    a2 += o->jp[k][r] * w * o->jp[k][c];
                hp[r * 3 + c] += a2;
            }
        }
        if (!P->fixed) {
            for (int r = 0; r < 3; r++)
                for (int c = 0; c < 6; c++) {
                    double a2 = 0;
                    for (int k = 0; k < D; k++)
                        a2 += o->jp[k][r] * w * o->jt[k][c];
                    o->hpl[r][c] = a2;
                }
            double *ht = hpose + 36 * (size_t)e->pose, *bt = bpose + 6 * (size_t)e->pose;
            for (int r = 0; r < 6; r++) {
                double acc = 0;
                for (int k = 0; k < D; k++)
                    acc += o->jt[k][r] * wr[k];
                bt[r] += acc;
                for (int c = 0; c < 6; c++) {
                    double a2 = 0;
                    for (int k = 0; k < D; k++)
                        a2 += o->jt[k][r] * w * o->jt[k][c];
                    ht[r * 6 + c] += a2;
                }
            }
        }
    }
}

/* SparseOptimizer::computeActiveErrors (sparse_optimizer.cpp:61-76: e->computeError() per
 * edge), the robustified chi2 activeRobustChi2 sums (:100-114; RobustKernelHuber::robustify,
 * robust_kernel_impl.cpp:78-91, with its float dsqr member, robust_kernel_impl.h:84) and
 * isDepthPositive (types_six_dof_expmap.h:97-101, 129-133), for every edge given.  Returns the
 * sum of the robust chi2 over the active edges in edge order.  Any output may be NULL. */
double orc_ba_errors(const orc_pose *poses, const double *points, const orc_edge *edges,
                     int nedge, double *err, double *chi2, double *rho0, uint8_t *depth_ok)
{
    double total = 0;
    for (int i = 0; i < nedge; i++) {
        const orc_edge *e = &edges[i];
        double ev[3], xc[3];
        edge_error(&poses[e->pose], points + 3 * (size_t)e->point, e, ev, xc);
        const int D = e->stereo ? 3 : 2;
        double c = 0;
        for (int k = 0; k < D; k++)
            c += ev[k] * (e->inv_sigma2 * ev[k]);
        double r = c;
        if (e->robust) {
            const float dsqr = (float)(e->huber_delta * e->huber_delta);
            if (!(c <= dsqr))
                r = 2 * sqrt(c) * e->huber_delta - dsqr;
        }
        if (err)
            for (int k = 0; k < 3; k++)
                err[3 * (size_t)i + k] = ev[k];
        if (chi2)
            chi2[i] = c;
        if (rho0)
            rho0[i] = r;
        if (depth_ok)
            depth_ok[i] = xc[2] > 0.0;
        if (e->active)
            total += r;
    }
    return total;
}

/* SE3Quat::exp(update) * T applied in rotation-matrix form (se3quat.h:223-257) */
static void oplus_pose(const double R[3][3], const double t[3], const double upd[6],
                       double R2[3][3], double t2[3])
{
    const double w[3] = {upd[0], upd[1], upd[2]}, u[3] = {upd[3], upd[4], upd[5]};
    const double theta = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    const double O[3][3] = {{0, -w[2], w[1]}, {w[2], 0, -w[0]}, {-w[1], w[0], 0}};
    double O2[3][3], Re[3][3], V[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            O2[i][j] = 0;
            for (int k = 0; k < 3; k++)
                O2[i][j] += O[i][k] * O[k][j];
        }
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            const double I = (i == j) ? 1.0 : 0.0;
            if (theta < 0.00001) {
                Re[i][j] = I + O[i][j] + O2[i][j];
                V[i][j] = Re[i][j];
            } else {
                Re[i][j] = I + sin(theta) / theta * O[i][j] +
                           (1 - cos(theta)) / (theta * theta) * O2[i][j];
                V[i][j] = I + (1 - cos(theta)) / (theta * theta) * O[i][j] +
                          (theta - sin(theta)) / pow(theta, 3) * O2[i][j];
            }
        }
    double te[3];
    for (int i = 0; i < 3; i++)
        te[i] = V[i][0] * u[0] + V[i][1] * u[1] + V[i][2] * u[2];
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++)
            R2[i][j] = Re[i][0] * R[0][j] + Re[i][1] * R[1][j] + Re[i][2] * R[2][j];
        t2[i] = Re[i][0] * t[0] + Re[i][1] * t[1] + Re[i][2] * t[2] + te[i];
    }
}

void orc_ba_numeric_jacobian(const orc_pose *pose, const double *xyz, const orc_edge *e,
                             double jp[3][3], double jt[3][6])
{
    const double delta = 1e-9, scalar = 1.0 / (2 * delta);
    double R[3][3];
    quat_to_rot(pose->q, R);
    double ep[3], em[3];
    for (int d = 0; d < 3; d++) {
        double Xp[3] = {xyz[0], xyz[1], xyz[2]}, Xm[3] = {xyz[0], xyz[1], xyz[2]};
        Xp[d] += delta;
        Xm[d] -= delta;
        edge_error_rt(R, pose->t, Xp, e, ep, 1);
        edge_error_rt(R, pose->t, Xm, e, em, 1);
        for (int k = 0; k < 3; k++)
            jp[k][d] = scalar * (ep[k] - em[k]);
    }
    for (int d = 0; d < 6; d++) {
        double up[6] = {0, 0, 0, 0, 0, 0}, um[6] = {0, 0, 0, 0, 0, 0};
        up[d] = delta;
        um[d] = -delta;
        double R2[3][3], t2[3];
        oplus_pose(R, pose->t, up, R2, t2);
        edge_error_rt(R2, t2, xyz, e, ep, 1);
        oplus_pose(R, pose->t, um, R2, t2);
        edge_error_rt(R2, t2, xyz, e, em, 1);
        for (int k = 0; k < 3; k++)
            jt[k][d] = scalar * (ep[k] - em[k]);
    }
}

/* ---- BlockSolver<6,3>::solve with Schur complement (block_solver.hpp:354-486) ----
 * Pinned orders (see orb_oracle.h): landmarks in index order, a landmark's blocks in
 * ascending pose order, every small product summed in index order, Hschur blocks updated
 * landmark by landmark ("S -= BDinv Bj^T").  Eigen's 3x3 inverse (cofactors / det).  The
 * pose system is solved by a dense LDLT without pivoting in natural order (g2o's
 * LinearSolverEigen runs Eigen's SimplicialLDLT with an AMD ordering: unpinned). */
static void inv3_eigen(const double m[9], double r[9])
{
#define M(i, j) m[(i) * 3 + (j)]
#define COF(i, j) (M(((i) + 1) % 3, ((j) + 1) % 3) * M(((i) + 2) % 3, ((j) + 2) % 3) - \
                   M(((i) + 1) % 3, ((j) + 2) % 3) * M(((i) + 2) % 3, ((j) + 1) % 3))
    const double c0 = COF(0, 0), c1 = COF(1, 0), c2 = COF(2, 0);
    const double det = (c0 * M(0, 0) + c1 * M(1, 0)) + c2 * M(2, 0);
    const double invdet = 1.0 / det;
    r[0] = c0 * invdet;
    r[1] = c1 * invdet;
    r[2] = c2 * invdet;
    r[3] = COF(0, 1) * invdet;
    r[4] = COF(1, 1) * invdet;
    r[5] = COF(2, 1) * invdet;
    r[6] = COF(0, 2) * invdet;
    r[7] = COF(1, 2) * invdet;
    r[8] = COF(2, 2) * invdet;
#undef COF
#undef M
}

/* dense LDLT (no pivoting), A n x n row-major (lower triangle read), solve in place */
int orc_ldlt_dense_solve(double *A, int n, double *x)
{
    for (int j = 0; j < n; j++) {
        double d = A[j * n + j];
        for (int k = 0; k < j; k++)
            d -= A[j * n + k] * A[j * n + k] * A[k * n + k];
        A[j * n + j] = d;
        if (d == 0.0 || !isfinite(d))
            return 0;
        for (int i = j + 1; i < n; i++) {
            double s = A[i * n + j];
            for (int k = 0; k < j; k++)
                s -= A[i * n + k] * A[j * n + k] * A[k * n + k];
            A[i * n + j] = s / d;
        }
    }
    for (int i = 0; i < n; i++) { /* L y = b */
        double s = x[i];
        for (int k = 0; k < i; k++)
            s -= A[i * n + k] * x[k];
        x[i] = s;
    }
    for (int i = 0; i < n; i++)
        x[i] /= A[i * n + i];
    /* L^T x = y, column by column (k descending): element i subtracts L_ki x_k for
     * k = n-1 down to i+1, so each finished x_k updates every lower row at once (the GPU's
     * k_schur_ldlt runs one k per step over all rows) */
    for (int k = n - 1; k >= 0; k--)
        for (int i = 0; i < k; i++)
            x[i] -= A[k * n + i] * x[k];
    return 1;
}

/* the GPU block workgroup's chain combine: a pairwise tree over 16 chains */
#define SCHUR_CHAINS 16
static double schur_tree16(const double v[16])
{
    double a[8], b[4], c[2];
    for (int i = 0; i < 8; i++)
        a[i] = v[2 * i] + v[2 * i + 1];
    for (int i = 0; i < 4; i++)
        b[i] = a[2 * i] + a[2 * i + 1];
    for (int i = 0; i < 2; i++)
        c[i] = b[2 * i] + b[2 * i + 1];
    return c[0] + c[1];
}

int orc_ba_schur_solve(const orc_pose *poses, int npose, int npoint, const orc_edge *edges,
                       int nedge, const orc_edge_out *eout, const double *hpose,
                       const double *bpose, const double *hpoint, const double *bpoint,
                       double lambda, double *dx_pose, double *dx_point)
{
    /* free poses -> Schur index; points with an active edge to a free or fixed pose */
    int *pidx = (int *)malloc(sizeof(int) * (npose > 0 ? npose : 1));
    int nfree = 0;
    for (int i = 0; i < npose; i++)
        pidx[i] = poses[i].fixed ? -1 : nfree++;
    /* active edges per point, ascending pose (at most one edge per (pose, point)) */
    int *cnt = (int *)calloc((size_t)npoint + 1, sizeof(int));
    for (int e = 0; e < nedge; e++)
        if (edges[e].active)
            cnt[edges[e].point + 1]++;
    for (int i = 0; i < npoint; i++)
        cnt[i + 1] += cnt[i];
    int *lst = (int *)malloc(sizeof(int) * (nedge > 0 ? nedge : 1));
    int *fill = (int *)malloc(sizeof(int) * (npoint > 0 ? npoint : 1));
    memcpy(fill, cnt, sizeof(int) * (npoint > 0 ? npoint : 1));
    for (int e = 0; e < nedge; e++)
        if (edges[e].active)
            lst[fill[edges[e].point]++] = e;
    for (int p = 0; p < npoint; p++) /* insertion sort by pose */
        for (int a = cnt[p] + 1; a < cnt[p + 1]; a++) {
            const int v = lst[a];
            int b = a - 1;
            while (b >= cnt[p] && edges[lst[b]].pose > edges[v].pose) {
                lst[b + 1] = lst[b];
                b--;
            }
            lst[b + 1] = v;
        }
    const int n = 6 * nfree;
    /* S accumulates in SCHUR_CHAINS = 16 chains per block (the block's landmark pairs in
     * landmark order, pair t into chain t % 16), each chain a v_mfma_f64_4x4x4f64 accumulator
     * (one wave of the GPU's block workgroup): per pair the 3 (+1 zero pad) products fused
     * into the chain in k order, c = fma(-BD[r][k], h2[k][c], c), the instruction's measured
     * arithmetic (tools/microbench/mfma_f64_pin.hip: 1,280,000 of 1,280,000 lanes bit-equal
     * to that fma chain); S = the pairwise tree of the 16 chains (schur_tree16) */
    double *S4 = (double *)calloc(SCHUR_CHAINS * ((size_t)n * n + 1), sizeof(double));
    double *S = S4;  /* chain 0, the result after the combine */
    int *npair = (int *)calloc((size_t)nfree * nfree + 1, sizeof(int));
    /* coef of free pose i: its landmark-ordered list of B D^-1 b_l terms summed as 64 lane
     * partials (term t into partial t % 64, in order) and the xor butterfly 32 .. 1 */
    double *cpart = (double *)calloc((size_t)n * 64 + 1, sizeof(double));
    int *ncoef = (int *)calloc((size_t)nfree + 1, sizeof(int));
    double *coef = (double *)calloc((size_t)n + 1, sizeof(double));
    double *Dinv = (double *)malloc(sizeof(double) * 9 * (npoint > 0 ? npoint : 1));
    /* Hschur = Hpp + lambda (diagonal blocks): chain 0's start */
    for (int i = 0; i < npose; i++) {
        if (pidx[i] < 0)
            continue;
        const int o = 6 * pidx[i];
        for (int r = 0; r < 6; r++)
            for (int c = 0; c < 6; c++)
                S[(o + r) * n + o + c] = hpose[36 * (size_t)i + r * 6 + c] + (r == c ? lambda : 0.0);
    }
    for (int p = 0; p < npoint; p++) {
        double D[9];
        for (int k = 0; k < 9; k++)
            D[k] = hpoint[9 * (size_t)p + k];
        D[0] += lambda;
        D[4] += lambda;
        D[8] += lambda;
        double *Di = Dinv + 9 * (size_t)p;
        if (cnt[p + 1] == cnt[p]) { /* no active edge: not in the optimisation */
            memset(Di, 0, sizeof(double) * 9);
            continue;
        }
        inv3_eigen(D, Di);
        const double *bl = bpoint + 3 * (size_t)p;
        double db[3];
        for (int r = 0; r < 3; r++)
            db[r] = (Di[r * 3] * bl[0] + Di[r * 3 + 1] * bl[1]) + Di[r * 3 + 2] * bl[2];
        for (int a = cnt[p]; a < cnt[p + 1]; a++) {
            const int e1 = lst[a], i1 = pidx[edges[e1].pose];
            if (i1 < 0)
                continue;
            const double (*h1)[6] = eout[e1].hpl; /* Bi = h1^T (6 x 3) */
            double BD[6][3];
            for (int r = 0; r < 6; r++)
                for (int c = 0; c < 3; c++)
                    BD[r][c] = (h1[0][r] * Di[c] + h1[1][r] * Di[3 + c]) + h1[2][r] * Di[6 + c];
            {
                const int t = ncoef[i1]++;
                for (int r = 0; r < 6; r++)
                    cpart[(6 * (size_t)i1 + r) * 64 + (t & 63)] +=
                        (h1[0][r] * db[0] + h1[1][r] * db[1]) + h1[2][r] * db[2];
            }
            for (int b2 = a; b2 < cnt[p + 1]; b2++) {
                const int e2 = lst[b2], i2 = pidx[edges[e2].pose];
                if (i2 < 0)
                    continue;
                const double (*h2)[6] = eout[e2].hpl;
                double *Sc = S4 + (size_t)(npair[(size_t)i1 * nfree + i2]++ % SCHUR_CHAINS) *
                                      ((size_t)n * n + 1);
                for (int r = 0; r < 6; r++)
                    for (int c = 0; c < 6; c++) {
                        double *v = &Sc[(6 * i1 + r) * n + 6 * i2 + c];
                        for (int k = 0; k < 3; k++)
                            *v = fma(-BD[r][k], h2[k][c], *v);
                        *v = fma(0.0, 0.0, *v); /* the zero-padded k = 3 */
                    }
            }
        }
    }
    /* the chains of every upper block combined (blocks without pairs stay 0 / Hpp + lambda:
     * x + 0 = x) */
    {
        const size_t cs = (size_t)n * n + 1;
        for (int r = 0; r < n; r++)
            for (int c = r / 6 * 6; c < n; c++) {
                const size_t o = (size_t)r * n + c;
                double v[SCHUR_CHAINS];
                for (int u = 0; u < SCHUR_CHAINS; u++)
                    v[u] = S4[u * cs + o];
                S[o] = schur_tree16(v);
            }
    }
    /* symmetric: lower blocks mirror the upper ones */
    for (int r = 0; r < n; r++)
        for (int c = 0; c < r; c++)
            S[r * n + c] = S[c * n + r];
    for (int i = 0; i < nfree; i++)
        for (int r = 0; r < 6; r++) {
            double v[64];
            memcpy(v, cpart + (6 * (size_t)i + r) * 64, sizeof(v));
            for (int off = 32; off >= 1; off >>= 1) {
                double w[64];
                for (int l = 0; l < 64; l++)
                    w[l] = v[l] + v[l ^ off];
                memcpy(v, w, sizeof(v));
            }
            coef[6 * i + r] = v[0];
        }
    double *xp = (double *)calloc((size_t)n + 1, sizeof(double));
    for (int i = 0; i < npose; i++)
        if (pidx[i] >= 0)
            for (int r = 0; r < 6; r++)
                xp[6 * pidx[i] + r] = bpose[6 * (size_t)i + r] - coef[6 * pidx[i] + r];
    const int ok = n == 0 ? 1 : orc_ldlt_dense_solve(S, n, xp);
    for (int i = 0; i < npose; i++)
        for (int r = 0; r < 6; r++)
            dx_pose[6 * (size_t)i + r] = (ok && pidx[i] >= 0) ? xp[6 * pidx[i] + r] : 0.0;
    for (int p = 0; p < npoint; p++) {
        double *xl = dx_point + 3 * (size_t)p;
        xl[0] = xl[1] = xl[2] = 0.0;
        if (!ok || cnt[p + 1] == cnt[p])
            continue;
        const double *bl = bpoint + 3 * (size_t)p;
        double cl[3] = {bl[0], bl[1], bl[2]};
        for (int a = cnt[p]; a < cnt[p + 1]; a++) {
            const int e1 = lst[a], i1 = pidx[edges[e1].pose];
            if (i1 < 0)
                continue;
            const double (*h1)[6] = eout[e1].hpl;
            for (int k = 0; k < 3; k++) {
                double s = 0;
                for (int r = 0; r < 6; r++)
                    s += h1[k][r] * -xp[6 * i1 + r];
                cl[k] += s;
            }
        }
        const double *Di = Dinv + 9 * (size_t)p;
        for (int r = 0; r < 3; r++)
            xl[r] = (Di[r * 3] * cl[0] + Di[r * 3 + 1] * cl[1]) + Di[r * 3 + 2] * cl[2];
    }
    free(pidx);
    free(cnt);
    free(lst);
    free(fill);
    free(S4);
    free(npair);
    free(cpart);
    free(ncoef);
    free(coef);
    free(Dinv);
    free(xp);
    return ok;
}

/* ---- the Levenberg-Marquardt loop of LocalBundleAdjustment's optimizer.optimize(n) ----
 * SparseOptimizer::optimize + OptimizationAlgorithmLevenberg::solve
 * (optimization_algorithm_levenberg.cpp:61-164; tau 1e-5 :47, goodStep scales 2/3 and 1/3
 * :48-49, maxTrialsAfterFailure 10 :51, computeLambdaInit :166-180, computeScale :182-189),
 * SparseOptimizer::update (oplusImpl of the two vertex types, types_six_dof_expmap.h:73-76 and
 * the point's +=), push / pop as copies.  Sums in g2o's sequential order (activeRobustChi2 over
 * the active edges in edge order, computeScale over [free poses' increments, points'] in
 * index order -- fixed poses and edge-less points contribute exact zeros). */
void orc_ba_update(orc_pose *poses, int npose, double *points, int npoint, const double *dx_pose,
                   const double *dx_point)
{
    for (int i = 0; i < npose; i++)
        if (!poses[i].fixed)
            orc_se3_oplus(poses[i].q, poses[i].t, dx_pose + 6 * (size_t)i);
    for (size_t j = 0; j < 3 * (size_t)npoint; j++)
        points[j] += dx_point[j];
}

/* optimize(iterations) with g2o's force-stop flag (SparseOptimizer::setForceStopFlag,
 * sparse_optimizer.h:184-188) restated for tests: the flag is polled where g2o polls
 * terminate() -- before every iteration (sparse_optimizer.cpp:376, after postIteration) and
 * after every trial (optimization_algorithm_levenberg.cpp:149).  The test's flag is raised
 * after trial stop_trial of iteration stop_it (stop_trial -1: after iteration stop_it's
 * postIteration; stop_it -1: never; stop_it -2: already raised before the call).
 * last_chi2 (NULL: not kept) receives every edge's chi2 from the last error pass the call
 * ran (g2o's edges keep the _error of the last computeActiveErrors: the last trial's, accepted
 * or not); untouched if no iteration ran.  report[6] as orc_ba_optimize, report[2] = 3 when the
 * flag stopped it and nothing else did. */
int orc_ba_optimize_ctl(orc_pose *poses, int npose, double *points, int npoint,
                        const orc_edge *edges, int nedge, int iterations, int stop_it,
                        int stop_trial, double *last_chi2, double report[6])
{
    const size_t np = npose > 0 ? (size_t)npose : 1, nq = npoint > 0 ? (size_t)npoint : 1;
    const size_t ne = nedge > 0 ? (size_t)nedge : 1;
    orc_edge_out *eo = (orc_edge_out *)calloc(ne, sizeof(orc_edge_out));
    double *hp = (double *)calloc(np * 36, 8), *bp = (double *)calloc(np * 6, 8);
    double *hq = (double *)calloc(nq * 9, 8), *bq = (double *)calloc(nq * 3, 8);
    double *dxp = (double *)calloc(np * 6, 8), *dxq = (double *)calloc(nq * 3, 8);
    double *chi = (double *)calloc(ne, 8);
    orc_pose *sp = (orc_pose *)calloc(np, sizeof(orc_pose));
    double *sq = (double *)calloc(nq * 3, 8);
    double currentChi = 0, lambda = 0;
    int ni = 2, nBad = 0, it = 0, trials = 0, term = 0, ran = 0;
    int stop = stop_it == -2;
    report[3] = 0;
    for (it = 0; it < iterations && !stop; it++) {
        if (it == 0) {
            currentChi = orc_ba_errors(poses, points, edges, nedge, NULL, chi, NULL, NULL);
            report[3] = currentChi;
        }
        ran = 1;
        const double iniChi = currentChi;
        orc_ba_linearize(poses, npose, points, npoint, edges, nedge, eo, hp, bp, hq, bq);
        if (it == 0) {
            double m = 0;
            for (int i = 0; i < npose; i++)
                if (!poses[i].fixed)
                    for (int j = 0; j < 6; j++)
                        m = fmax(fabs(hp[36 * (size_t)i + 7 * j]), m);
            for (int p = 0; p < npoint; p++)
                for (int j = 0; j < 3; j++)
                    m = fmax(fabs(hq[9 * (size_t)p + 4 * j]), m);
            lambda = 1e-5 * m;
            ni = 2;
            nBad = 0;
        }
        double rho = 0;
        int qmax = 0;
        do {
            memcpy(sp, poses, (size_t)npose * sizeof(orc_pose));
            memcpy(sq, points, (size_t)npoint * 24);
            const int ok2 = orc_ba_schur_solve(poses, npose, npoint, edges, nedge, eo, hp, bp, hq,
                                               bq, lambda, dxp, dxq);
            orc_ba_update(poses, npose, points, npoint, dxp, dxq);
            double tempChi = orc_ba_errors(poses, points, edges, nedge, NULL, chi, NULL, NULL);
            if (!ok2)
                tempChi = DBL_MAX;
            rho = currentChi - tempChi;
            double scale = 0;
            for (int i = 0; i < npose; i++)
                if (!poses[i].fixed)
                    for (int j = 0; j < 6; j++) {
                        const double x = dxp[6 * (size_t)i + j];
                        scale += x * (lambda * x + bp[6 * (size_t)i + j]);
                    }
            for (size_t j = 0; j < 3 * (size_t)npoint; j++)
                scale += dxq[j] * (lambda * dxq[j] + bq[j]);
            scale += 1e-3;
            rho /= scale;
            trials++;
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
                memcpy(poses, sp, (size_t)npose * sizeof(orc_pose));
                memcpy(points, sq, (size_t)npoint * 24);
            }
            qmax++;
            if (it == stop_it && qmax - 1 == stop_trial)
                stop = 1;
        } while (rho < 0 && qmax < 10 && !stop);
        int ok = 1;
        if (qmax == 10 || rho == 0) {
            term = 1;
            ok = 0;
        } else {
            if ((iniChi - currentChi) * 1e3 < iniChi)
                nBad++;
            else
                nBad = 0;
            if (nBad >= 3) {
                term = 2;
                ok = 0;
            }
        }
        if (it == stop_it && stop_trial == -1)
            stop = 1;  /* postIteration(i) */
        if (!ok) {
            it++;
            break;
        }
    }
    if (!ran)
        report[3] = currentChi = orc_ba_errors(poses, points, edges, nedge, NULL, NULL, NULL, NULL);
    else if (last_chi2)
        memcpy(last_chi2, chi, (size_t)nedge * 8);
    if (stop && !term)
        term = 3;
    report[0] = it;
    report[1] = trials;
    report[2] = term;
    report[4] = currentChi;
    report[5] = lambda;
    free(eo);
    free(hp);
    free(bp);
    free(hq);
    free(bq);
    free(dxp);
    free(dxq);
    free(chi);
    free(sp);
    free(sq);
    return it;
}

int orc_ba_optimize(orc_pose *poses, int npose, double *points, int npoint, const orc_edge *edges,
                    int nedge, int iterations, double report[6])
{
    return orc_ba_optimize_ctl(poses, npose, points, npoint, edges, nedge, iterations, -1, -1,
                               NULL, report);
}
