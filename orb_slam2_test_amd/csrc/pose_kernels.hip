// pose_kernels.hip -- Optimizer::PoseOptimization (src/Optimizer.cc:356-631) for gfx950.
//
// One 256-thread workgroup per frame runs the whole motion-only BA: four rounds of
// g2o's Levenberg-Marquardt optimize(10) on one VertexSE3Expmap with unary
// EdgeSE3ProjectXYZOnlyPose / EdgeStereoSE3ProjectXYZOnlyPose edges (Huber in rounds 0-2),
// re-classifying outliers after each round.  Every LM trial is one pass over the frame's
// edges: thread t takes edges t, t+256, ... and accumulates the robust chi2, the lower
// triangle of H = J^T W J and b = -rho' J^T Omega e in registers (28 doubles), then the
// workgroup reduces them in the pinned order of oracle/pose_oracle.c (butterfly within a
// wave, (w0 + w1) + (w2 + w3) across waves), so the result is bit-identical to the oracle.
// The 6x6 LDLT solve, the SE3 exp update and the step control run on lane 0 (state in LDS).  A trial's
// pass also yields the system at the trial pose, which the next iteration reuses when the
// step is accepted (g2o rebuilds it at the same pose: same values).
//
// fp64 throughout; no FMA contraction; sin/cos of the exp map pinned (orbg_device.h).
#include <hip/hip_runtime.h>

#include <cfloat>
#include <climits>

#include "../../include/orbg.h"
#include "orbg_internal.h"
#include "orbg_device.h"
#include "se3_device.h"
#include "match_device.h"

#pragma clang fp contract(off)

namespace orbg {

void prof_begin(void *prof, hipStream_t s, const char *n, hipEvent_t *a);
void prof_end(void *prof, hipStream_t s, const char *n, hipEvent_t a);

struct PoseInvSigma2 {
    float v[16];
};

#define PO_T 256
#define PO_NV 28  // robust chi2, 21 lower-triangle H entries, 6 b entries

// Eigen LDLT (lower, diagonal pivoting) + solve; returns isPositive()
__device__ bool ldlt_solve6(double m[6][6], const double b[6], double x[6])
{
    int tr[6];
    int sign = 0;  // 0 zero, 1 positive semidef, 2 negative semidef, 3 indefinite
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
        if (k > 0) {
            for (int j = 0; j < k; j++) temp[j] = m[j][j] * m[k][j];
            double dot = 0;
            for (int j = 0; j < k; j++) dot += m[k][j] * temp[j];
            m[k][k] -= dot;
            for (int i = k + 1; i < 6; i++) {
                double s = 0;
                for (int j = 0; j < k; j++) s += m[i][j] * temp[j];
                m[i][k] -= s;
            }
        }
        const double akk = m[k][k];
        const bool valid = fabs(akk) > 0.0;
        if (k == 0 && !valid) {
            sign = 0;
            for (int j = 0; j < 6; j++) tr[j] = j;
            break;
        }
        if (k < 5 && valid)
            for (int i = k + 1; i < 6; i++) m[i][k] /= akk;
        if (sign == 0 || sign == 1) {
            if (akk > 0) sign = 1;
            else if (akk < 0) sign = sign == 0 ? 2 : 3;
        } else if (sign == 2 && akk > 0) {
            sign = 3;
        }
    }
    if (!(sign == 1 || sign == 0)) return false;
    double d[6];
    for (int i = 0; i < 6; i++) d[i] = b[i];
    for (int k = 0; k < 6; k++) {
        const double s = d[k];
        d[k] = d[tr[k]];
        d[tr[k]] = s;
    }
    for (int i = 0; i < 6; i++) {
        double s = 0;
        for (int j = 0; j < i; j++) s += m[i][j] * d[j];
        d[i] -= s;
    }
    for (int i = 0; i < 6; i++) d[i] = fabs(m[i][i]) > DBL_MIN ? d[i] / m[i][i] : 0.0;
    for (int i = 5; i >= 0; i--) {
        double s = 0;
        for (int j = i + 1; j < 6; j++) s += m[j][i] * d[j];
        d[i] -= s;
    }
    for (int k = 5; k >= 0; k--) {
        const double s = d[k];
        d[k] = d[tr[k]];
        d[tr[k]] = s;
    }
    for (int i = 0; i < 6; i++) x[i] = d[i];
    return true;
}

// ---- the unary edges ----
__device__ __forceinline__ int pedge_error(const double q[4], const double t[3],
                                           const orbg_pose_edge &e, const orbg_pose_camera &cam,
                                           double err[3], double xc[3])
{
    const double X[3] = {e.xw[0], e.xw[1], e.xw[2]};
    q_rotate(q, X, xc);
    xc[0] += t[0];
    xc[1] += t[1];
    xc[2] += t[2];
    const double fx = cam.fx, fy = cam.fy, cx = cam.cx, cy = cam.cy;
    if (!e.stereo) {
        const double px = xc[0] / xc[2], py = xc[1] / xc[2];
        err[0] = (double)e.obs[0] - (px * fx + cx);
        err[1] = (double)e.obs[1] - (py * fy + cy);
        err[2] = 0;
        return 2;
    }
    const float invz = (float)(1.0f / xc[2]);
    const double u = xc[0] * invz * fx + cx;
    const double v = xc[1] * invz * fy + cy;
    err[0] = (double)e.obs[0] - u;
    err[1] = (double)e.obs[1] - v;
    err[2] = (double)e.obs[2] - (u - (double)cam.bf * invz);
    return 3;
}

__device__ __forceinline__ double pedge_chi2(const double err[3], int D, double info)
{
    // err[2] = 0 for a mono edge: the third term adds +0 (see po_partial)
    (void)D;
    double chi2 = 0;
#pragma unroll
    for (int k = 0; k < 3; k++) chi2 += err[k] * (info * err[k]);
    return chi2;
}

// per-thread partial sums of one pass at (q, t) over the active edges
__device__ void po_partial(const double q[4], const double t[3], const orbg_pose_edge *edges,
                           int n, const uint8_t *outlier, bool robust,
                           const orbg_pose_camera &cam, double p[PO_NV])
{
    for (int j = 0; j < PO_NV; j++) p[j] = 0;
    const double dmono = (double)(float)sqrt(5.991), dstereo = (double)(float)sqrt(7.815);
    for (int e = threadIdx.x; e < n; e += PO_T) {
        if (outlier[e]) continue;
        const orbg_pose_edge E = edges[e];
        double err[3], xc[3];
        const int D = pedge_error(q, t, E, cam, err, xc);
        const double info = E.inv_sigma2;
        const double chi2 = pedge_chi2(err, D, info);
        double rho1 = 1.0, rho0 = chi2;
        if (robust) {
            const double delta = E.stereo ? dstereo : dmono;
            const float dsqr = (float)(delta * delta);
            if (!(chi2 <= dsqr)) {
                const double sq = sqrt(chi2);
                rho1 = delta / sq;
                rho0 = 2 * sq * delta - dsqr;
            }
        }
        p[0] += rho0;
        // linearizeOplus (types_six_dof_expmap.cpp:266-288, 335-364)
        double J[3][6];
        {
            const double x = xc[0], y = xc[1];
            const double invz = 1.0 / xc[2], invz_2 = invz * invz;
            const double fx = cam.fx, fy = cam.fy, bf = cam.bf;
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
            if (D == 3) {
                J[2][0] = J[0][0] - bf * y * invz_2;
                J[2][1] = J[0][1] + bf * x * invz_2;
                J[2][2] = J[0][2];
                J[2][3] = J[0][3];
                J[2][4] = 0;
                J[2][5] = J[0][5] - bf * invz_2;
            } else {
#pragma unroll
                for (int c = 0; c < 6; c++) J[2][c] = 0;
            }
        }
        // fixed three rows: a mono edge's third row is +0 (J) / -0 (wr), and adding those
        // to sums that start at +0 leaves every bit as the oracle's two-row loop does
        const double w = rho1 * info;
        double wr[3];
#pragma unroll
        for (int k = 0; k < 3; k++) wr[k] = -info * err[k] * rho1;
        int hi = 1;
#pragma unroll
        for (int r = 0; r < 6; r++)
#pragma unroll
            for (int c = 0; c <= r; c++) {
                double a2 = 0;
#pragma unroll
                for (int k = 0; k < 3; k++) a2 += J[k][r] * w * J[k][c];
                p[hi++] += a2;
            }
#pragma unroll
        for (int r = 0; r < 6; r++) {
            double acc = 0;
#pragma unroll
            for (int k = 0; k < 3; k++) acc += J[k][r] * wr[k];
            p[22 + r] += acc;
        }
    }
}

// pinned reduction: butterfly within each wave, (w0 + w1) + (w2 + w3); result in red[0..27]
__device__ void po_reduce(double p[PO_NV], double *wred /* [4][PO_NV] */, double *red)
{
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int j = 0; j < PO_NV; j++) {
        double v = p[j];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v = v + __shfl_xor(v, o, 64);
        if (lane == 0) wred[wv * PO_NV + j] = v;
    }
    __syncthreads();
    if (threadIdx.x < PO_NV) {
        const int j = threadIdx.x;
        red[j] = (wred[j] + wred[PO_NV + j]) + (wred[2 * PO_NV + j] + wred[3 * PO_NV + j]);
    }
    __syncthreads();
}

__device__ __forceinline__ void unpack_sys(const double *red, double *H, double *b)
{
    int hi = 1;
    for (int r = 0; r < 6; r++)
        for (int c = 0; c <= r; c++) {
            H[r * 6 + c] = red[hi];
            H[c * 6 + r] = red[hi];
            hi++;
        }
    for (int r = 0; r < 6; r++) b[r] = red[22 + r];
}

struct PoShared {
    double red[PO_NV];
    double wred[4 * PO_NV];
    double q[4], t[3];     // current estimate
    double tq[4], tt[3];   // trial estimate
    double lq[4], lt[3];   // where computeActiveErrors last ran
    double H[36], b[6], x[6];
    int go;                // lane 0's loop decisions: bit 0 continue trials, bit 1 stop LM
};

// Lane 0 owns all of the LM scalar state (lambda, ni, chi values, the 6x6 system and its
// solve); the workgroup only runs the edge passes.  Barriers hand the trial pose out and
// the reduced sums back.
__global__ __launch_bounds__(PO_T) void k_pose_opt(const orbg_pose_edge *__restrict__ edges_all,
                                                    const int32_t *__restrict__ counts, int cap,
                                                    const orbg_pose_camera *__restrict__ cams,
                                                    const float *__restrict__ tcw_in,
                                                    double *__restrict__ q_out,
                                                    double *__restrict__ t_out,
                                                    float *__restrict__ tcw_out,
                                                    uint8_t *__restrict__ outlier_all,
                                                    int32_t *__restrict__ ninliers)
{
    __shared__ PoShared S;
    const int f = blockIdx.x, tid = threadIdx.x;
    const int n = counts[f];
    const orbg_pose_edge *edges = edges_all + (size_t)f * cap;
    uint8_t *outlier = outlier_all + (size_t)f * cap;
    const orbg_pose_camera cam = cams[f];
    const float *Tin = tcw_in + (size_t)f * 12;
    for (int i = tid; i < n; i += PO_T) outlier[i] = 0;
    if (tid == 0) {
        // Converter::toSE3Quat
        double R[3][3];
        for (int i = 0; i < 3; i++) {
            for (int j = 0; j < 3; j++) R[i][j] = Tin[4 * i + j];
            S.tt[i] = Tin[4 * i + 3];
        }
        q_from_rot(R, S.tq);
        q_normalize(S.tq);
    }
    __syncthreads();
    double q0[4], t0[3];
    for (int i = 0; i < 4; i++) q0[i] = S.tq[i];
    for (int i = 0; i < 3; i++) t0[i] = S.tt[i];
    if (n < 3) {
        if (tid == 0) {
            for (int i = 0; i < 4; i++) q_out[f * 4 + i] = q0[i];
            for (int i = 0; i < 3; i++) t_out[f * 3 + i] = t0[i];
            for (int i = 0; i < 12; i++) tcw_out[f * 12 + i] = Tin[i];
            ninliers[f] = 0;
        }
        return;
    }
    bool robust = true;
    int nBad = 0;
    double p[PO_NV];
    // lane-0 state
    double lambda = 0, ni = 2, currentChi = 0, iniChi = 0;
    int nBadLM = 0, qmax = 0;
    bool have_sys = false;
    for (int round = 0; round < 4; round++) {
        if (tid == 0) {
            for (int i = 0; i < 4; i++) S.q[i] = q0[i];
            for (int i = 0; i < 3; i++) S.t[i] = t0[i];
        }
        int act = 0;
        for (int i = tid; i < n; i += PO_T) act += !outlier[i];
        act = __syncthreads_or(act);
        if (act) {
            // ---- optimize(10): OptimizationAlgorithmLevenberg::solve per iteration ----
            have_sys = false;
            for (int it = 0; it < 10; it++) {
                if (!__syncthreads_or(have_sys)) {
                    // computeActiveErrors + buildSystem at the current estimate
                    po_partial(S.q, S.t, edges, n, outlier, robust, cam, p);
                    po_reduce(p, S.wred, S.red);
                    if (tid == 0) {
                        for (int i = 0; i < 4; i++) S.lq[i] = S.q[i];
                        for (int i = 0; i < 3; i++) S.lt[i] = S.t[i];
                        currentChi = S.red[0];
                        unpack_sys(S.red, S.H, S.b);
                    }
                }
                if (tid == 0) {
                    have_sys = false;
                    iniChi = currentChi;
                    if (it == 0) {
                        double maxd = 0;
                        for (int j = 0; j < 6; j++) maxd = fmax(fabs(S.H[j * 7]), maxd);
                        lambda = 1e-5 * maxd;
                        ni = 2;
                        nBadLM = 0;
                    }
                    qmax = 0;
                }
                for (;;) {
                    bool ok2 = false;
                    if (tid == 0) {
                        // setLambda, LDLT solve, oplus (trial), restoreDiagonal
                        double Hd[6][6];
                        for (int r = 0; r < 6; r++)
                            for (int c = 0; c < 6; c++) Hd[r][c] = S.H[r * 6 + c];
                        for (int j = 0; j < 6; j++) Hd[j][j] += lambda;
                        ok2 = ldlt_solve6(Hd, S.b, S.x);
                        for (int i = 0; i < 4; i++) S.tq[i] = S.q[i];
                        for (int i = 0; i < 3; i++) S.tt[i] = S.t[i];
                        se3_oplus(S.tq, S.tt, S.x);
                        for (int i = 0; i < 4; i++) S.lq[i] = S.tq[i];
                        for (int i = 0; i < 3; i++) S.lt[i] = S.tt[i];
                    }
                    __syncthreads();
                    po_partial(S.tq, S.tt, edges, n, outlier, robust, cam, p);
                    po_reduce(p, S.wred, S.red);
                    if (tid == 0) {
                        double tempChi = S.red[0];
                        if (!ok2) tempChi = DBL_MAX;
                        double rho = currentChi - tempChi;
                        double scale = 0;
                        for (int j = 0; j < 6; j++) scale += S.x[j] * (lambda * S.x[j] + S.b[j]);
                        scale += 1e-3;
                        rho /= scale;
                        if (rho > 0 && isfinite(tempChi)) {
                            double alpha = 1. - lm_cube(2 * rho - 1);
                            alpha = fmin(alpha, 2. / 3.);
                            const double sf = fmax(1. / 3., alpha);
                            lambda *= sf;
                            ni = 2;
                            currentChi = tempChi;
                            for (int i = 0; i < 4; i++) S.q[i] = S.tq[i];
                            for (int i = 0; i < 3; i++) S.t[i] = S.tt[i];
                            // the system at the accepted pose is the next buildSystem's
                            unpack_sys(S.red, S.H, S.b);
                            have_sys = true;
                        } else {
                            lambda *= ni;
                            ni *= 2;
                        }
                        qmax++;
                        int go = 0;
                        if (rho < 0 && qmax < 10) {
                            go = 1;  // another trial
                        } else if (qmax == 10 || rho == 0) {
                            go = 2;  // Terminate
                        } else {
                            if ((iniChi - currentChi) * 1e3 < iniChi)
                                nBadLM++;
                            else
                                nBadLM = 0;
                            if (nBadLM >= 3) go = 2;
                        }
                        S.go = go;
                    }
                    __syncthreads();
                    if (S.go != 1) break;
                }
                if (S.go == 2) break;
            }
        }
        __syncthreads();
        // ---- classification (Optimizer.cc:518-580) ----
        int bad = 0;
        for (int i = tid; i < n; i += PO_T) {
            const orbg_pose_edge E = edges[i];
            double err[3], xc[3];
            const bool was_active = !outlier[i];
            const int D = was_active ? pedge_error(S.lq, S.lt, E, cam, err, xc)
                                     : pedge_error(S.q, S.t, E, cam, err, xc);
            const float chi2 = (float)pedge_chi2(err, D, E.inv_sigma2);
            const bool o = chi2 > (E.stereo ? 7.815f : 5.991f);
            outlier[i] = o;
            bad += o;
        }
        bad = wave_isum(bad);
        if ((tid & 63) == 0) S.wred[tid >> 6] = bad;
        __syncthreads();
        nBad = (int)(S.wred[0] + S.wred[1] + S.wred[2] + S.wred[3]);
        __syncthreads();
        if (round == 2) robust = false;
        if (n < 10) break;
    }
    if (tid == 0) {
        for (int i = 0; i < 4; i++) q_out[f * 4 + i] = S.q[i];
        for (int i = 0; i < 3; i++) t_out[f * 3 + i] = S.t[i];
        // Converter::toCvMat(SE3Quat)
        const double *q = S.q;
        const double tx = 2 * q[0], ty = 2 * q[1], tz = 2 * q[2];
        const double twx = tx * q[3], twy = ty * q[3], twz = tz * q[3];
        const double txx = tx * q[0], txy = ty * q[0], txz = tz * q[0];
        const double tyy = ty * q[1], tyz = tz * q[1], tzz = tz * q[2];
        const double R[3][3] = {{1 - (tyy + tzz), txy - twz, txz + twy},
                                {txy + twz, 1 - (txx + tzz), tyz - twx},
                                {txz - twy, tyz + twx, 1 - (txx + tyy)}};
        for (int i = 0; i < 3; i++) {
            for (int j = 0; j < 3; j++) tcw_out[f * 12 + 4 * i + j] = (float)R[i][j];
            tcw_out[f * 12 + 4 * i + 3] = (float)S.t[i];
        }
        ninliers[f] = n - nBad;
    }
}

// ---- the batched-sequence trajectory stub: PoseOptimization edges from the matches ----
// One workgroup per frame pair p (F1 = f1[p], F2 = f2[p]): SearchForInitialization's
// vnMatches12 (m12[p][i] = F2 index matched to F1 keypoint i) inverted in LDS, then one mono
// edge per matched F2 keypoint j in index order (PoseOptimization's loop over pFrame,
// Optimizer.cc:381): obs = F2 keypoint j, Xw = F1 keypoint back-projected at `depth` in F1's
// camera (float, oracle/pose_oracle.c orc_match_pose), Omega = mvInvLevelSigma2[octave j].
// Also the pair's camera and identity initial pose for k_pose_opt.
__global__ __launch_bounds__(256) void k_match_pose_edges(
    const orbg_keypoint *__restrict__ kps, const int32_t *__restrict__ counts, int fc,
    const int32_t *__restrict__ f1, const int32_t *__restrict__ f2,
    const int32_t *__restrict__ m12, orbg_pose_camera cam, float depth, PoseInvSigma2 inv2,
    orbg_pose_edge *__restrict__ edges, int32_t *__restrict__ ecount,
    orbg_pose_camera *__restrict__ cams, float *__restrict__ tcw0)
{
    extern __shared__ int pinv[];  // fc entries
    __shared__ int wsum[4];
    const int p = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int a = f1[p], b = f2[p];
    const int n1 = counts[a], n2 = counts[b];
    const orbg_keypoint *k1 = kps + (size_t)a * fc, *k2 = kps + (size_t)b * fc;
    for (int j = tid; j < n2; j += 256) pinv[j] = -1;
    __syncthreads();
    for (int i = tid; i < n1; i += 256) {
        const int j = m12[(size_t)p * fc + i];
        if (j >= 0 && j < n2) pinv[j] = i;
    }
    __syncthreads();
    orbg_pose_edge *E = edges + (size_t)p * fc;
    int run = 0;
    for (int j0 = 0; j0 < n2; j0 += 256) {
        const int j = j0 + tid;
        const int i = j < n2 ? pinv[j] : -1;
        const int f = i >= 0;
        const int incl = wave_incl_scan(f);
        if (lane == 63) wsum[wv] = incl;
        __syncthreads();
        int before = run, tot = run;
        for (int w = 0; w < 4; w++) {
            before += w < wv ? wsum[w] : 0;
            tot += wsum[w];
        }
        if (f) {
            const orbg_keypoint kq = k2[j], kr = k1[i];
            orbg_pose_edge e;
            e.obs[0] = kq.x;
            e.obs[1] = kq.y;
            e.obs[2] = -1.f;
            e.xw[0] = (kr.x - cam.cx) * depth / cam.fx;
            e.xw[1] = (kr.y - cam.cy) * depth / cam.fy;
            e.xw[2] = depth;
            e.inv_sigma2 = inv2.v[kq.octave];
            e.stereo = 0;
            E[before + incl - 1] = e;
        }
        run = tot;
        __syncthreads();
    }
    if (tid == 0) {
        ecount[p] = run;
        cams[p] = cam;
    }
    if (tid < 12) tcw0[12 * (size_t)p + tid] = (tid % 5 == 0) ? 1.f : 0.f;  // [I | 0]
}

int launch_pose_opt(hipStream_t st, const orbg_pose_edge *edges, const int32_t *counts, int cap,
                    const orbg_pose_camera *cams, const float *tcw_in, double *q_out,
                    double *t_out, float *tcw_out, uint8_t *outlier, int32_t *ninliers,
                    int nframes, void *prof);

int launch_match_pose(hipStream_t st, const orbg_keypoint *kps, const int32_t *counts, int fc,
                      const int32_t *f1, const int32_t *f2, const int32_t *m12, int npairs,
                      const orbg_pose_camera &cam, float depth, const float *inv_sigma2, int nlev,
                      orbg_pose_edge *edges, int32_t *ecount, orbg_pose_camera *cams,
                      float *tcw0, float *tcw_out, uint8_t *outlier, double *q_out,
                      double *t_out, int32_t *ninliers, void *prof)
{
    if (npairs <= 0) return ORBG_OK;
    PoseInvSigma2 inv2{};
    for (int l = 0; l < nlev && l < 16; l++) inv2.v[l] = inv_sigma2[l];
    hipLaunchKernelGGL(k_match_pose_edges, dim3(npairs), dim3(256), (size_t)fc * 4, st, kps,
                       counts, fc, f1, f2, m12, cam, depth, inv2, edges, ecount, cams, tcw0);
    if (hipGetLastError() != hipSuccess) return ORBG_EIO;
    return launch_pose_opt(st, edges, ecount, fc, cams, tcw0, q_out, t_out, tcw_out, outlier,
                           ninliers, npairs, prof);
}

int launch_pose_opt(hipStream_t st, const orbg_pose_edge *edges, const int32_t *counts, int cap,
                    const orbg_pose_camera *cams, const float *tcw_in, double *q_out,
                    double *t_out, float *tcw_out, uint8_t *outlier, int32_t *ninliers,
                    int nframes, void *prof)
{
    if (nframes <= 0) return ORBG_OK;
    hipEvent_t ev = nullptr;
    prof_begin(prof, st, "pose_opt", &ev);
    hipLaunchKernelGGL(k_pose_opt, dim3(nframes), dim3(PO_T), 0, st, edges, counts, cap, cams,
                       tcw_in, q_out, t_out, tcw_out, outlier, ninliers);
    prof_end(prof, st, "pose_opt", ev);
    return hipGetLastError() == hipSuccess ? ORBG_OK : ORBG_EIO;
}

}  // namespace orbg
