/*
 * oracle/stereo_oracle.c -- TEST INFRASTRUCTURE ONLY (see orb_oracle.h).
 *
 * Frame::ComputeStereoMatches (src/Frame.cc:619-834) restated in plain C:
 *   :637-662  row table: right keypoint iR is listed in rows floor(y - r) .. ceil(y + r),
 *             r = 2 * mvScaleFactors[octave]
 *   :664-668  minZ = mb, minD = 0, maxD = mbf / minZ.  The reference reads mb before the
 *             constructor assigns it (Frame.cc:661 vs :148, an uninitialised member); here
 *             it is the parameter min_z (callers pass bf / fx, the value assigned right
 *             after; min_z <= 0 gives maxD = +inf)
 *   :676-738  per left keypoint: candidates of row (size_t)vL, octave within +-1,
 *             uL - maxD <= uR <= uL; best = first strictly smaller Hamming distance
 *             starting from TH_HIGH; accepted if < (TH_HIGH + TH_LOW) / 2
 *   :740-797  11x11 SAD at the keypoint's level, window centred on round(x * invScale),
 *             both patches minus their centre pixel, shifts -5..5 (first minimum),
 *             boundary check iniu < 0 || endu >= cols as written (right side only)
 *   :799-832  parabola through the three SADs around the minimum (float), |delta| <= 1,
 *             uR = scale * (round(uR0 * inv) + inc + delta), disparity in [0, maxD)
 *             (0 -> 0.01), depth = bf / disparity
 *   :836-851  sort (SAD, iL); median = element size/2; clear every match with
 *             SAD >= 1.5f * 1.4f * median
 * The patch values are integers, so cv::norm(NORM_L1) of the float patches is an exact
 * integer; it is computed in int here.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "orb_oracle.h"

#define TH_HIGH 100
#define TH_LOW 50

typedef struct {
    int dist, idx;
} dist_idx;

static int cmp_dist_idx(const void *a, const void *b)
{
    const dist_idx *x = (const dist_idx *)a, *y = (const dist_idx *)b;
    if (x->dist != y->dist) return x->dist < y->dist ? -1 : 1;
    return x->idx < y->idx ? -1 : (x->idx > y->idx);
}

int orc_stereo_matches(const orc_params *p, const orc_keypoint *kl, const uint8_t *dl, int nl,
                       const orc_keypoint *kr, const uint8_t *dr, int nr, const uint8_t *pyr_l,
                       const uint8_t *pyr_r, int w, int h, float bf, float min_z,
                       float *uright, float *depth)
{
    const int thOrbDist = (TH_HIGH + TH_LOW) / 2;
    const int nRows = h;
    int lw[ORC_MAX_LEVELS], lh[ORC_MAX_LEVELS];
    size_t loff[ORC_MAX_LEVELS];
    size_t off = 0;
    for (int l = 0; l < p->nlevels; l++) {
        orc_level_size(p, w, h, l, &lw[l], &lh[l]);
        loff[l] = off;
        off += (size_t)lw[l] * lh[l];
    }
    for (int i = 0; i < nl; i++) {
        uright[i] = -1.0f;
        depth[i] = -1.0f;
    }
    /* row table (:637-662), rows outside the image dropped */
    int *rcount = (int *)calloc((size_t)nRows + 1, sizeof(int));
    for (int iR = 0; iR < nr; iR++) {
        const float kpY = kr[iR].y;
        const float r = 2.0f * p->scale[kr[iR].octave];
        const int maxr = (int)ceilf(kpY + r), minr = (int)floorf(kpY - r);
        for (int yi = minr; yi <= maxr; yi++)
            if (yi >= 0 && yi < nRows) rcount[yi + 1]++;
    }
    for (int y = 0; y < nRows; y++) rcount[y + 1] += rcount[y];
    int *rows = (int *)malloc(sizeof(int) * (size_t)(rcount[nRows] > 0 ? rcount[nRows] : 1));
    int *fill = (int *)malloc(sizeof(int) * (size_t)(nRows > 0 ? nRows : 1));
    memcpy(fill, rcount, sizeof(int) * (size_t)nRows);
    for (int iR = 0; iR < nr; iR++) {
        const float kpY = kr[iR].y;
        const float r = 2.0f * p->scale[kr[iR].octave];
        const int maxr = (int)ceilf(kpY + r), minr = (int)floorf(kpY - r);
        for (int yi = minr; yi <= maxr; yi++)
            if (yi >= 0 && yi < nRows) rows[fill[yi]++] = iR;
    }
    const float minZ = min_z;
    const float minD = 0;
    const float maxD = minZ > 0 ? bf / minZ : INFINITY;
    dist_idx *vd = (dist_idx *)malloc(sizeof(dist_idx) * (size_t)(nl > 0 ? nl : 1));
    int nv = 0;
    for (int iL = 0; iL < nl; iL++) {
        const int levelL = kl[iL].octave;
        const float vL = kl[iL].y, uL = kl[iL].x;
        const int row = (int)vL;
        if (row < 0 || row >= nRows) continue;
        const int c0 = rcount[row], c1 = rcount[row + 1];
        if (c0 == c1) continue;
        const float minU = uL - maxD, maxU = uL - minD;
        if (maxU < 0) continue;
        int bestDist = TH_HIGH, bestIdxR = 0;
        for (int c = c0; c < c1; c++) {
            const int iR = rows[c];
            if (kr[iR].octave < levelL - 1 || kr[iR].octave > levelL + 1) continue;
            const float uR = kr[iR].x;
            if (uR >= minU && uR <= maxU) {
                const int dist = orc_descriptor_distance(dl + (size_t)iL * 32, dr + (size_t)iR * 32);
                if (dist < bestDist) {
                    bestDist = dist;
                    bestIdxR = iR;
                }
            }
        }
        if (bestDist >= thOrbDist) continue;
        /* SAD refinement at the keypoint's level (:740-797) */
        const float uR0 = kr[bestIdxR].x;
        const float scaleFactor = p->inv_scale[levelL];
        const float scaleduL = roundf(kl[iL].x * scaleFactor);
        const float scaledvL = roundf(kl[iL].y * scaleFactor);
        const float scaleduR0 = roundf(uR0 * scaleFactor);
        const int W = 5, L = 5;
        const int cols = lw[levelL];
        const uint8_t *imL = pyr_l + loff[levelL], *imR = pyr_r + loff[levelL];
        const float iniu = scaleduR0 + L - W;
        const float endu = scaleduR0 + L + W + 1;
        if (iniu < 0 || endu >= cols) continue;
        const int yl = (int)scaledvL, xl = (int)scaleduL, xr = (int)scaleduR0;
        const int cl = imL[(size_t)yl * cols + xl];
        int bestSad = 0x7FFFFFFF, bestincR = 0;
        int vDists[11];
        for (int incR = -L; incR <= L; incR++) {
            const int cr = imR[(size_t)yl * cols + xr + incR];
            int sad = 0;
            for (int dy = -W; dy <= W; dy++)
                for (int dx = -W; dx <= W; dx++) {
                    const int a = imL[(size_t)(yl + dy) * cols + xl + dx] - cl;
                    const int b = imR[(size_t)(yl + dy) * cols + xr + incR + dx] - cr;
                    sad += abs(a - b);
                }
            if (sad < bestSad) {
                bestSad = sad;
                bestincR = incR;
            }
            vDists[L + incR] = sad;
        }
        if (bestincR == -L || bestincR == L) continue;
        /* parabola (:799-810) */
        const float dist1 = (float)vDists[L + bestincR - 1];
        const float dist2 = (float)vDists[L + bestincR];
        const float dist3 = (float)vDists[L + bestincR + 1];
        const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
        if (deltaR < -1 || deltaR > 1) continue;
        float bestuR = p->scale[levelL] * ((float)scaleduR0 + (float)bestincR + deltaR);
        float disparity = (uL - bestuR);
        if (disparity >= minD && disparity < maxD) {
            if (disparity <= 0) {
                disparity = 0.01f;
                bestuR = (float)((double)uL - 0.01);
            }
            depth[iL] = bf / disparity;
            uright[iL] = bestuR;
            vd[nv].dist = bestSad;
            vd[nv].idx = iL;
            nv++;
        }
    }
    /* median cut (:836-851) */
    if (nv > 0) {
        qsort(vd, (size_t)nv, sizeof(dist_idx), cmp_dist_idx);
        const float median = (float)vd[nv / 2].dist;
        const float thDist = 1.5f * 1.4f * median;
        for (int i = nv - 1; i >= 0; i--) {
            if ((float)vd[i].dist < thDist) break;
            uright[vd[i].idx] = -1.0f;
            depth[vd[i].idx] = -1.0f;
        }
    }
    int nvalid = 0;
    for (int i = 0; i < nl; i++) nvalid += depth[i] > 0;
    free(rcount);
    free(rows);
    free(fill);
    free(vd);
    return nvalid;
}
