/*
 * oracle/match_oracle.c -- TEST INFRASTRUCTURE ONLY (see orb_oracle.h).
 *
 * Plain-C restatement of ORBmatcher::DescriptorDistance (src/ORBmatcher.cc:1846-1862),
 * ORBmatcher::SearchForInitialization (:487-631) with ComputeThreeMaxima (:1800-1841),
 * and the Frame grid it searches (Frame::AssignFeaturesToGrid / PosInGrid /
 * GetFeaturesInArea, src/Frame.cc:292-307, 421-520).
 */
#include "orb_oracle.h"

#include <limits.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define TH_LOW 50    /* ORBmatcher.cc:38 */

/* bit-parallel popcount over 8 x int32, ORBmatcher.cc:1846-1862 */
int orc_descriptor_distance(const uint8_t *a, const uint8_t *b)
{
    int dist = 0;
    for (int i = 0; i < 8; i++) {
        uint32_t pa, pb;
        memcpy(&pa, a + 4 * i, 4);
        memcpy(&pb, b + 4 * i, 4);
        uint32_t v = pa ^ pb;
        v = v - ((v >> 1) & 0x55555555u);
        v = (v & 0x33333333u) + ((v >> 2) & 0x33333333u);
        dist += (int)((((v + (v >> 4)) & 0xF0F0F0Fu) * 0x1010101u) >> 24);
    }
    return dist;
}

/* brute-force 2-NN with the matcher loops' strict-< update rule (first index wins ties) */
void orc_knn2(const uint8_t *qdesc, int nq, const uint8_t *tdesc, int nt, int32_t *best_idx,
              int32_t *best_dist, int32_t *second_dist)
{
    for (int i = 0; i < nq; i++) {
        int b = INT_MAX, b2 = INT_MAX, bi = -1;
        for (int j = 0; j < nt; j++) {
            const int d = orc_descriptor_distance(qdesc + (size_t)i * 32, tdesc + (size_t)j * 32);
            if (d < b) {
                b2 = b;
                b = d;
                bi = j;
            } else if (d < b2) {
                b2 = d;
            }
        }
        best_idx[i] = bi;
        best_dist[i] = b;
        second_dist[i] = b2;
    }
}

#include "orc_grid.h"

static int pos_in_grid(const ogrid *g, const orc_keypoint *kp, int *px, int *py)
{
    /* Frame::PosInGrid, Frame.cc:510-520: round() of float */
    *px = (int)roundf((kp->x - g->b.min_x) * g->inv_w);
    *py = (int)roundf((kp->y - g->b.min_y) * g->inv_h);
    return !(*px < 0 || *px >= GRID_COLS || *py < 0 || *py >= GRID_ROWS);
}

void orc_grid_build(ogrid *g, const orc_keypoint *kps, int n, const orc_bounds *b)
{
    g->b = *b;
    /* Frame.cc:273-274 */
    g->inv_w = (float)GRID_COLS / (float)(b->max_x - b->min_x);
    g->inv_h = (float)GRID_ROWS / (float)(b->max_y - b->min_y);
    const int ncell = GRID_COLS * GRID_ROWS;
    g->start = (int *)calloc(ncell + 1, sizeof(int));
    g->idx = (int *)malloc(sizeof(int) * (n > 0 ? n : 1));
    int *cell = (int *)malloc(sizeof(int) * (n > 0 ? n : 1));
    for (int i = 0; i < n; i++) {
        int px, py;
        cell[i] = pos_in_grid(g, &kps[i], &px, &py) ? px * GRID_ROWS + py : -1;
        if (cell[i] >= 0)
            g->start[cell[i] + 1]++;
    }
    for (int c = 0; c < ncell; c++)
        g->start[c + 1] += g->start[c];
    int *fill = (int *)malloc(sizeof(int) * ncell);
    memcpy(fill, g->start, sizeof(int) * ncell);
    for (int i = 0; i < n; i++)
        if (cell[i] >= 0)
            g->idx[fill[cell[i]]++] = i;
    free(fill);
    free(cell);
}

void orc_grid_free(ogrid *g)
{
    free(g->start);
    free(g->idx);
}

/* Frame::GetFeaturesInArea, Frame.cc:421-504 */
int orc_features_in_area(const ogrid *g, const orc_keypoint *kps, float x, float y, float r,
                            int minLevel, int maxLevel, int *out)
{
    int n = 0;
    const int nMinCellX = (int)floorf((x - g->b.min_x - r) * g->inv_w) > 0
                              ? (int)floorf((x - g->b.min_x - r) * g->inv_w)
                              : 0;
    if (nMinCellX >= GRID_COLS)
        return 0;
    int nMaxCellX = (int)ceilf((x - g->b.min_x + r) * g->inv_w);
    if (nMaxCellX > GRID_COLS - 1)
        nMaxCellX = GRID_COLS - 1;
    if (nMaxCellX < 0)
        return 0;
    const int nMinCellY = (int)floorf((y - g->b.min_y - r) * g->inv_h) > 0
                              ? (int)floorf((y - g->b.min_y - r) * g->inv_h)
                              : 0;
    if (nMinCellY >= GRID_ROWS)
        return 0;
    int nMaxCellY = (int)ceilf((y - g->b.min_y + r) * g->inv_h);
    if (nMaxCellY > GRID_ROWS - 1)
        nMaxCellY = GRID_ROWS - 1;
    if (nMaxCellY < 0)
        return 0;
    const int bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
    for (int ix = nMinCellX; ix <= nMaxCellX; ix++)
        for (int iy = nMinCellY; iy <= nMaxCellY; iy++) {
            const int c = ix * GRID_ROWS + iy;
            for (int j = g->start[c]; j < g->start[c + 1]; j++) {
                const orc_keypoint *kp = &kps[g->idx[j]];
                if (bCheckLevels) {
                    if (kp->octave < minLevel)
                        continue;
                    if (maxLevel >= 0 && kp->octave > maxLevel)
                        continue;
                }
                const float distx = kp->x - x, disty = kp->y - y;
                if (fabsf(distx) < r && fabsf(disty) < r)
                    out[n++] = g->idx[j];
            }
        }
    return n;
}

/* ORBmatcher::ComputeThreeMaxima, :1800-1841 */
void orc_three_maxima(const int *hsize, int *ind1, int *ind2, int *ind3)
{
    int max1 = 0, max2 = 0, max3 = 0;
    for (int i = 0; i < HISTO_LENGTH; i++) {
        const int s = hsize[i];
        if (s > max1) {
            max3 = max2;
            max2 = max1;
            max1 = s;
            *ind3 = *ind2;
            *ind2 = *ind1;
            *ind1 = i;
        } else if (s > max2) {
            max3 = max2;
            max2 = s;
            *ind3 = *ind2;
            *ind2 = i;
        } else if (s > max3) {
            max3 = s;
            *ind3 = i;
        }
    }
    if (max2 < 0.1f * (float)max1) {
        *ind2 = -1;
        *ind3 = -1;
    } else if (max3 < 0.1f * (float)max1) {
        *ind3 = -1;
    }
}

int orc_search_for_initialization(const orc_keypoint *kps1, const uint8_t *desc1, int n1,
                                  const orc_keypoint *kps2, const uint8_t *desc2, int n2,
                                  const orc_bounds *b2, float *prev_xy, int32_t *matches12,
                                  int window, float nnratio, int check_ori)
{
    int nmatches = 0;
    ogrid g;
    orc_grid_build(&g, kps2, n2, b2);
    for (int i = 0; i < n1; i++)
        matches12[i] = -1;
    int *hist = (int *)malloc(sizeof(int) * HISTO_LENGTH * (n1 > 0 ? n1 : 1));
    int hsize[HISTO_LENGTH];
    memset(hsize, 0, sizeof(hsize));
    const float factor = 1.0f / HISTO_LENGTH;
    int *matched_dist = (int *)malloc(sizeof(int) * (n2 > 0 ? n2 : 1));
    int *matches21 = (int *)malloc(sizeof(int) * (n2 > 0 ? n2 : 1));
    for (int i = 0; i < n2; i++) {
        matched_dist[i] = INT_MAX;
        matches21[i] = -1;
    }
    int *cand = (int *)malloc(sizeof(int) * (n2 > 0 ? n2 : 1));

    for (int i1 = 0; i1 < n1; i1++) {
        const int level1 = kps1[i1].octave;
        if (level1 > 0)
            continue;
        const int nc = orc_features_in_area(&g, kps2, prev_xy[2 * i1], prev_xy[2 * i1 + 1],
                                        (float)window, level1, level1, cand);
        if (nc == 0)
            continue;
        int bestDist = INT_MAX, bestDist2 = INT_MAX, bestIdx2 = -1;
        for (int k = 0; k < nc; k++) {
            const int i2 = cand[k];
            const int dist =
                orc_descriptor_distance(desc1 + (size_t)i1 * 32, desc2 + (size_t)i2 * 32);
            if (matched_dist[i2] <= dist)
                continue;
            if (dist < bestDist) {
                bestDist2 = bestDist;
                bestDist = dist;
                bestIdx2 = i2;
            } else if (dist < bestDist2) {
                bestDist2 = dist;
            }
        }
        if (bestDist <= TH_LOW) {
            if (bestDist < (float)bestDist2 * nnratio) {
                if (matches21[bestIdx2] >= 0) {
                    matches12[matches21[bestIdx2]] = -1;
                    nmatches--;
                }
                matches12[i1] = bestIdx2;
                matches21[bestIdx2] = i1;
                matched_dist[bestIdx2] = bestDist;
                nmatches++;
                if (check_ori) {
                    float rot = kps1[i1].angle - kps2[bestIdx2].angle;
                    if (rot < 0.0)
                        rot += 360.0f;
                    int bin = (int)roundf(rot * factor);
                    if (bin == HISTO_LENGTH)
                        bin = 0;
                    hist[bin * (n1 > 0 ? n1 : 1) + hsize[bin]++] = i1;
                }
            }
        }
    }
    if (check_ori) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        orc_three_maxima(hsize, &ind1, &ind2, &ind3);
        for (int i = 0; i < HISTO_LENGTH; i++) {
            if (i == ind1 || i == ind2 || i == ind3)
                continue;
            for (int j = 0; j < hsize[i]; j++) {
                const int idx1 = hist[i * (n1 > 0 ? n1 : 1) + j];
                if (matches12[idx1] >= 0) {
                    matches12[idx1] = -1;
                    nmatches--;
                }
            }
        }
    }
    for (int i1 = 0; i1 < n1; i1++)
        if (matches12[i1] >= 0) {
            prev_xy[2 * i1] = kps2[matches12[i1]].x;
            prev_xy[2 * i1 + 1] = kps2[matches12[i1]].y;
        }
    free(hist);
    free(matched_dist);
    free(matches21);
    free(cand);
    orc_grid_free(&g);
    return nmatches;
}
