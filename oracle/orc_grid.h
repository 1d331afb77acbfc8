/* oracle/orc_grid.h -- TEST INFRASTRUCTURE ONLY (oracle-private helpers shared by
 * match_oracle.c and track_oracle.c). */
#ifndef ORC_GRID_H
#define ORC_GRID_H

#include "orb_oracle.h"

#define GRID_COLS 64
#define GRID_ROWS 48
#define HISTO_LENGTH 30

/* Frame grid (Frame::AssignFeaturesToGrid, Frame.cc:292-307): mGrid[ix][iy] = keypoint
 * indices in increasing order, cell c = ix * GRID_ROWS + iy, CSR */
typedef struct {
    int *start; /* GRID_COLS*GRID_ROWS + 1 */
    int *idx;
    float inv_w, inv_h;
    orc_bounds b;
} ogrid;

void orc_grid_build(ogrid *g, const orc_keypoint *kps, int n, const orc_bounds *b);
void orc_grid_free(ogrid *g);
/* Frame::GetFeaturesInArea (Frame.cc:421-504): candidate indices in the reference's order */
int orc_features_in_area(const ogrid *g, const orc_keypoint *kps, float x, float y, float r,
                         int minLevel, int maxLevel, int *out);
/* ORBmatcher::ComputeThreeMaxima (ORBmatcher.cc:1800-1841) */
void orc_three_maxima(const int *hsize, int *ind1, int *ind2, int *ind3);

#endif
