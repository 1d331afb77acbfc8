/*
 * oracle/bow_oracle.c -- TEST INFRASTRUCTURE ONLY (see orb_oracle.h).
 *
 * Restatement of DBoW2's TemplatedVocabulary<FORB::TDescriptor, FORB>::transform(features,
 * BowVector, FeatureVector, levelsup) (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:
 * 1127-1189, 1220-1259) for the ORB vocabulary's settings (TF_IDF weighting, L1 scoring:
 * mustNormalize -> L1), as Frame::ComputeBoW calls it (src/Frame.cc:532-539, levelsup 4):
 *   - per feature: descend from the root choosing the child with the smallest
 *     FORB::distance (strict <, first child wins ties) until a leaf; the node reached at
 *     level L - levelsup is the FeatureVector key (root if <= 0; the leaf if the descent
 *     ends above that level, where the reference reads an uninitialised NodeId);
 *   - TF / TF_IDF: BowVector::addWeight (BowVector.cpp:34-46), per word the weights of its
 *     features summed in feature order; IDF / BINARY: addIfNotExist (:50-58), the first
 *     feature's weight; stopped words (weight <= 0, or NaN) are skipped;
 *   - mustNormalize (ScoringObject.h:73-88): BowVector::normalize (BowVector.cpp:62-84) by
 *     the sum of |w| (L1) or sqrt of the sum of w^2 (L2_NORM) in word-id order; DOT_PRODUCT
 *     does not normalise, and TF weights are then divided by the word count;
 *   - FeatureVector::addFeature (FeatureVector.cpp:31-45): feature indices per node, in
 *     feature order.
 * The vocabulary is a flat node array (what loadFromTextFile builds, :1338-1420): node
 * descriptors, idf weights, word ids (-1 for inner nodes) and children as CSR.
 */
#include "orb_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

void orc_bow_word(const orc_vocab *v, const uint8_t *feat, int levelsup, int32_t *word,
                  double *weight, int32_t *nid)
{
    const int nid_level = v->L - levelsup;
    if (nid_level <= 0)
        *nid = 0;
    int final_id = 0, level = 0;
    do {
        ++level;
        const int c0 = v->child_off[final_id], c1 = v->child_off[final_id + 1];
        final_id = v->child_idx[c0];
        int best_d = orc_descriptor_distance(feat, v->desc + (size_t)final_id * 32);
        for (int c = c0 + 1; c < c1; c++) {
            const int id = v->child_idx[c];
            const int d = orc_descriptor_distance(feat, v->desc + (size_t)id * 32);
            if (d < best_d) {
                best_d = d;
                final_id = id;
            }
        }
        if (level == nid_level)
            *nid = final_id;
    } while (v->child_off[final_id + 1] > v->child_off[final_id]);
    /* A leaf above nid_level leaves *nid unwritten in the reference (the caller's
     * uninitialised NodeId: undefined, never reached with ORBvoc.txt's full tree); pinned
     * here to the leaf itself. */
    if (level < nid_level)
        *nid = final_id;
    *word = v->word_id[final_id];
    *weight = v->weight[final_id];
}

static int cmp_pair(const void *a, const void *b)
{
    const int64_t x = *(const int64_t *)a, y = *(const int64_t *)b;
    return x < y ? -1 : x > y;
}

int orc_bow_transform(const orc_vocab *v, const uint8_t *desc, int n, int levelsup,
                      int32_t *bow_words, double *bow_weights, int *nbow, int32_t *fv_nodes,
                      int32_t *fv_off, int32_t *fv_feats, int *nfv)
{
    *nbow = 0;
    *nfv = 0;
    fv_off[0] = 0;
    if (v->nwords == 0 || n <= 0)  /* TemplatedVocabulary::empty() */
        return 0;
    const int nn = n;
    int32_t *w = (int32_t *)malloc(sizeof(int32_t) * nn);
    int32_t *nd = (int32_t *)malloc(sizeof(int32_t) * nn);
    double *wt = (double *)malloc(sizeof(double) * nn);
    int64_t *pw = (int64_t *)malloc(sizeof(int64_t) * nn);
    int64_t *pn = (int64_t *)malloc(sizeof(int64_t) * nn);
    int m = 0;
    for (int i = 0; i < n; i++) {
        orc_bow_word(v, desc + (size_t)i * 32, levelsup, &w[i], &wt[i], &nd[i]);
        if (wt[i] > 0) {  /* not stopped */
            pw[m] = ((int64_t)(uint32_t)w[i] << 32) | i;
            pn[m] = ((int64_t)(uint32_t)nd[i] << 32) | i;
            m++;
        }
    }
    /* std::map<WordId, ...> / std::map<NodeId, ...>: ascending unsigned ids */
    qsort(pw, m, sizeof(int64_t), cmp_pair);
    qsort(pn, m, sizeof(int64_t), cmp_pair);
    const int tf = v->weighting == ORC_TF_IDF || v->weighting == ORC_TF;
    int nb = 0;
    for (int k = 0; k < m; k++) {
        const int32_t word = (int32_t)(pw[k] >> 32), f = (int32_t)(pw[k] & 0xFFFFFFFF);
        if (nb > 0 && bow_words[nb - 1] == word) {
            if (tf)  /* addWeight; IDF / BINARY: addIfNotExist keeps the first */
                bow_weights[nb - 1] += wt[f];
        } else {
            bow_words[nb] = word;
            bow_weights[nb] = wt[f];
            nb++;
        }
    }
    /* mustNormalize: every scoring but DOT_PRODUCT; L2 for L2_NORM, L1 otherwise */
    const int must = v->scoring != ORC_DOT_PRODUCT;
    if (tf && nb > 0 && !must) {
        const double cnt = nb;
        for (int k = 0; k < nb; k++)
            bow_weights[k] /= cnt;
    }
    if (must) {
        double norm = 0.0;
        if (v->scoring == ORC_L2_NORM) {
            for (int k = 0; k < nb; k++)
                norm += bow_weights[k] * bow_weights[k];
            norm = sqrt(norm);
        } else {
            for (int k = 0; k < nb; k++)
                norm += fabs(bow_weights[k]);
        }
        if (norm > 0.0)
            for (int k = 0; k < nb; k++)
                bow_weights[k] /= norm;
    }
    int nf = 0;
    for (int k = 0; k < m; k++) {
        const int32_t node = (int32_t)(pn[k] >> 32);
        if (!(nf > 0 && fv_nodes[nf - 1] == node)) {
            fv_nodes[nf] = node;
            fv_off[nf + 1] = fv_off[nf];
            nf++;
        }
        fv_feats[fv_off[nf]++] = (int32_t)(pn[k] & 0xFFFFFFFF);
    }
    *nbow = nb;
    *nfv = nf;
    free(w);
    free(nd);
    free(wt);
    free(pw);
    free(pn);
    return m;
}

/*
 * ORBmatcher::SearchByBoW(KeyFrame *pKF, Frame &F, vector<MapPoint*> &vpMapPointMatches)
 * (src/ORBmatcher.cc:195-348; callers Tracking::TrackReferenceKeyFrame Tracking.cc:1069 and
 * Tracking::Relocalization :2009).  The two FeatureVectors (ascending node ids, per node the
 * feature indices in feature order) are walked as the reference walks its std::maps: equal
 * ids are matched, the smaller side jumps to lower_bound of the other's id -- a merge join.
 * Per common node, in the KF node's feature order: a KF feature whose MapPoint is NULL or bad
 * (kf_valid[i] == 0) is skipped; otherwise best / second over the node's F features not yet
 * matched in this call (bestDist1 = bestDist2 = 256, strict <, the first best wins ties); a
 * match needs bestDist1 <= TH_LOW and (float)bestDist1 < nnratio * (float)bestDist2.  With
 * check_ori the rotation kp.angle (KF mvKeysUn) - F.mvKeys[best].angle bins as
 * SearchForInitialization's, and every match outside ComputeThreeMaxima's bins is dropped.
 * match[i] (F feature i) = the KF feature index whose MapPoint matched it, -1 if none.
 */
#define BOW_TH_LOW 50

int orc_search_by_bow(const uint8_t *kf_desc, const float *kf_angle, const uint8_t *kf_valid,
                      int n_kf, const int32_t *kf_nodes, const int32_t *kf_off,
                      const int32_t *kf_feats, int kf_nfv, const uint8_t *f_desc,
                      const float *f_angle, int n_f, const int32_t *f_nodes, const int32_t *f_off,
                      const int32_t *f_feats, int f_nfv, float nnratio, int check_ori,
                      int32_t *match)
{
    (void)n_kf;
    for (int i = 0; i < n_f; i++) match[i] = -1;
    int *bins = (int *)malloc(sizeof(int) * (n_f > 0 ? n_f : 1));
    int hsize[30] = {0};
    const float factor = 1.0f / 30;
    int nmatches = 0;
    int a = 0, b = 0;
    while (a < kf_nfv && b < f_nfv) {
        if (kf_nodes[a] == f_nodes[b]) {
            for (int ik = kf_off[a]; ik < kf_off[a + 1]; ik++) {
                const int realKF = kf_feats[ik];
                if (!kf_valid[realKF]) continue;
                const uint8_t *dKF = kf_desc + (size_t)realKF * 32;
                int best1 = 256, bestIdx = -1, best2 = 256;
                for (int jf = f_off[b]; jf < f_off[b + 1]; jf++) {
                    const int realF = f_feats[jf];
                    if (match[realF] >= 0) continue;
                    const int d = orc_descriptor_distance(dKF, f_desc + (size_t)realF * 32);
                    if (d < best1) {
                        best2 = best1;
                        best1 = d;
                        bestIdx = realF;
                    } else if (d < best2) {
                        best2 = d;
                    }
                }
                if (best1 <= BOW_TH_LOW && (float)best1 < nnratio * (float)best2) {
                    match[bestIdx] = realKF;
                    if (check_ori) {
                        float rot = kf_angle[realKF] - f_angle[bestIdx];
                        if (rot < 0.0)
                            rot += 360.0f;
                        int bin = (int)roundf(rot * factor);
                        if (bin == 30)
                            bin = 0;
                        bins[bestIdx] = bin;
                        hsize[bin]++;
                    }
                    nmatches++;
                }
            }
            a++;
            b++;
        } else if (kf_nodes[a] < f_nodes[b]) {
            a++;
        } else {
            b++;
        }
    }
    if (check_ori) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        orc_three_maxima(hsize, &ind1, &ind2, &ind3);
        for (int i = 0; i < n_f; i++)
            if (match[i] >= 0 && bins[i] != ind1 && bins[i] != ind2 && bins[i] != ind3) {
                match[i] = -1;
                nmatches--;
            }
    }
    free(bins);
    return nmatches;
}

/* ORBmatcher::SearchByBoW(KeyFrame *pKF1, KeyFrame *pKF2, vector<MapPoint*> &vpMatches12)
 * (src/ORBmatcher.cc:634-769): KF1 features with a good MapPoint (valid1) against the KF2
 * features of the same node with a good MapPoint (valid2) not yet matched (vbMatched2);
 * best / second by strict <, accepted when bestDist1 < TH_LOW (strict, unlike the
 * KeyFrame-Frame form's <=) and the float ratio test; rotation histogram over
 * mvKeysUn[idx1].angle - mvKeysUn[idx2].angle.  match12[n1] = the KF2 feature matched to KF1
 * feature i (vpMatches12[i] = vpMapPoints2[match12[i]]), -1 if NULL. */
int orc_search_by_bow_kf(const uint8_t *desc1, const float *angle1, const uint8_t *valid1,
                         int n1, const int32_t *nodes1, const int32_t *off1,
                         const int32_t *feats1, int nfv1, const uint8_t *desc2,
                         const float *angle2, const uint8_t *valid2, int n2,
                         const int32_t *nodes2, const int32_t *off2, const int32_t *feats2,
                         int nfv2, float nnratio, int check_ori, int32_t *match12)
{
    for (int i = 0; i < n1; i++) match12[i] = -1;
    uint8_t *matched2 = (uint8_t *)calloc(n2 > 0 ? n2 : 1, 1);
    int *bins = (int *)malloc(sizeof(int) * (n1 > 0 ? n1 : 1));
    int hsize[30] = {0};
    const float factor = 1.0f / 30;
    int nmatches = 0;
    int a = 0, b = 0;
    while (a < nfv1 && b < nfv2) {
        if (nodes1[a] == nodes2[b]) {
            for (int i1 = off1[a]; i1 < off1[a + 1]; i1++) {
                const int idx1 = feats1[i1];
                if (!valid1[idx1]) continue;
                const uint8_t *d1 = desc1 + (size_t)idx1 * 32;
                int best1 = 256, bestIdx2 = -1, best2 = 256;
                for (int i2 = off2[b]; i2 < off2[b + 1]; i2++) {
                    const int idx2 = feats2[i2];
                    if (matched2[idx2] || !valid2[idx2]) continue;
                    const int d = orc_descriptor_distance(d1, desc2 + (size_t)idx2 * 32);
                    if (d < best1) {
                        best2 = best1;
                        best1 = d;
                        bestIdx2 = idx2;
                    } else if (d < best2) {
                        best2 = d;
                    }
                }
                if (best1 < BOW_TH_LOW && (float)best1 < nnratio * (float)best2) {
                    match12[idx1] = bestIdx2;
                    matched2[bestIdx2] = 1;
                    if (check_ori) {
                        float rot = angle1[idx1] - angle2[bestIdx2];
                        if (rot < 0.0)
                            rot += 360.0f;
                        int bin = (int)roundf(rot * factor);
                        if (bin == 30)
                            bin = 0;
                        bins[idx1] = bin;
                        hsize[bin]++;
                    }
                    nmatches++;
                }
            }
            a++;
            b++;
        } else if (nodes1[a] < nodes2[b]) {
            a++;
        } else {
            b++;
        }
    }
    if (check_ori) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        orc_three_maxima(hsize, &ind1, &ind2, &ind3);
        for (int i = 0; i < n1; i++)
            if (match12[i] >= 0 && bins[i] != ind1 && bins[i] != ind2 && bins[i] != ind3) {
                match12[i] = -1;
                nmatches--;
            }
    }
    free(bins);
    free(matched2);
    return nmatches;
}
