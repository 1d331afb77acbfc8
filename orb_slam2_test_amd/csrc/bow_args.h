// bow_args.h -- device layout and launch arguments of the DBoW2 transform (bow_kernels.hip),
// shared with the host entry points (orbg_api.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace orbg {

// One 64-byte record per tree edge, in children-CSR order: slot c is child number
// c - first_child(parent) of its parent, so a node's children are contiguous and the
// records one descent step compares are one coalesced 64 x k byte read.  Each record
// carries what the step after it needs: the child's own children range, its node id (the
// FeatureVector key), word id and weight (read only at the leaf).
struct alignas(16) BowSlot {
    uint32_t d[8];      // node descriptor (32 bytes)
    int32_t c0, c1;     // children of this node: slots [c0, c1); c0 == c1 for a leaf
    int32_t node;       // node id (TemplatedVocabulary m_nodes index)
    int32_t word;       // word id (leaves); 0 for inner nodes (Node() default)
    double weight;      // idf weight (Node::weight)
    int64_t pad;
};
static_assert(sizeof(BowSlot) == 64, "BowSlot is one 64-byte record");

struct BowArgs {
    const BowSlot *slots;
    int32_t root_c0, root_c1;   // root's children
    int32_t group;              // lanes per descriptor (16 / 32 / 64 >= max children)
    int32_t nid_level;          // L - levelsup
    int32_t scoring, weighting;
    int32_t empty;              // no words: TemplatedVocabulary::empty(), every feature dropped
    const uint8_t *desc;        // [nframes][cap][32]
    const int32_t *counts;      // [nframes]
    int32_t cap, nframes;
    int32_t *fword;             // [nframes][cap] word id, -1 if stopped
    int32_t *fnode;             // [nframes][cap] FeatureVector node
    double *fweight;            // [nframes][cap]
    int32_t *bow_words;         // [nframes][cap]
    double *bow_weights;
    int32_t *nbow;              // [nframes]
    int32_t *fv_nodes;          // [nframes][cap]
    int32_t *fv_off;            // [nframes][cap + 1]
    int32_t *fv_feats;          // [nframes][cap]
    int32_t *nfv;               // [nframes]
};

int launch_bow(hipStream_t st, const BowArgs &A, void *prof);
size_t bow_vectors_lds(int cap);

}  // namespace orbg
