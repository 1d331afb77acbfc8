"""ORBVocabulary -- DBoW2's TemplatedVocabulary<FORB::TDescriptor, FORB> (include/ORBVocabulary.h)
for the part the tracking hot path calls: loadFromTextFile and transform(features, BowVector,
FeatureVector, levelsup) (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1126-1189, 1220-1259,
1337-1420), as Frame::ComputeBoW uses it (src/Frame.cc:532-539, levelsup 4).

The tree lives in HBM (one 64-byte record per tree edge, see bow_kernels.hip); transform runs
the descent and the BowVector / FeatureVector assembly on the GPU through liborbg
(orbg_vocab_* / orbg_bow_transform*).  Results are bit-identical to the reference, the
normalised double weights included.

    voc = ORBVocabulary()
    voc.loadFromTextFile("ORBvoc.txt")
    bow, feat = voc.transform(descriptors, 4)   # Frame::ComputeBoW
    bow   -> BowVector: dict word id -> weight, ascending word ids
    feat  -> FeatureVector: dict node id -> list of feature indices, ascending
"""
import ctypes as C

import numpy as np

from . import _lib as L
from .orbmatcher import _ctx

TF_IDF, TF, IDF, BINARY = 0, 1, 2, 3                                   # BowVector.h:36-42
L1_NORM, L2_NORM, CHI_SQUARE, KL, BHATTACHARYYA, DOT_PRODUCT = range(6)  # BowVector.h:45-53


class BowVector(dict):
    """std::map<WordId, WordValue> (BowVector.h:56); iteration in ascending word id."""


class FeatureVector(dict):
    """std::map<NodeId, std::vector<unsigned int>> (FeatureVector.h:24)."""


class ORBVocabulary:
    def __init__(self, device=0):
        self.device = device
        self._h = None

    # ---- construction ----
    def loadFromTextFile(self, path):
        """TemplatedVocabulary::loadFromTextFile; returns False for a malformed file
        (the reference's bool), raising nothing."""
        self._free()
        h = C.c_void_p()
        rc = L.lib().orbg_vocab_load_text(_ctx(self.device).handle, str(path).encode(), C.byref(h))
        if rc != L.ORBG_OK:
            return False
        self._h = h
        return True

    @classmethod
    def from_tree(cls, k, L_, scoring, weighting, parent, is_leaf, desc, weight, device=0):
        """The tree as loadFromTextFile builds it: node 0 is the root, parent[i] < i."""
        v = cls(device)
        parent = np.ascontiguousarray(parent, np.int32)
        is_leaf = np.ascontiguousarray(is_leaf, np.uint8)
        desc = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        weight = np.ascontiguousarray(weight, np.float64)
        h = C.c_void_p()
        L.check(L.lib().orbg_vocab_create(_ctx(device).handle, k, L_, scoring, weighting,
                                          len(parent), L.ptr(parent), L.ptr(is_leaf),
                                          L.ptr(desc), L.ptr(weight), C.byref(h)),
                "orbg_vocab_create")
        v._h = h
        return v

    def _free(self):
        if self._h is not None and self._h.value:
            L.lib().orbg_vocab_destroy(self._h)
        self._h = None

    def __del__(self):
        try:
            self._free()
        except Exception:
            pass

    # ---- TemplatedVocabulary accessors ----
    def _info(self):
        if self._h is None:
            raise RuntimeError("vocabulary not loaded")
        v = [C.c_int32() for _ in range(6)]
        L.check(L.lib().orbg_vocab_info(self._h, *[C.byref(x) for x in v]), "orbg_vocab_info")
        return [x.value for x in v]

    def getBranchingFactor(self):
        return self._info()[0]

    def getDepthLevels(self):
        return self._info()[1]

    def getScoringType(self):
        return self._info()[2]

    def getWeightingType(self):
        return self._info()[3]

    def size(self):
        """number of words"""
        return self._info()[5]

    def empty(self):
        return self.size() == 0

    @property
    def handle(self):
        if self._h is None:
            raise RuntimeError("vocabulary not loaded")
        return self._h

    # ---- transform ----
    def transform_arrays(self, descriptors, levelsup=4):
        """(bow_words, bow_weights, fv_nodes, fv_off, fv_feats) as flat arrays."""
        d = np.ascontiguousarray(descriptors, np.uint8).reshape(-1, 32)
        n = len(d)
        cap = max(n, 1)
        bw = np.zeros(cap, np.int32)
        bx = np.zeros(cap, np.float64)
        vn = np.zeros(cap, np.int32)
        vo = np.zeros(cap + 1, np.int32)
        vf = np.zeros(cap, np.int32)
        nb, nf = C.c_int(), C.c_int()
        L.check(L.lib().orbg_bow_transform(_ctx(self.device).handle, self.handle, L.ptr(d), n,
                                           levelsup, L.ptr(bw), L.ptr(bx), C.byref(nb),
                                           L.ptr(vn), L.ptr(vo), L.ptr(vf), C.byref(nf)),
                "orbg_bow_transform")
        nb, nf = nb.value, nf.value
        return bw[:nb], bx[:nb], vn[:nf], vo[:nf + 1], vf[:vo[nf]]

    def transform(self, descriptors, levelsup=0):
        """transform(features, BowVector &v, FeatureVector &fv, levelsup) -> (v, fv)."""
        bw, bx, vn, vo, vf = self.transform_arrays(descriptors, levelsup)
        bow = BowVector(zip(bw.tolist(), bx.tolist()))
        fv = FeatureVector((int(vn[j]), vf[vo[j]:vo[j + 1]].tolist()) for j in range(len(vn)))
        return bow, fv

    def transform_batch_device(self, d_desc, d_counts, cap, nframes, levelsup, out, ctx=None):
        """Device-resident batch (orbg_bow_transform_batch_device); `out` maps the output
        names (bow_words, bow_weights, nbow, fv_nodes, fv_off, fv_feats, nfv, word_of,
        node_of) to device pointers (ints; word_of / node_of may be None)."""
        ctx = ctx if ctx is not None else _ctx(self.device)
        L.check(L.lib().orbg_bow_transform_batch_device(
            ctx.handle, self.handle, d_desc, d_counts, cap, nframes, levelsup,
            out["bow_words"], out["bow_weights"], out["nbow"], out["fv_nodes"], out["fv_off"],
            out["fv_feats"], out["nfv"], out.get("word_of"), out.get("node_of")),
            "orbg_bow_transform_batch_device")
