"""CPU: the DBoW2 transform oracle (oracle/bow_oracle.c) against an independent pure-Python
restatement of TemplatedVocabulary::transform (TemplatedVocabulary.h:1126-1189, 1220-1259),
BowVector::addWeight / addIfNotExist / normalize (BowVector.cpp:34-84) and
FeatureVector::addFeature (FeatureVector.cpp:31-45), plus the text format round trip.

Parity note: the reference ships no vocabulary (Vocabulary/ORBvoc.txt is a missing blob) and
no DBoW2 tests, so this row is "parity unpinned" against reference outputs; the two
restatements here are written independently (C and Python) and must agree bit for bit on
synthetic trees that exercise every rule (ties, ragged depth, stopped words, levelsup).
"""
import math

import numpy as np
import pytest

from orb_slam2_test_amd import synthetic as S


def py_transform(voc, desc, levelsup):
    parent = voc["parent"]
    n = len(parent)
    children = [[] for _ in range(n)]
    for i in range(1, n):
        children[parent[i]].append(i)
    word_id = [0] * n
    w = 0
    for i in range(1, n):
        if voc["is_leaf"][i]:
            word_id[i] = w
            w += 1
    if w == 0:
        return [], [], [], [0], []
    nd = voc["desc"]

    def dist(a, b):
        return int(np.unpackbits(np.bitwise_xor(a, b)).sum())

    bow = {}
    fv = {}
    tf = voc["weighting"] in (0, 1)
    for fi, f in enumerate(desc):
        nid_level = voc["L"] - levelsup
        nid = 0 if nid_level <= 0 else None
        final, level = 0, 0
        while True:
            level += 1
            kids = children[final]
            final = kids[0]
            best = dist(f, nd[final])
            for c in kids[1:]:
                d = dist(f, nd[c])
                if d < best:
                    best, final = d, c
            if level == nid_level:
                nid = final
            if not children[final]:
                if level < nid_level:     # reference: uninitialised NodeId; pinned to the leaf
                    nid = final
                break
        wt = float(voc["weight"][final])
        if wt > 0:
            wd = word_id[final]
            if wd in bow:
                if tf:
                    bow[wd] += wt
            else:
                bow[wd] = wt
            fv.setdefault(nid, []).append(fi)
    words = sorted(bow)
    vals = [bow[k] for k in words]
    must = voc["scoring"] != 5
    if tf and vals and not must:
        vals = [v / float(len(vals)) for v in vals]
    if must:
        if voc["scoring"] == 1:
            norm = 0.0
            for v in vals:
                norm += v * v
            norm = math.sqrt(norm)
        else:
            norm = 0.0
            for v in vals:
                norm += abs(v)
        if norm > 0:
            vals = [v / norm for v in vals]
    nodes = sorted(fv)
    off = [0]
    feats = []
    for k in nodes:
        feats += fv[k]
        off.append(len(feats))
    return words, vals, nodes, off, feats


def near_descriptors(voc, n, seed):
    """descriptors near random tree nodes (a few bits flipped) plus exact node copies"""
    rng = np.random.default_rng(seed)
    base = voc["desc"][rng.integers(1, len(voc["parent"]), n)].copy()
    flip = S._flip_mask(rng, n, 3)
    flip[rng.random(n) < 0.2] = 0
    return base ^ flip


def check(oracle, voc, desc, levelsup):
    ov = oracle.Vocab(voc["k"], voc["L"], voc["scoring"], voc["weighting"], voc["parent"],
                      voc["is_leaf"], voc["desc"], voc["weight"])
    bw, bx, vn, vo, vf = oracle.bow_transform(ov, desc, levelsup)
    pw, px, pn, po, pf = py_transform(voc, desc, levelsup)
    assert bw.tolist() == pw
    assert np.array_equal(bx, np.asarray(px, np.float64).reshape(-1))  # bit-exact doubles
    assert vn.tolist() == pn and vo.tolist() == po and vf.tolist() == pf
    return len(bw)


@pytest.mark.parametrize("scoring,weighting", [(0, 0), (1, 0), (5, 0), (5, 1), (0, 2), (2, 3),
                                               (1, 1), (5, 2)])
def test_oracle_matches_python_restatement(oracle, scoring, weighting):
    voc = S.ragged_vocabulary(k=6, L=4, seed=S.DEFAULT_SEED + scoring * 7 + weighting,
                              scoring=scoring, weighting=weighting, max_nodes=1500)
    desc = near_descriptors(voc, 300, 3)
    assert check(oracle, voc, desc, 2) > 20
    check(oracle, voc, desc, 0)              # leaves above nid_level


@pytest.mark.parametrize("levelsup", [0, 1, 4, 6, 9])
def test_levelsup(oracle, levelsup):
    voc = S.vocabulary(k=5, L=4, seed=S.DEFAULT_SEED + 1)
    check(oracle, voc, near_descriptors(voc, 200, 4), levelsup)


def test_ties_first_child_wins(oracle):
    """identical sibling descriptors: the first child (lowest node id) always wins"""
    voc = S.vocabulary(k=4, L=2, seed=5)
    voc["desc"][2] = voc["desc"][1]          # root children 1 and 2 identical
    voc["desc"][3] = voc["desc"][1]
    ov = oracle.Vocab(4, 2, 0, 0, voc["parent"], voc["is_leaf"], voc["desc"], voc["weight"])
    w, x, nid = oracle.bow_word(ov, voc["desc"][1], 1)
    assert nid == 1                      # level L - levelsup = 1 node: first of the tied
    check(oracle, voc, np.repeat(voc["desc"][1:4], 3, axis=0), 1)


def test_stopped_and_empty(oracle):
    voc = S.vocabulary(k=3, L=2, seed=6)
    voc["weight"][:] = 0.0                  # every word stopped
    assert check(oracle, voc, near_descriptors(voc, 50, 1), 1) == 0
    root = dict(k=3, L=2, scoring=0, weighting=0, parent=np.zeros(1, np.int32),
                is_leaf=np.zeros(1, np.uint8), desc=np.zeros((1, 32), np.uint8),
                weight=np.zeros(1))
    assert check(oracle, root, near_descriptors(voc, 10, 2), 1) == 0   # empty(): no words
    voc = S.vocabulary(k=3, L=2, seed=6)
    assert check(oracle, voc, np.zeros((0, 32), np.uint8), 1) == 0


def test_text_format_round_trip(tmp_path):
    """write_vocabulary_text emits saveToTextFile's layout; parsing it back the way
    loadFromTextFile does (TemplatedVocabulary.h:1376-1417) recovers the node list."""
    voc = S.ragged_vocabulary(k=5, L=3, seed=9, max_nodes=400)
    p = tmp_path / "voc.txt"
    S.write_vocabulary_text(p, voc)
    lines = p.read_text().split("\n")
    k, L_, sc, wt = map(int, lines[0].split())
    assert (k, L_, sc, wt) == (5, 3, 0, 0)
    rows = [ln.split() for ln in lines[1:] if ln.strip()]
    assert len(rows) == len(voc["parent"]) - 1
    for i, r in enumerate(rows, start=1):
        assert int(r[0]) == voc["parent"][i] and int(r[1]) == voc["is_leaf"][i]
        assert [int(v) for v in r[2:34]] == voc["desc"][i].tolist()
        assert float(r[34]) == voc["weight"][i]
