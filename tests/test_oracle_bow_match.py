"""CPU: the SearchByBoW oracle (oracle/bow_oracle.c orc_search_by_bow) against a second,
pure-Python restatement of ORBmatcher::SearchByBoW(KeyFrame*, Frame&, ...)
(src/ORBmatcher.cc:195-348, ComputeThreeMaxima :1800-1841) written line by line from the
reference's loop (std::map iteration with lower_bound jumps, the taken-F skip, strict < best
/ second, TH_LOW, the float ratio test, round() of the float rotation), and a hand-made
known-answer case for each rule.  The reference cannot run here (OpenCV / DBoW2 absent), so
these two restatements pin each other; the GPU is checked against the C one.
"""
import math

import numpy as np
import pytest

TH_LOW = 50


def _dist(a, b):
    return int(np.unpackbits(np.bitwise_xor(a, b)).sum())


def py_search_by_bow(kf_desc, kf_angle, kf_valid, kf_fv, f_desc, f_angle, f_fv, nnratio,
                     check_ori):
    kn, ko, kfe = kf_fv
    fn, fo, ffe = f_fv
    kmap = {int(kn[j]): [int(x) for x in kfe[ko[j]:ko[j + 1]]] for j in range(len(kn))}
    fmap = {int(fn[j]): [int(x) for x in ffe[fo[j]:fo[j + 1]]] for j in range(len(fn))}
    kkeys, fkeys = sorted(kmap), sorted(fmap)
    matches = [None] * len(f_desc)
    rot_hist = [[] for _ in range(30)]
    factor = np.float32(1.0) / np.float32(30)
    nmatches = 0
    a = b = 0
    while a < len(kkeys) and b < len(fkeys):
        if kkeys[a] == fkeys[b]:
            for real_kf in kmap[kkeys[a]]:
                if not kf_valid[real_kf]:
                    continue
                best1, best_idx, best2 = 256, -1, 256
                for real_f in fmap[fkeys[b]]:
                    if matches[real_f] is not None:
                        continue
                    d = _dist(kf_desc[real_kf], f_desc[real_f])
                    if d < best1:
                        best2, best1, best_idx = best1, d, real_f
                    elif d < best2:
                        best2 = d
                if best1 <= TH_LOW and np.float32(best1) < np.float32(nnratio) * np.float32(best2):
                    matches[best_idx] = real_kf
                    if check_ori:
                        rot = np.float32(kf_angle[real_kf]) - np.float32(f_angle[best_idx])
                        if rot < 0.0:
                            rot = np.float32(rot + np.float32(360.0))
                        x = float(np.float32(rot * factor))
                        b_ = int(math.floor(x + 0.5)) if x >= 0 else -int(math.floor(-x + 0.5))
                        if b_ == 30:
                            b_ = 0
                        rot_hist[b_].append(best_idx)
                    nmatches += 1
            a += 1
            b += 1
        elif kkeys[a] < fkeys[b]:
            a = next((i for i in range(a, len(kkeys)) if kkeys[i] >= fkeys[b]), len(kkeys))
        else:
            b = next((i for i in range(b, len(fkeys)) if fkeys[i] >= kkeys[a]), len(fkeys))
    if check_ori:
        m1 = m2 = m3 = 0
        i1 = i2 = i3 = -1
        for i in range(30):
            s = len(rot_hist[i])
            if s > m1:
                m3, m2, m1, i3, i2, i1 = m2, m1, s, i2, i1, i
            elif s > m2:
                m3, m2, i3, i2 = m2, s, i2, i
            elif s > m3:
                m3, i3 = s, i
        if m2 < np.float32(0.1) * np.float32(m1):
            i2 = i3 = -1
        elif m3 < np.float32(0.1) * np.float32(m1):
            i3 = -1
        for i in range(30):
            if i in (i1, i2, i3):
                continue
            for j in rot_hist[i]:
                matches[j] = None
                nmatches -= 1
    return nmatches, np.array([-1 if m is None else m for m in matches], np.int32)


def _fv(n, nodes_pool, rng):
    """A FeatureVector of n features: node ids ascending, feature lists ascending."""
    node_of = rng.choice(nodes_pool, size=n)
    nodes = np.unique(node_of).astype(np.int32)
    off = [0]
    feats = []
    for nd in nodes:
        f = np.nonzero(node_of == nd)[0]
        feats.extend(f.tolist())
        off.append(len(feats))
    return nodes, np.array(off, np.int32), np.array(feats, np.int32)


def _case(seed, n_kf=120, n_f=110, pool=12, noise=6):
    rng = np.random.default_rng(seed)
    base = rng.integers(0, 256, (n_f, 32), dtype=np.uint8)
    f_desc = base.copy()
    # KF descriptors: noisy copies of F features (some far away), duplicates for ties
    src = rng.integers(0, n_f, n_kf)
    kf_desc = base[src].copy()
    bits = rng.integers(0, 256, (n_kf, noise), dtype=np.uint8)
    kf_desc[:, :noise] ^= bits & rng.integers(0, 2, (n_kf, noise), dtype=np.uint8)
    far = rng.random(n_kf) < 0.2
    kf_desc[far] = rng.integers(0, 256, (far.sum(), 32), dtype=np.uint8)
    kf_angle = rng.uniform(0, 360, n_kf).astype(np.float32)
    f_angle = (kf_angle[rng.integers(0, n_kf, n_f)] + rng.normal(0, 8, n_f)).astype(np.float32) % 360
    kf_valid = (rng.random(n_kf) > 0.15).astype(np.uint8)
    nodes_pool = np.arange(100, 100 + pool * 3, 3)
    return (kf_desc, kf_angle, kf_valid, _fv(n_kf, nodes_pool, rng), f_desc,
            f_angle.astype(np.float32), _fv(n_f, nodes_pool, rng))


@pytest.mark.parametrize("seed", range(12))
@pytest.mark.parametrize("nnratio,check_ori", [(0.75, True), (0.7, False), (0.9, True)])
def test_oracle_equals_python_restatement(oracle, seed, nnratio, check_ori):
    c = _case(seed)
    got = oracle.search_by_bow(*c, nnratio=nnratio, check_ori=check_ori)
    ref = py_search_by_bow(*c, nnratio=nnratio, check_ori=check_ori)
    assert got[0] == ref[0]
    assert np.array_equal(got[1], ref[1])


def _flip(d, k, rng):
    """d with exactly k distinct bits flipped."""
    bits = np.unpackbits(d.copy())
    idx = rng.choice(256, k, replace=False)
    bits[idx] ^= 1
    return np.packbits(bits)


def test_known_answers(oracle):
    """One node, the reference's rules case by case, in the node's KF order:
    KF0 = F1 exactly: takes F1; KF1 = F1 with 10 bits flipped: F1 is taken, the rest are far
    (> TH_LOW): no match; KF2 = F0 exactly but without a valid MapPoint: skipped; KF3 = F5 with
    51 bits flipped: rejected (TH_LOW = 50); KF4 = F5 with 50 flipped: taken (the boundary);
    KF5 = F2 = F3 (a tie at 0): best == second fails the ratio; KF6 = F4 with 5 flipped: F4."""
    rng = np.random.default_rng(11)
    f_desc = rng.integers(0, 256, (6, 32), dtype=np.uint8)
    f_desc[3] = f_desc[2]
    kf_desc = np.stack([f_desc[1], _flip(f_desc[1], 10, rng), f_desc[0],
                        _flip(f_desc[5], 51, rng), _flip(f_desc[5], 50, rng), f_desc[2],
                        _flip(f_desc[4], 5, rng)])
    for i, j in ((1, 0), (1, 2), (1, 4), (1, 5), (3, 0), (3, 4), (4, 0), (6, 0)):
        assert _dist(kf_desc[i], f_desc[j]) > 80  # far from every non-target feature
    kf_valid = np.array([1, 1, 0, 1, 1, 1, 1], np.uint8)
    angle_kf = np.zeros(7, np.float32)
    angle_f = np.zeros(6, np.float32)
    fv_kf = (np.array([7], np.int32), np.array([0, 7], np.int32), np.arange(7, dtype=np.int32))
    fv_f = (np.array([7], np.int32), np.array([0, 6], np.int32), np.arange(6, dtype=np.int32))
    n, m = oracle.search_by_bow(kf_desc, angle_kf, kf_valid, fv_kf, f_desc, angle_f, fv_f,
                                nnratio=0.75, check_ori=True)
    assert m.tolist() == [-1, 0, -1, -1, 6, 4] and n == 3
    ref = py_search_by_bow(kf_desc, angle_kf, kf_valid, fv_kf, f_desc, angle_f, fv_f, 0.75, True)
    assert ref[0] == n and np.array_equal(ref[1], m)
    # a node on one side only matches nothing
    fv_f2 = (np.array([9], np.int32), fv_f[1], fv_f[2])
    n2, m2 = oracle.search_by_bow(kf_desc, angle_kf, kf_valid, fv_kf, f_desc, angle_f, fv_f2)
    assert n2 == 0 and (m2 == -1).all()


def test_rotation_filter_drops_minor_bins(oracle):
    """Matches in a bin below 10% of the largest are dropped by ComputeThreeMaxima."""
    rng = np.random.default_rng(5)
    n = 60
    f_desc = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    kf_desc = f_desc.copy()
    kf_angle = np.full(n, 10.0, np.float32)
    f_angle = np.zeros(n, np.float32)
    f_angle[:3] = 200.0                        # 3 matches rotated by -190 -> bin 6 (170 deg)
    fv = (np.array([1], np.int32), np.array([0, n], np.int32), np.arange(n, dtype=np.int32))
    n_ori, m_ori = oracle.search_by_bow(kf_desc, kf_angle, None, fv, f_desc, f_angle, fv,
                                        nnratio=0.75, check_ori=True)
    n_all, _ = oracle.search_by_bow(kf_desc, kf_angle, None, fv, f_desc, f_angle, fv,
                                    nnratio=0.75, check_ori=False)
    assert n_all == n and n_ori == n - 3
    assert (m_ori[:3] == -1).all() and (m_ori[3:] == np.arange(3, n)).all()


# ------------------------------------------- SearchByBoW(KeyFrame*, KeyFrame*, vpMatches12)
def py_search_by_bow_kf(d1, a1, v1, fv1, d2, a2, v2, fv2, nnratio, check_ori):
    """ORBmatcher.cc:634-769 line by line: KF1's good MapPoints against KF2's (vbMatched2,
    strict < TH_LOW)."""
    n1_, o1_, f1_ = fv1
    n2_, o2_, f2_ = fv2
    m1 = {int(n1_[j]): [int(x) for x in f1_[o1_[j]:o1_[j + 1]]] for j in range(len(n1_))}
    m2 = {int(n2_[j]): [int(x) for x in f2_[o2_[j]:o2_[j + 1]]] for j in range(len(n2_))}
    k1, k2 = sorted(m1), sorted(m2)
    match = [-1] * len(d1)
    matched2 = [False] * len(d2)
    hist = [[] for _ in range(30)]
    factor = np.float32(1.0) / np.float32(30)
    nm = 0
    a = b = 0
    while a < len(k1) and b < len(k2):
        if k1[a] == k2[b]:
            for i1 in m1[k1[a]]:
                if not v1[i1]:
                    continue
                b1, bi, b2 = 256, -1, 256
                for i2 in m2[k2[b]]:
                    if matched2[i2] or not v2[i2]:
                        continue
                    d = _dist(d1[i1], d2[i2])
                    if d < b1:
                        b2, b1, bi = b1, d, i2
                    elif d < b2:
                        b2 = d
                if b1 < TH_LOW and np.float32(b1) < np.float32(nnratio) * np.float32(b2):
                    match[i1] = bi
                    matched2[bi] = True
                    if check_ori:
                        rot = np.float32(a1[i1]) - np.float32(a2[bi])
                        if rot < 0.0:
                            rot = np.float32(rot + np.float32(360.0))
                        x = float(np.float32(rot * factor))
                        bb = int(math.floor(x + 0.5))
                        hist[0 if bb == 30 else bb].append(i1)
                    nm += 1
            a += 1
            b += 1
        elif k1[a] < k2[b]:
            a += 1
        else:
            b += 1
    if check_ori:
        s_ = [len(h) for h in hist]
        mx1 = mx2 = mx3 = 0
        j1 = j2 = j3 = -1
        for i in range(30):
            if s_[i] > mx1:
                mx3, mx2, mx1, j3, j2, j1 = mx2, mx1, s_[i], j2, j1, i
            elif s_[i] > mx2:
                mx3, mx2, j3, j2 = mx2, s_[i], j2, i
            elif s_[i] > mx3:
                mx3, j3 = s_[i], i
        if mx2 < np.float32(0.1) * np.float32(mx1):
            j2 = j3 = -1
        elif mx3 < np.float32(0.1) * np.float32(mx1):
            j3 = -1
        for i in range(30):
            if i not in (j1, j2, j3):
                for j in hist[i]:
                    match[j] = -1
                    nm -= 1
    return nm, np.array(match, np.int32)


def kf_case(seed):
    """a KeyFrame-KeyFrame pair: _case's KF as KF1, its F side as KF2 with MapPoint flags"""
    kd, ka, kv, kfv, fd, fa, ffv = _case(seed)
    rng = np.random.default_rng(seed + 100)
    fv_ = (rng.random(len(fd)) > 0.2).astype(np.uint8)
    return kd, ka, kv, kfv, fd, fa, fv_, ffv


@pytest.mark.parametrize("seed", range(12))
@pytest.mark.parametrize("nnratio,check_ori", [(0.75, True), (0.6, False), (0.9, True)])
def test_kf_oracle_equals_python_restatement(oracle, seed, nnratio, check_ori):
    c = kf_case(seed)
    got = oracle.search_by_bow_kf(*c, nnratio=nnratio, check_ori=check_ori)
    ref = py_search_by_bow_kf(*c, nnratio=nnratio, check_ori=check_ori)
    assert got[0] == ref[0] and np.array_equal(got[1], ref[1])
    assert got[0] > 0


def test_kf_known_answers(oracle):
    """KF-KF rules: strict < TH_LOW (50 rejected, 49 taken), KF2 features without a good
    MapPoint are no candidates, a taken KF2 feature is skipped by the next KF1 feature."""
    rng = np.random.default_rng(3)
    d2 = rng.integers(0, 256, (5, 32), dtype=np.uint8)
    d1 = np.stack([_flip(d2[0], 50, rng), _flip(d2[0], 49, rng), d2[1], d2[2], d2[2]])
    for i, j in ((0, 1), (0, 2), (0, 3), (0, 4), (1, 1), (1, 2), (1, 3), (1, 4)):
        assert _dist(d1[i], d2[j]) > 80
    v1 = np.ones(5, np.uint8)
    v2 = np.array([1, 0, 1, 1, 1], np.uint8)   # KF2 feature 1: no good MapPoint
    fv1 = (np.array([4], np.int32), np.array([0, 5], np.int32), np.arange(5, dtype=np.int32))
    fv2 = (np.array([4], np.int32), np.array([0, 5], np.int32), np.arange(5, dtype=np.int32))
    z1, z2 = np.zeros(5, np.float32), np.zeros(5, np.float32)
    n, m = oracle.search_by_bow_kf(d1, z1, v1, fv1, d2, z2, v2, fv2, 0.75, True)
    # 0: 50 bits (rejected); 1: 49 bits -> KF2 0; 2: KF2 1 invalid, the rest far -> none;
    # 3: KF2 2 exactly; 4: KF2 2 taken, the rest far -> none
    assert m.tolist() == [-1, 0, -1, 2, -1] and n == 2
    assert py_search_by_bow_kf(d1, z1, v1, fv1, d2, z2, v2, fv2, 0.75, True)[0] == 2
