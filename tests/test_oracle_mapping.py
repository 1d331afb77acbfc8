"""CPU: the oracle's LocalMapping matchers (oracle/mapping_oracle.c) pinned against a second,
pure-Python restatement of ORBmatcher::SearchForTriangulation (src/ORBmatcher.cc:779-957,
CheckDistEpipolarLine :165-182, ComputeThreeMaxima :1800-1841) on generated KeyFrame pairs:
two cameras seeing one set of 3-D points (F12 from the poses as LocalMapping::ComputeF12,
LocalMapping.cc:690-707), noisy descriptor copies, monocular and stereo observations,
features that already carry a MapPoint, FeatureVectors with shared and private nodes, a
forward motion that puts the epipole inside the image, bOnlyStereo and checkOri both ways.
The GPU kernel is checked against this oracle in tests/test_gpu_mapping.py.
"""
import numpy as np
import pytest

KITTI_K = (718.856, 718.856, 607.1928, 185.2157)
BF = 386.1448


def _rot(rng, s):
    w = rng.normal(0, s, 3)
    th = np.linalg.norm(w)
    k = w / max(th, 1e-12)
    Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * Kx + (1 - np.cos(th)) * Kx @ Kx


def _fv(nodes_of):
    """FeatureVector of per-feature node ids: ascending nodes, features ascending."""
    order = np.lexsort((np.arange(len(nodes_of)), nodes_of))
    nodes, start = np.unique(nodes_of[order], return_index=True)
    off = np.concatenate([start, [len(order)]]).astype(np.int32)
    return nodes.astype(np.int32), off, order.astype(np.int32)


def tri_case(kp_dtype, geom_dtype, seed, n=1500, forward=False, nnodes=120, w=1241, h=376):
    """(kf1, kf2, geom, scale_factors, sigma2) for one KeyFrame pair."""
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy = KITTI_K
    K = np.array([[fx, 0, cx], [0, fy, cy], [0, 0, 1]])
    sf = (np.float32(1.2) ** np.arange(8)).astype(np.float32)
    s2 = (sf * sf).astype(np.float32)
    # KF1 at a random pose, KF2 moved by a baseline (sideways, or forward: epipole inside)
    R1w = _rot(rng, 0.2)
    t1w = rng.uniform(-20, 20, 3)
    R21 = _rot(rng, 0.03)
    base = np.array([0.0, 0.0, 1.5]) if forward else np.array([rng.uniform(0.5, 2), rng.uniform(-0.2, 0.2), rng.uniform(-0.3, 0.3)])
    t21 = -R21 @ base
    R2w = R21 @ R1w
    t2w = R21 @ t1w + t21
    # 3-D points in KF1's camera, seen by both
    z = rng.uniform(4, 45, n)
    u1 = rng.uniform(20, w - 20, n)
    v1 = rng.uniform(20, h - 20, n)
    X1 = np.stack([(u1 - cx) * z / fx, (v1 - cy) * z / fy, z], 1)
    X2 = (R21 @ X1.T).T + t21
    u2 = fx * X2[:, 0] / X2[:, 2] + cx
    v2 = fy * X2[:, 1] / X2[:, 2] + cy
    oct1 = rng.integers(0, 8, n)
    oct2 = np.clip(oct1 + rng.integers(-1, 2, n), 0, 7)
    noise = rng.normal(0, 0.7, (n, 4)) * np.sqrt(s2[oct2])[:, None]

    def kf(u, v, octv, zc, nz):
        kp = np.zeros(n, kp_dtype)
        kp["x"], kp["y"], kp["octave"] = u + nz[:, 0], v + nz[:, 1], octv
        kp["size"], kp["response"] = 31, 20
        return kp

    kp1 = kf(u1, v1, oct1, z, noise[:, :2] * 0.2)
    kp2 = kf(u2, v2, oct2, X2[:, 2], noise[:, 2:])
    a1 = rng.uniform(0, 360, n).astype(np.float32)
    rotd = np.where(rng.random(n) < 0.85, rng.normal(0, 4, n), rng.uniform(0, 360, n))
    kp1["angle"], kp2["angle"] = a1, np.mod(a1 + rotd, 360).astype(np.float32)
    base_d = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    d1 = base_d ^ np.packbits(rng.random((n, 256)) < 0.03, axis=1)
    d2 = base_d ^ np.packbits(rng.random((n, 256)) < rng.uniform(0.01, 0.15, (n, 1)), axis=1)
    # a fifth of KF2's features are distractors: fresh positions / descriptors
    dis = rng.random(n) < 0.2
    kp2["x"][dis] = rng.uniform(0, w, dis.sum())
    kp2["y"][dis] = rng.uniform(0, h, dis.sum())
    d2[dis] = rng.integers(0, 256, (dis.sum(), 32), dtype=np.uint8)
    # stereo for 60% (mvuRight = u - bf / z >= 0), MapPoints on 25%
    ur1 = np.where(rng.random(n) < 0.6, kp1["x"] - BF / z, -1).astype(np.float32)
    ur2 = np.where(rng.random(n) < 0.6, kp2["x"] - BF / X2[:, 2], -1).astype(np.float32)
    mp1 = (rng.random(n) < 0.25).astype(np.uint8)
    mp2 = (rng.random(n) < 0.25).astype(np.uint8)
    # KF2's feature order shuffled (index i of KF1 is not index i of KF2)
    perm = rng.permutation(n)
    kp2, d2, ur2, mp2 = kp2[perm], d2[perm], ur2[perm], mp2[perm]
    node = rng.integers(0, nnodes, n)
    node2 = np.where(rng.random(n) < 0.9, node, rng.integers(0, nnodes + 20, n))[perm]
    # F12 = K1^-T [t12]x R12 K2^-1 (ComputeF12) with R12 = R1w R2w^T, t12 = -R12 t2w + t1w
    R12 = R1w @ R2w.T
    t12 = -R12 @ t2w + t1w
    tx = np.array([[0, -t12[2], t12[1]], [t12[2], 0, -t12[0]], [-t12[1], t12[0], 0]])
    F12 = np.linalg.inv(K).T @ tx @ R12 @ np.linalg.inv(K)
    F12 /= np.abs(F12).max()
    g = np.zeros((), geom_dtype)
    g["F12"] = F12.astype(np.float32).reshape(9)
    g["Cw1"] = (-R1w.T @ t1w).astype(np.float32)
    g["Tcw2"] = np.concatenate([R2w, t2w[:, None]], 1).astype(np.float32).reshape(12)
    g["fx2"], g["fy2"], g["cx2"], g["cy2"] = fx, fy, cx, cy
    kf1 = dict(kps=kp1, desc=d1, uright=ur1, has_mp=mp1, fv=_fv(node))
    kf2 = dict(kps=kp2, desc=d2, uright=ur2, has_mp=mp2, fv=_fv(node2))
    return kf1, kf2, g, sf, s2


def py_triangulation(kf1, kf2, g, sf, s2, only_stereo, check_ori):
    """pure-Python restatement (float32 scalars, the reference's evaluation order)."""
    f32 = np.float32
    T = g["Tcw2"].reshape(3, 4)
    C2 = [f32(sum(float(T[r, k]) * float(g["Cw1"][k]) for k in range(3)) * 1.0 + float(T[r, 3]))
          for r in range(3)]
    invz = f32(1.0) / C2[2]
    ex = f32(g["fx2"]) * C2[0] * invz + f32(g["cx2"])
    ey = f32(g["fy2"]) * C2[1] * invz + f32(g["cy2"])
    F = g["F12"].astype(np.float32)
    n1 = len(kf1["kps"])
    m12 = np.full(n1, -1, np.int32)
    bins = {}
    hist = np.zeros(30, np.int64)
    nodes1, off1, feats1 = kf1["fv"]
    nodes2, off2, feats2 = kf2["fv"]
    pos2 = {int(nid): j for j, nid in enumerate(nodes2)}
    nm = 0
    bits1 = np.unpackbits(kf1["desc"], axis=1)
    bits2 = np.unpackbits(kf2["desc"], axis=1)
    for j1, nid in enumerate(nodes1):
        j2 = pos2.get(int(nid))
        if j2 is None:
            continue
        for idx1 in feats1[off1[j1]:off1[j1 + 1]]:
            if kf1["has_mp"][idx1]:
                continue
            st1 = kf1["uright"][idx1] >= 0
            if only_stereo and not st1:
                continue
            k1 = kf1["kps"][idx1]
            best, bidx = 50, -1
            for idx2 in feats2[off2[j2]:off2[j2 + 1]]:
                if kf2["has_mp"][idx2]:
                    continue
                st2 = kf2["uright"][idx2] >= 0
                if only_stereo and not st2:
                    continue
                dist = int((bits1[idx1] != bits2[idx2]).sum())
                if dist > 50 or dist > best:
                    continue
                k2 = kf2["kps"][idx2]
                if not st1 and not st2:
                    dx, dy = ex - k2["x"], ey - k2["y"]
                    if dx * dx + dy * dy < f32(100) * sf[k2["octave"]]:
                        continue
                a = k1["x"] * F[0] + k1["y"] * F[3] + F[6]
                b = k1["x"] * F[1] + k1["y"] * F[4] + F[7]
                c = k1["x"] * F[2] + k1["y"] * F[5] + F[8]
                num = a * k2["x"] + b * k2["y"] + c
                den = a * a + b * b
                if den == 0:
                    continue
                if float(num * num / den) < 3.84 * float(s2[k2["octave"]]):
                    best, bidx = dist, int(idx2)
            if bidx >= 0:
                m12[idx1] = bidx
                nm += 1
                if check_ori:
                    rot = f32(k1["angle"] - kf2["kps"][bidx]["angle"])
                    if rot < 0.0:
                        rot = f32(rot + f32(360.0))
                    b_ = int(np.round(rot * f32(1.0 / 30)))
                    b_ = 0 if b_ == 30 else b_
                    bins[int(idx1)] = b_
                    hist[b_] += 1
    if check_ori:
        m1 = m2 = m3 = 0
        i1 = i2 = i3 = -1
        for i in range(30):
            s = hist[i]
            if s > m1:
                m3, m2, m1, i3, i2, i1 = m2, m1, s, i2, i1, i
            elif s > m2:
                m3, m2, i3, i2 = m2, s, i2, i
            elif s > m3:
                m3, i3 = s, i
        if m2 < 0.1 * m1:
            i2 = i3 = -1
        elif m3 < 0.1 * m1:
            i3 = -1
        for i in range(n1):
            if m12[i] >= 0 and bins[i] not in (i1, i2, i3):
                m12[i] = -1
                nm -= 1
    return nm, m12


@pytest.mark.parametrize("seed", range(3))
@pytest.mark.parametrize("only_stereo,check_ori", [(False, False), (True, False), (False, True)])
def test_triangulation_equals_python(oracle, seed, only_stereo, check_ori):
    kf1, kf2, g, sf, s2 = tri_case(oracle.KP_DTYPE, oracle.TRI_GEOM_DTYPE, seed, n=400,
                                   forward=seed == 2)
    n, m = oracle.search_for_triangulation(kf1, kf2, g, sf, s2, only_stereo, check_ori)
    rn, rm = py_triangulation(kf1, kf2, g, sf, s2, only_stereo, check_ori)
    assert n == rn and np.array_equal(m, rm)
    assert n >= 20


def test_triangulation_semantics(oracle):
    """the rules the kernel relies on: a KF2 feature may match several KF1 features (vbMatched2
    is never set), and a forward motion's epipole rejects monocular pairs near it."""
    kf1, kf2, g, sf, s2 = tri_case(oracle.KP_DTYPE, oracle.TRI_GEOM_DTYPE, 5, n=600)
    n, m = oracle.search_for_triangulation(kf1, kf2, g, sf, s2)
    assert n > 50 and (m >= 0).sum() == n
    # make KF1 feature j a twin of a matched feature i of the same node: both match m[i]
    nodes, off, feats = kf1["fv"]
    done = 0
    for k in range(len(nodes)):
        fs = feats[off[k]:off[k + 1]]
        hit = [f for f in fs if m[f] >= 0]
        free = [f for f in fs if m[f] < 0 and not kf1["has_mp"][f]]
        if hit and free:
            i, j = hit[0], free[0]
            for key in ("kps", "desc", "uright"):
                kf1[key][j] = kf1[key][i]
            done += 1
    n2, m2 = oracle.search_for_triangulation(kf1, kf2, g, sf, s2)
    assert done >= 10 and n2 == n + done
    assert len(np.unique(m2[m2 >= 0])) < n2  # several KF1 features share a KF2 feature
    kf1f, kf2f, gf, _, _ = tri_case(oracle.KP_DTYPE, oracle.TRI_GEOM_DTYPE, 6, n=600, forward=True)
    # KF2 features moved onto the epipole (every epipolar line passes it): a monocular pair
    # there is rejected by the epipole test, a stereo one is not
    T = gf["Tcw2"].reshape(3, 4).astype(np.float64)
    C2 = T[:, :3] @ gf["Cw1"].astype(np.float64) + T[:, 3]
    ex, ey = 718.856 * C2[0] / C2[2] + 607.1928, 718.856 * C2[1] / C2[2] + 185.2157
    assert 0 < ex < 1241 and 0 < ey < 376
    kf2f["kps"]["x"][:150] = ex + np.random.default_rng(1).uniform(-0.3, 0.3, 150)
    kf2f["kps"]["y"][:150] = ey + np.random.default_rng(2).uniform(-0.3, 0.3, 150)
    kf2f["kps"]["octave"][:150] = 7
    kf1m = dict(kf1f, uright=np.full(600, -1.0, np.float32))
    kf2m = dict(kf2f, uright=np.full(600, -1.0, np.float32))
    kf1s = dict(kf1f, uright=np.full(600, 5.0, np.float32))
    nf, _ = oracle.search_for_triangulation(kf1m, kf2m, gf, sf, s2)
    ns, _ = oracle.search_for_triangulation(kf1s, kf2m, gf, sf, s2)
    assert 20 < nf < ns


def test_triangulation_empty(oracle):
    kf1, kf2, g, sf, s2 = tri_case(oracle.KP_DTYPE, oracle.TRI_GEOM_DTYPE, 1, n=50)
    e = dict(kps=kf2["kps"][:0], desc=kf2["desc"][:0], fv=(np.zeros(0), np.zeros(1), np.zeros(0)))
    n, m = oracle.search_for_triangulation(kf1, e, g, sf, s2)
    assert n == 0 and np.all(m == -1)


# ------------------------------------------------------------------------ Fuse
def fuse_case(mod, seed, n=2000, nmp=1500, w=1241, h=376, ties=True, bounds=None, scale=None):
    """A KeyFrame (mvKeysUn, mDescriptors, mvuRight, its FRUSTUM_DTYPE state) and nmp map
    points: most project next to one of its keypoints with a noisy copy of its descriptor
    (fusion targets), some carry a descriptor equal to several nearby keypoints' (ties broken
    by GetFeaturesInArea's order), the rest are far / behind / out of range / unrelated."""
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy = KITTI_K
    R = _rot(rng, 0.2)
    Ow = rng.uniform(-30, 30, 3)
    t = -R @ Ow
    Tcw = np.concatenate([R, t[:, None]], 1).astype(np.float32)
    p = None
    sf = (np.float32(1.2) ** np.arange(8)).astype(np.float32)
    kp = np.zeros(n, mod.KP_DTYPE)
    kp["x"], kp["y"] = rng.uniform(0, w, n), rng.uniform(0, h, n)
    kp["octave"] = rng.integers(0, 8, n)
    kp["angle"], kp["size"], kp["response"] = rng.uniform(0, 360, n), 31, 20
    desc = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    z = rng.uniform(3, 50, n)
    ur = np.where(rng.random(n) < 0.5, kp["x"] - BF / z, -1).astype(np.float32)
    # map points: seeded from keypoints (true position + noise), some far off
    src = rng.integers(0, n, nmp)
    zz = z[src] * rng.uniform(0.97, 1.03, nmp)
    uu = kp["x"][src] + rng.normal(0, 1.2, nmp) * sf[kp["octave"][src]]
    vv = kp["y"][src] + rng.normal(0, 1.2, nmp) * sf[kp["octave"][src]]
    far = rng.random(nmp) < 0.15
    uu[far] = rng.uniform(-300, w + 300, far.sum())
    zz[rng.random(nmp) < 0.05] *= -1
    pc = np.stack([(uu - cx) * zz / fx, (vv - cy) * zz / fy, zz], 1)
    pw = (R.T @ (pc - t).T).T
    mps = np.zeros(nmp, mod.MAPPOINT_DTYPE)
    mps["x"], mps["y"], mps["z"] = pw[:, 0], pw[:, 1], pw[:, 2]
    d = pw - Ow
    dist = np.linalg.norm(d, axis=1)
    nrm = d / dist[:, None] + rng.normal(0, 0.4, (nmp, 3))
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    mps["nx"], mps["ny"], mps["nz"] = nrm[:, 0], nrm[:, 1], nrm[:, 2]
    # distances consistent with the source keypoint's octave (PredictScale lands near it)
    lvl = kp["octave"][src]
    mps["max_dist"] = dist * (np.float32(1.2) ** lvl) * rng.uniform(0.9, 1.1, nmp)
    mps["min_dist"] = mps["max_dist"] / np.float32(1.2) ** 7 * rng.uniform(0.5, 2.0, nmp)
    mps["flags"] = np.where(rng.random(nmp) < 0.92, 1, 0)
    mdesc = desc[src] ^ np.packbits(rng.random((nmp, 256)) < rng.uniform(0.0, 0.25, (nmp, 1)), axis=1)
    mdesc[rng.random(nmp) < 0.1] = rng.integers(0, 256, 32, dtype=np.uint8)
    if ties:
        # clusters of keypoints with one descriptor next to a point: equal distances
        for j in range(0, min(nmp, 200), 4):
            s = src[j]
            near = np.argsort(np.hypot(kp["x"] - kp["x"][s], kp["y"] - kp["y"][s]))[:4]
            desc[near] = desc[s]
            kp["octave"][near] = kp["octave"][s]
            mdesc[j] = desc[s]
    fcam = np.zeros((), mod.FRUSTUM_DTYPE)
    # LoopClosing's Scw = Converter::toCvMat(g2o::Sim3): s * R and the scaled translation
    fcam["Tcw"] = (Tcw if scale is None else (np.float64(scale) * Tcw).astype(np.float32)).reshape(12)
    for k, val in zip(("fx", "fy", "cx", "cy", "bf", "log_scale_factor"),
                      (fx, fy, cx, cy, BF, np.float32(np.log(np.float64(np.float32(1.2)))))):
        fcam[k] = val
    fcam["nlevels"] = 8
    fcam["min_x"], fcam["max_x"], fcam["min_y"], fcam["max_y"] = bounds or (0.0, float(w), 0.0, float(h))
    del p
    return dict(kps=kp, desc=desc, uright=ur), fcam, mps, mdesc


def py_sim3_decompose(S):
    """Fuse(pKF, Scw, ...)'s scw = sqrt(row0 . row0) (double products), Rcw | tcw = Scw / scw
    (float alpha = 1 / scw, one rounding per element)."""
    S = np.asarray(S, np.float32).reshape(3, 4)
    d = 0.0
    for k in range(3):
        d += float(S[0, k]) * float(S[0, k])
    scw = np.float32(np.sqrt(d))
    a = np.float32(1.0 / float(scw))
    return (S * a).astype(np.float32)


def py_fuse(kf, fcam, mps, mdesc, th, sf, isg, sim3=False):
    """pure-Python restatement of Fuse's search over the reference grid and order; sim3: the
    Fuse(pKF, Scw, vpPoints, th, vpReplacePoint) variant (Scw decomposed, no reprojection
    gate, ORBmatcher.cc:1133-1238)."""
    f32 = np.float32
    T = py_sim3_decompose(fcam["Tcw"]) if sim3 else fcam["Tcw"].reshape(3, 4)
    b = (f32(fcam["min_x"]), f32(fcam["max_x"]), f32(fcam["min_y"]), f32(fcam["max_y"]))
    iw = f32(64) / f32(b[1] - b[0])
    ih = f32(48) / f32(b[3] - b[2])
    kps = kf["kps"]
    grid = {}
    for i in range(len(kps)):
        px = int(np.round(f32(kps["x"][i] - b[0]) * iw))
        py = int(np.round(f32(kps["y"][i] - b[2]) * ih))
        if 0 <= px < 64 and 0 <= py < 48:
            grid.setdefault((px, py), []).append(i)
    kb = tuple(f32(int(x)) for x in b)  # KeyFrame's int mnMinX .. (KeyFrame.h:288-291)
    Ow = [f32(sum(float(T[k, r]) * float(T[k, 3]) for k in range(3)) * -1.0) for r in range(3)]
    bits_k = np.unpackbits(kf["desc"], axis=1)
    bits_m = np.unpackbits(np.ascontiguousarray(mdesc, np.uint8), axis=1)
    bi = np.full(len(mps), -1, np.int32)
    bd = np.full(len(mps), 256, np.int32)
    for i, mp in enumerate(mps):
        if not mp["flags"] & 1:
            continue
        P = [f32(mp["x"]), f32(mp["y"]), f32(mp["z"])]
        Pc = [f32(sum(float(T[r, k]) * float(P[k]) for k in range(3)) * 1.0 + float(T[r, 3]))
              for r in range(3)]
        if Pc[2] < 0:
            continue
        invz = f32(1) / Pc[2]
        u = f32(fcam["fx"]) * (Pc[0] * invz) + f32(fcam["cx"])
        v = f32(fcam["fy"]) * (Pc[1] * invz) + f32(fcam["cy"])
        if not (u >= kb[0] and u < kb[1] and v >= kb[2] and v < kb[3]):
            continue
        ur = u - f32(fcam["bf"]) * invz
        PO = [P[k] - Ow[k] for k in range(3)]
        d3 = f32(np.sqrt(sum(float(x) * float(x) for x in PO)))
        if d3 < f32(0.8) * mp["min_dist"] or d3 > f32(1.2) * mp["max_dist"]:
            continue
        dot = float(PO[0]) * float(mp["nx"]) + float(PO[1]) * float(mp["ny"]) + float(PO[2]) * float(mp["nz"])
        if dot < 0.5 * float(d3):
            continue
        lvl = int(np.ceil(np.log(float(mp["max_dist"] / d3)) / float(fcam["log_scale_factor"])))
        lvl = min(max(lvl, 0), int(fcam["nlevels"]) - 1)
        r = f32(th) * sf[lvl]
        cx0 = max(0, int(np.floor((u - kb[0] - r) * iw)))
        cx1 = min(63, int(np.ceil((u - kb[0] + r) * iw)))
        cy0 = max(0, int(np.floor((v - kb[2] - r) * ih)))
        cy1 = min(47, int(np.ceil((v - kb[2] + r) * ih)))
        if cx0 >= 64 or cx1 < 0 or cy0 >= 48 or cy1 < 0:
            continue
        best, bidx = 256, -1
        for ix in range(cx0, cx1 + 1):
            for iy in range(cy0, cy1 + 1):
                for idx in grid.get((ix, iy), []):
                    k = kps[idx]
                    if not (abs(f32(k["x"] - u)) < r and abs(f32(k["y"] - v)) < r):
                        continue
                    if k["octave"] < lvl - 1 or k["octave"] > lvl:
                        continue
                    ex, ey = u - k["x"], v - k["y"]
                    if sim3:
                        pass
                    elif kf["uright"][idx] >= 0:
                        er = ur - kf["uright"][idx]
                        if float((ex * ex + ey * ey + er * er) * isg[k["octave"]]) > 7.8:
                            continue
                    elif float((ex * ex + ey * ey) * isg[k["octave"]]) > 5.99:
                        continue
                    dist = int((bits_m[i] != bits_k[idx]).sum())
                    if dist < best:
                        best, bidx = dist, idx
        bd[i] = best
        if best <= 50:
            bi[i] = bidx
    return int((bi >= 0).sum()), bi, bd


def _fuse_tables(oracle):
    p = oracle.params(nfeatures=2000, scale_factor=1.2, nlevels=8)
    return np.array(p.scale[:8], np.float32), np.array(p.inv_sigma2[:8], np.float32)


@pytest.mark.parametrize("seed", range(3))
def test_fuse_equals_python(oracle, seed):
    kf, fcam, mps, mdesc = fuse_case(oracle, seed, n=1200, nmp=500)
    sf, isg = _fuse_tables(oracle)
    th = 3.0 if seed else 5.0
    n, bi, bd = oracle.fuse_search(kf, fcam, mps, mdesc, th, sf, isg)
    rn, rbi, rbd = py_fuse(kf, fcam, mps, mdesc, th, sf, isg)
    assert n == rn and np.array_equal(bi, rbi) and np.array_equal(bd, rbd)
    assert n > 50 and (bd < 256).sum() > n  # targets, and candidates past TH_LOW


def test_fuse_fractional_bounds(oracle):
    """undistorted-camera bounds (TUM1's, fractional): the KeyFrame tests IsInImage and
    GetFeaturesInArea's cells against its int mnMinX .. (the Frame's truncated) while its grid
    is the Frame's float one"""
    b = (10.80118465423584, 1230.0478515625, 14.668615341186523, 370.3118896484375)
    kf, fcam, mps, mdesc = fuse_case(oracle, 11, n=1200, nmp=600, bounds=b)
    sf, isg = _fuse_tables(oracle)
    n, bi, bd = oracle.fuse_search(kf, fcam, mps, mdesc, 3.0, sf, isg)
    rn, rbi, rbd = py_fuse(kf, fcam, mps, mdesc, 3.0, sf, isg)
    assert n == rn and np.array_equal(bi, rbi) and np.array_equal(bd, rbd) and n > 50


@pytest.mark.parametrize("seed,scale", [(20, 1.0), (21, 0.37), (22, 2.9)])
def test_fuse_sim3_equals_python(oracle, seed, scale):
    """Fuse(pKF, Scw, vpPoints, th = 4, vpReplacePoint) (LoopClosing::SearchAndFuse): the Sim3
    decomposition and the search without the reprojection gate, C vs Python"""
    kf, fcam, mps, mdesc = fuse_case(oracle, seed, n=1200, nmp=500, scale=scale)
    sf, isg = _fuse_tables(oracle)
    assert np.array_equal(oracle.sim3_decompose(fcam["Tcw"]), py_sim3_decompose(fcam["Tcw"]))
    n, bi, bd = oracle.fuse_sim3_search(kf, fcam, mps, mdesc, 4.0, sf)
    rn, rbi, rbd = py_fuse(kf, fcam, mps, mdesc, 4.0, sf, isg, sim3=True)
    assert n == rn and np.array_equal(bi, rbi) and np.array_equal(bd, rbd)
    assert n > 50 and (bd < 256).sum() > n
    # without the reprojection gate at least as many points find a target as in Fuse(pKF, ...)
    f1 = fcam.copy()
    f1["Tcw"] = py_sim3_decompose(fcam["Tcw"]).reshape(12)
    n1, _, _ = oracle.fuse_search(kf, f1, mps, mdesc, 4.0, sf, isg)
    assert n >= n1


def test_sim3_decompose_known():
    """scale 2 of an exact rotation: Rcw and tcw come back exactly (power-of-two alpha)"""
    from oracle import pyoracle as O
    R = np.array([[0, -1, 0], [1, 0, 0], [0, 0, 1]], np.float32)
    S = np.concatenate([2 * R, np.array([[2.0], [-4.0], [6.0]], np.float32)], 1)
    T = O.sim3_decompose(S)
    assert np.array_equal(T[:, :3], R) and np.array_equal(T[:, 3], [1, -2, 3])
