"""Oracle pins for the Relocalization and LoopClosing projection matchers
(oracle/loop_oracle.c), each against an independent pure-Python restatement of the
reference's loop:

  ORBmatcher::SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist)
      src/ORBmatcher.cc:1670-1798 (Tracking::Relocalization, Tracking.cc:2120, 2141)
  ORBmatcher::SearchByProjection(pKF, Scw, vpPoints, vpMatched, th)
      src/ORBmatcher.cc:353-470 (LoopClosing::ComputeSim3, LoopClosing.cc:669)

Both write a keypoint-indexed array and skip keypoints already written, so a later point's
candidates depend on the earlier points' picks; the cases put several points on one keypoint
to exercise that, and (relocalization) rotations outside the dominant bins.
Parity unpinned beyond these restatements: OpenCV is absent, the pins are the ones
documented in DESIGN.md §4 (cv::gemm small-matrix path, norm / dot in double).
"""
import numpy as np
import pytest

from test_oracle_mapping import BF, KITTI_K, _rot, py_sim3_decompose

f32 = np.float32
W, H = 1241, 376


def _grid(kps, b):
    iw = f32(64) / f32(b[1] - b[0])
    ih = f32(48) / f32(b[3] - b[2])
    grid = {}
    for i in range(len(kps)):
        px = int(np.round(f32(kps["x"][i] - b[0]) * iw))
        py = int(np.round(f32(kps["y"][i] - b[2]) * ih))
        if 0 <= px < 64 and 0 <= py < 48:
            grid.setdefault((px, py), []).append(i)
    return grid, iw, ih


def _in_area(grid, iw, ih, wmin_x, wmin_y, kps, x, y, r, minL, maxL):
    """Frame::GetFeaturesInArea (Frame.cc:421-504) in the reference's enumeration order;
    wmin_x / wmin_y: the bounds the cell range uses (the KeyFrame's int ones in KeyFrame's)"""
    cx0 = max(0, int(np.floor((x - wmin_x - r) * iw)))
    cx1 = min(63, int(np.ceil((x - wmin_x + r) * iw)))
    cy0 = max(0, int(np.floor((y - wmin_y - r) * ih)))
    cy1 = min(47, int(np.ceil((y - wmin_y + r) * ih)))
    if cx0 >= 64 or cx1 < 0 or cy0 >= 48 or cy1 < 0:
        return []
    chk = minL > 0 or maxL >= 0
    out = []
    for ix in range(cx0, cx1 + 1):
        for iy in range(cy0, cy1 + 1):
            for idx in grid.get((ix, iy), []):
                o = int(kps["octave"][idx])
                if chk and (o < minL or (maxL >= 0 and o > maxL)):
                    continue
                if abs(f32(kps["x"][idx] - x)) < r and abs(f32(kps["y"][idx] - y)) < r:
                    out.append(idx)
    return out


def _gemm(T, X, alpha, c):
    return [f32((sum(float(T[r][k]) * float(X[k]) for k in range(3)) * alpha)
                + (float(c[r]) if c is not None else 0.0)) for r in range(3)]


def _gemm_t(T, X, alpha):
    return [f32(sum(float(T[k][r]) * float(X[k]) for k in range(3)) * alpha) for r in range(3)]


def _predict(max_dist, d, lsf, nl):
    lvl = int(np.ceil(np.log(float(f32(max_dist) / d)) / float(lsf)))
    return min(max(lvl, 0), nl - 1)


def _ham(a, b):
    return int(np.unpackbits(np.bitwise_xor(a, b)).sum())


def _three_maxima(h):
    m1 = m2 = m3 = 0
    i1 = i2 = i3 = -1
    for i, s in enumerate(h):
        if s > m1:
            m3, m2, m1, i3, i2, i1 = m2, m1, s, i2, i1, i
        elif s > m2:
            m3, m2, i3, i2 = m2, s, i2, i
        elif s > m3:
            m3, i3 = s, i
    if m2 < f32(0.1) * f32(m1):
        i2 = i3 = -1
    elif m3 < f32(0.1) * f32(m1):
        i3 = -1
    return i1, i2, i3


def py_reloc(kps, desc, taken0, fcam, sf, pts, pdesc, th, orb_dist, check_ori=True):
    b = tuple(f32(fcam[k]) for k in ("min_x", "max_x", "min_y", "max_y"))
    grid, iw, ih = _grid(kps, b)
    T = fcam["Tcw"].reshape(3, 4)
    tcw = T[:, 3]
    Ow = _gemm_t(T, tcw, -1.0)
    taken = np.array(taken0, bool) if taken0 is not None else np.zeros(len(kps), bool)
    match = np.full(len(kps), -1, np.int32)
    pushes = []
    nm = 0
    for i, P in enumerate(pts):
        if not P["flags"] & 1:
            continue
        X = [f32(P["x"]), f32(P["y"]), f32(P["z"])]
        xc = _gemm(T, X, 1.0, tcw)
        invzc = f32(1.0 / float(xc[2]))
        u = f32(fcam["fx"]) * xc[0] * invzc + f32(fcam["cx"])
        v = f32(fcam["fy"]) * xc[1] * invzc + f32(fcam["cy"])
        if u < b[0] or u > b[1] or v < b[2] or v > b[3]:
            continue
        PO = [X[k] - Ow[k] for k in range(3)]
        d3 = f32(np.sqrt(sum(float(x) * float(x) for x in PO)))
        if d3 < f32(0.8) * P["min_dist"] or d3 > f32(1.2) * P["max_dist"]:
            continue
        lvl = _predict(P["max_dist"], d3, fcam["log_scale_factor"], int(fcam["nlevels"]))
        r = f32(th) * sf[lvl]
        best, bi = 256, -1
        for i2 in _in_area(grid, iw, ih, b[0], b[2], kps, u, v, r, lvl - 1, lvl + 1):
            if taken[i2]:
                continue
            d = _ham(pdesc[i], desc[i2])
            if d < best:
                best, bi = d, i2
        if best <= orb_dist:
            match[bi] = i
            taken[bi] = True
            nm += 1
            if check_ori:
                rot = f32(P["angle"]) - f32(kps["angle"][bi])
                if rot < 0.0:
                    rot = rot + f32(360)
                q = float(rot * (f32(1) / f32(30)))  # roundf: halves away from zero
                bn = int(np.floor(q))
                bn += 1 if q - bn >= 0.5 else 0
                if bn == 30:
                    bn = 0
                pushes.append((bn, bi))
    if check_ori:
        h = [0] * 30
        for bn, _ in pushes:
            h[bn] += 1
        keep = _three_maxima(h)
        for bn, bi in pushes:
            if bn not in keep:
                match[bi] = -2
                nm -= 1
    return nm, match


def py_sim3_proj(kps, desc, taken0, fcam, sf, mps, mdesc, th):
    b = tuple(f32(fcam[k]) for k in ("min_x", "max_x", "min_y", "max_y"))
    grid, iw, ih = _grid(kps, b)
    kb = tuple(f32(int(x)) for x in b)
    T = py_sim3_decompose(fcam["Tcw"])
    tcw = T[:, 3]
    Ow = _gemm_t(T, tcw, -1.0)
    taken = np.array(taken0, bool) if taken0 is not None else np.zeros(len(kps), bool)
    match = np.full(len(kps), -1, np.int32)
    nm = 0
    for i, M in enumerate(mps):
        if not M["flags"] & 1:
            continue
        X = [f32(M["x"]), f32(M["y"]), f32(M["z"])]
        Pc = _gemm(T, X, 1.0, tcw)
        if Pc[2] < 0.0:
            continue
        invz = f32(1) / Pc[2]
        u = f32(fcam["fx"]) * (Pc[0] * invz) + f32(fcam["cx"])
        v = f32(fcam["fy"]) * (Pc[1] * invz) + f32(fcam["cy"])
        if not (u >= kb[0] and u < kb[1] and v >= kb[2] and v < kb[3]):
            continue
        PO = [X[k] - Ow[k] for k in range(3)]
        d3 = f32(np.sqrt(sum(float(x) * float(x) for x in PO)))
        if d3 < f32(0.8) * M["min_dist"] or d3 > f32(1.2) * M["max_dist"]:
            continue
        dot = float(PO[0]) * float(M["nx"]) + float(PO[1]) * float(M["ny"]) + float(PO[2]) * float(M["nz"])
        if dot < 0.5 * float(d3):
            continue
        lvl = _predict(M["max_dist"], d3, fcam["log_scale_factor"], int(fcam["nlevels"]))
        r = f32(th) * sf[lvl]
        best, bi = 256, -1
        for idx in _in_area(grid, iw, ih, kb[0], kb[2], kps, u, v, r, -1, -1):
            if taken[idx]:
                continue
            o = int(kps["octave"][idx])
            if o < lvl - 1 or o > lvl:
                continue
            d = _ham(mdesc[i], desc[idx])
            if d < best:
                best, bi = d, idx
        if best <= 50:
            match[bi] = i
            taken[bi] = True
            nm += 1
    return nm, match


def _frame(mod, rng, n, w=W, h=H):
    kp = np.zeros(n, mod.KP_DTYPE)
    kp["x"], kp["y"] = rng.uniform(0, w, n), rng.uniform(0, h, n)
    kp["octave"] = rng.integers(0, 8, n)
    kp["angle"], kp["size"], kp["response"] = rng.uniform(0, 360, n), 31, 20
    desc = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    return kp, desc


def _points(rng, kp, desc, R, t, Ow, npts, dup=0.2, behind=0.05):
    """npts points seeded from keypoints (a fraction of them sharing one keypoint)"""
    fx, fy, cx, cy = KITTI_K
    n = len(kp)
    sf = f32(1.2) ** np.arange(8)
    src = rng.integers(0, n, npts)
    d = rng.random(npts) < dup
    src[d] = src[rng.integers(0, npts, d.sum())]
    z = rng.uniform(3, 50, npts)
    uu = kp["x"][src] + rng.normal(0, 1.0, npts) * sf[kp["octave"][src]]
    vv = kp["y"][src] + rng.normal(0, 1.0, npts) * sf[kp["octave"][src]]
    far = rng.random(npts) < 0.1
    uu[far] = rng.uniform(-200, W + 200, far.sum())
    z[rng.random(npts) < behind] *= -1
    pc = np.stack([(uu - cx) * z / fx, (vv - cy) * z / fy, z], 1)
    pw = (R.T @ (pc - t).T).T
    dist = np.linalg.norm(pw - Ow, axis=1)
    mx = dist * f32(1.2) ** kp["octave"][src] * rng.uniform(0.9, 1.1, npts)
    mn = mx / f32(1.2) ** 7 * rng.uniform(0.5, 2.0, npts)
    pd = desc[src] ^ np.packbits(rng.random((npts, 256)) < rng.uniform(0.0, 0.2, (npts, 1)), axis=1)
    return src, pw, mx, mn, pd


def _fcam(mod, T, bounds):
    fcam = np.zeros((), mod.FRUSTUM_DTYPE)
    fcam["Tcw"] = T.reshape(12)
    for k, val in zip(("fx", "fy", "cx", "cy", "bf", "log_scale_factor"),
                      (*KITTI_K, BF, f32(np.log(np.float64(f32(1.2)))))):
        fcam[k] = val
    fcam["nlevels"] = 8
    fcam["min_x"], fcam["max_x"], fcam["min_y"], fcam["max_y"] = bounds or (0.0, float(W), 0.0, float(H))
    return fcam


def reloc_case(mod, seed, n=2000, npts=1500, bounds=None):
    """CurrentFrame (mvKeysUn, mDescriptors, mvpMapPoints != NULL on entry) and a candidate
    KeyFrame's map points: most near a frame keypoint with a noisy descriptor copy and the
    keypoint angle turned by a common 25 degrees (15% random: the rotation filter drops
    them), some sharing a keypoint, some behind the camera (the loop has no depth test)."""
    rng = np.random.default_rng(seed)
    kp, desc = _frame(mod, rng, n)
    R = _rot(rng, 0.2)
    Ow = rng.uniform(-30, 30, 3)
    t = -R @ Ow
    src, pw, mx, mn, pd = _points(rng, kp, desc, R, t, Ow, npts)
    pts = np.zeros(npts, mod.RELOC_DTYPE)
    pts["x"], pts["y"], pts["z"] = pw[:, 0], pw[:, 1], pw[:, 2]
    pts["max_dist"], pts["min_dist"] = mx, mn
    ang = (kp["angle"][src] + 25 + rng.normal(0, 3, npts)) % 360
    odd = rng.random(npts) < 0.15
    ang[odd] = rng.uniform(0, 360, odd.sum())
    pts["angle"] = ang
    pts["flags"] = np.where(rng.random(npts) < 0.9, 1, 0)
    taken0 = (rng.random(n) < 0.08).astype(np.uint8)
    T = np.concatenate([R, t[:, None]], 1).astype(np.float32)
    return dict(kps=kp, desc=desc, taken0=taken0), _fcam(mod, T, bounds), pts, pd


def sim3proj_case(mod, seed, n=2000, nm=1500, scale=1.0, bounds=None):
    """pKF (mvKeysUn, mDescriptors, vpMatched != NULL on entry), Scw = scale [R | t] and the
    loop's map points (vpPoints) near its keypoints, some sharing one."""
    rng = np.random.default_rng(seed)
    kp, desc = _frame(mod, rng, n)
    R = _rot(rng, 0.2)
    Ow = rng.uniform(-30, 30, 3)
    t = -R @ Ow
    src, pw, mx, mn, pd = _points(rng, kp, desc, R, t, Ow, nm)
    mps = np.zeros(nm, mod.MAPPOINT_DTYPE)
    mps["x"], mps["y"], mps["z"] = pw[:, 0], pw[:, 1], pw[:, 2]
    dv = pw - Ow
    nrm = dv / np.linalg.norm(dv, axis=1)[:, None] + rng.normal(0, 0.4, (nm, 3))
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    mps["nx"], mps["ny"], mps["nz"] = nrm[:, 0], nrm[:, 1], nrm[:, 2]
    mps["max_dist"], mps["min_dist"] = mx, mn
    mps["flags"] = np.where(rng.random(nm) < 0.9, 1, 0)
    taken0 = (rng.random(n) < 0.08).astype(np.uint8)
    T = np.concatenate([R, t[:, None]], 1)
    S = (np.float64(scale) * T).astype(np.float32)
    return dict(kps=kp, desc=desc, taken0=taken0), _fcam(mod, S, bounds), mps, pd


def _sf(oracle):
    p = oracle.params(nfeatures=2000, scale_factor=1.2, nlevels=8)
    return np.array(p.scale[:8], np.float32)


FRAC = (10.80118465423584, 1230.0478515625, 14.668615341186523, 370.3118896484375)


@pytest.mark.parametrize("seed,th,orb_dist,bounds", [(0, 10, 100, None), (1, 3, 64, None),
                                                      (2, 10, 100, FRAC)])
def test_reloc_equals_python(oracle, seed, th, orb_dist, bounds):
    f, fcam, pts, pd = reloc_case(oracle, seed, n=1200, npts=700, bounds=bounds)
    sf = _sf(oracle)
    n, m = oracle.search_by_projection_reloc(f["kps"], f["desc"], f["taken0"], fcam, sf, pts, pd,
                                             th, orb_dist)
    rn, rm = py_reloc(f["kps"], f["desc"], f["taken0"], fcam, sf, pts, pd, th, orb_dist)
    assert n == rn and np.array_equal(m, rm)
    assert n > 100 and (m == -2).sum() > 0
    assert np.all(m[f["taken0"] == 1] == -1)


def test_reloc_no_rotation_check(oracle):
    f, fcam, pts, pd = reloc_case(oracle, 3, n=1200, npts=700)
    sf = _sf(oracle)
    n, m = oracle.search_by_projection_reloc(f["kps"], f["desc"], None, fcam, sf, pts, pd, 10,
                                             100, check_ori=False)
    rn, rm = py_reloc(f["kps"], f["desc"], None, fcam, sf, pts, pd, 10, 100, check_ori=False)
    assert n == rn and np.array_equal(m, rm) and (m == -2).sum() == 0 and n > 100


@pytest.mark.parametrize("seed,scale,bounds", [(10, 1.0, None), (11, 0.45, None),
                                               (12, 2.6, FRAC)])
def test_sim3_projection_equals_python(oracle, seed, scale, bounds):
    f, fcam, mps, md = sim3proj_case(oracle, seed, n=1200, nm=700, scale=scale, bounds=bounds)
    sf = _sf(oracle)
    n, m = oracle.search_by_projection_sim3(f["kps"], f["desc"], f["taken0"], fcam, sf, mps, md, 10)
    rn, rm = py_sim3_proj(f["kps"], f["desc"], f["taken0"], fcam, sf, mps, md, 10)
    assert n == rn and np.array_equal(m, rm) and n > 100
    assert np.all(m[f["taken0"] == 1] == -1)


def test_taken_order_dependence(oracle):
    """two points on one keypoint: the first takes it, the second falls to another
    candidate or none -- the result differs from an order-free per-point best"""
    f, fcam, mps, md = sim3proj_case(oracle, 13, n=1200, nm=700)
    sf = _sf(oracle)
    n, m = oracle.search_by_projection_sim3(f["kps"], f["desc"], None, fcam, sf, mps, md, 10)
    rev = mps[::-1].copy()
    n2, m2 = oracle.search_by_projection_sim3(f["kps"], f["desc"], None, fcam, sf, rev,
                                              md[::-1].copy(), 10)
    m2r = np.where(m2 >= 0, len(mps) - 1 - m2, m2)
    assert not np.array_equal(m, m2r)


def test_loop_matchers_empty(oracle):
    f, fcam, pts, pd = reloc_case(oracle, 4, n=50, npts=20)
    sf = _sf(oracle)
    n, m = oracle.search_by_projection_reloc(f["kps"], f["desc"], None, fcam, sf, pts[:0],
                                             pd[:0], 10, 100)
    assert n == 0 and np.all(m == -1)
    n, m = oracle.search_by_projection_reloc(f["kps"][:0], f["desc"][:0], None, fcam, sf, pts,
                                             pd, 10, 100)
    assert n == 0 and len(m) == 0


# ------------------------------------------------------------------ SearchBySim3
def sim3_case(mod, seed, n=1500, m=900, s12=1.3, bounds=None):
    """two KeyFrames of one scene in two map frames related by a Sim3: pKF1 sees m common
    points at slots 0..m-1, pKF2 at a permutation of its slots; S12 = [s12 R12 | t12] maps
    camera-2 to camera-1 coordinates.  Map point descriptors are noisy copies of their
    keypoint's; some slots have no (or a bad) point; a few are matched before the call."""
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy = KITTI_K
    R12 = _rot(rng, 0.05)
    t12 = rng.normal(0, 0.3, 3)
    R1, R2 = _rot(rng, 0.3), _rot(rng, 0.3)
    t1, t2 = rng.normal(0, 5, 3), rng.normal(0, 5, 3)
    u1 = rng.uniform(5, W - 5, n)
    v1 = rng.uniform(5, H - 5, n)
    z1 = rng.uniform(4, 40, n)
    pc1 = np.stack([(u1 - cx) * z1 / fx, (v1 - cy) * z1 / fy, z1], 1)
    pc2 = ((pc1 - t12) @ R12) / s12  # R12^T (p - t12) / s12, row form
    perm = rng.permutation(n)
    sf = f32(1.2) ** np.arange(8)

    octs = rng.integers(0, 8, n)  # one octave per scene point in both KeyFrames

    def kf(pc, order, R, t):
        k = np.zeros(n, mod.KP_DTYPE)
        oc = octs
        u = fx * pc[:, 0] / pc[:, 2] + cx + rng.normal(0, 0.8, n) * sf[oc]
        v = fy * pc[:, 1] / pc[:, 2] + cy + rng.normal(0, 0.8, n) * sf[oc]
        k["x"][order], k["y"][order], k["octave"][order] = u, v, oc
        k["angle"], k["size"], k["response"] = rng.uniform(0, 360, n), 31, 20
        # non-common slots (m..n-1 of pKF1's order): random points of the image
        extra = order[m:]
        k["x"][extra] = rng.uniform(0, W, len(extra))
        k["y"][extra] = rng.uniform(0, H, len(extra))
        pw = (pc - t) @ R  # R^T (pc - t)
        mp = np.zeros(n, mod.MAPPOINT_DTYPE)
        mp["x"][order], mp["y"][order], mp["z"][order] = pw[:, 0], pw[:, 1], pw[:, 2]
        dist = np.linalg.norm(pc, axis=1)
        mx = dist * f32(1.2) ** oc * rng.uniform(0.9, 1.1, n)
        mp["max_dist"][order] = mx
        mp["min_dist"][order] = mx / f32(1.2) ** 7 * rng.uniform(0.5, 2.0, n)
        mp["flags"] = np.where(rng.random(n) < 0.88, 1, 0)
        return k, mp

    k1, mp1 = kf(pc1, np.arange(n), R1, t1)
    k2, mp2 = kf(pc2, perm, R2, t2)
    d1 = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    d2 = np.zeros_like(d1)
    d2[perm[:m]] = d1[:m] ^ np.packbits(rng.random((m, 256)) < rng.uniform(0.0, 0.2, (m, 1)), axis=1)
    d2[perm[m:]] = rng.integers(0, 256, (n - m, 32), dtype=np.uint8)
    md1 = d1 ^ np.packbits(rng.random((n, 256)) < 0.05, axis=1)
    md2 = d2 ^ np.packbits(rng.random((n, 256)) < 0.05, axis=1)
    matched1 = (rng.random(n) < 0.05).astype(np.uint8)
    matched2 = np.zeros(n, np.uint8)
    common = np.nonzero(matched1[:m])[0]
    matched2[perm[common]] = 1
    g = np.zeros((), mod.SIM3_PAIR_DTYPE)
    g["T1w"] = np.concatenate([R1, t1[:, None]], 1).astype(np.float32).reshape(12)
    g["T2w"] = np.concatenate([R2, t2[:, None]], 1).astype(np.float32).reshape(12)
    g["R12"] = R12.astype(np.float32).reshape(9)
    g["t12"] = t12.astype(np.float32)
    g["s12"] = s12
    g["fx"], g["fy"], g["cx"], g["cy"] = fx, fy, cx, cy
    g["log_scale_factor"] = f32(np.log(np.float64(f32(1.2))))
    g["nlevels"] = 8
    g["min_x"], g["max_x"], g["min_y"], g["max_y"] = bounds or (0.0, float(W), 0.0, float(H))
    return (dict(kps=k1, desc=d1), mp1, md1, matched1, dict(kps=k2, desc=d2), mp2, md2,
            matched2, g, perm)


def py_search_by_sim3(kf1, mp1, md1, am1, kf2, mp2, md2, am2, g, th, sf):
    b = tuple(f32(g[k]) for k in ("min_x", "max_x", "min_y", "max_y"))
    kb = tuple(f32(int(x)) for x in b)
    R12 = g["R12"].reshape(3, 3)
    s12 = f32(g["s12"])
    a = f32(1.0 / float(s12))
    sR12 = (R12 * s12).astype(np.float32)
    sR21 = (R12.T * a).astype(np.float32)
    t21 = _gemm(sR21, g["t12"], -1.0, None)

    def direction(tk, tdesc, mps, mdesc, am, Tsw, M, tm):
        grid, iw, ih = _grid(tk, b)
        T = Tsw.reshape(3, 4)
        out = np.full(len(mps), -1, np.int32)
        for i, mp in enumerate(mps):
            if not mp["flags"] & 1 or (am is not None and am[i]):
                continue
            X = [f32(mp["x"]), f32(mp["y"]), f32(mp["z"])]
            pcs = _gemm(T, X, 1.0, T[:, 3])
            pc = _gemm(M, pcs, 1.0, tm)
            if pc[2] < 0.0:
                continue
            invz = f32(1.0 / float(pc[2]))
            u = f32(g["fx"]) * (pc[0] * invz) + f32(g["cx"])
            v = f32(g["fy"]) * (pc[1] * invz) + f32(g["cy"])
            if not (u >= kb[0] and u < kb[1] and v >= kb[2] and v < kb[3]):
                continue
            d3 = f32(np.sqrt(sum(float(x) * float(x) for x in pc)))
            if d3 < f32(0.8) * mp["min_dist"] or d3 > f32(1.2) * mp["max_dist"]:
                continue
            lvl = _predict(mp["max_dist"], d3, g["log_scale_factor"], int(g["nlevels"]))
            r = f32(th) * sf[lvl]
            best, bi = 1 << 30, -1
            for idx in _in_area(grid, iw, ih, kb[0], kb[2], tk, u, v, r, -1, -1):
                o = int(tk["octave"][idx])
                if o < lvl - 1 or o > lvl:
                    continue
                d = _ham(mdesc[i], tdesc[idx])
                if d < best:
                    best, bi = d, idx
            if best <= 100:
                out[i] = bi
        return out

    vn1 = direction(kf2["kps"], kf2["desc"], mp1, md1, am1, g["T1w"], sR21, t21)
    vn2 = direction(kf1["kps"], kf1["desc"], mp2, md2, am2, g["T2w"], sR12, g["t12"])
    m12 = np.full(len(mp1), -1, np.int32)
    for i1, i2 in enumerate(vn1):
        if i2 >= 0 and vn2[i2] == i1:
            m12[i1] = i2
    return int((m12 >= 0).sum()), m12


@pytest.mark.parametrize("seed,s12,th,bounds", [(50, 1.05, 7.5, None), (51, 0.9, 7.5, FRAC),
                                                (52, 1.02, 3.0, None), (53, 1.15, 7.5, None)])
def test_search_by_sim3_equals_python(oracle, seed, s12, th, bounds):
    c = sim3_case(oracle, seed, n=900, m=600, s12=s12, bounds=bounds)
    kf1, mp1, md1, a1, kf2, mp2, md2, a2, g, perm = c
    sf = _sf(oracle)
    n, m = oracle.search_by_sim3(kf1, mp1, md1, a1, kf2, mp2, md2, a2, g, th, sf)
    rn, rm = py_search_by_sim3(kf1, mp1, md1, a1, kf2, mp2, md2, a2, g, th, sf)
    assert n == rn and np.array_equal(m, rm)
    assert n > 100
    ok = m >= 0
    assert (m[ok] == perm[np.nonzero(ok)[0]]).mean() > 0.9  # mostly the true correspondences
    assert np.all(m[a1 == 1] == -1)
