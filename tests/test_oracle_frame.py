"""CPU: the oracle's Frame / MapPoint geometry (oracle/frame_oracle.c) pinned against an
independent numpy restatement and against the semantics it must have:

  Frame::UndistortKeyPoints / ComputeImageBounds (src/Frame.cc:542-611) over
      cv::undistortPoints (OpenCV 3.4 cvUndistortPointsInternal, COUNT 5): the C oracle
      equals a float64 numpy restatement of the same iteration bit for bit; the result
      inverts OpenCV's forward distortion model (distort(undistort(p)) = p to 1e-3 px within
      200 px of the centre, where 5 iterations converge); k1 == 0 is a copy (Frame.cc:544-548);
  Frame::isInFrustum (src/Frame.cc:342-409, PredictScale src/MapPoint.cc:575-590): equals a
      numpy restatement (cv::gemm / norm / dot in double) on random map points, each early-out
      (behind the camera, outside the bounds, outside [0.8 dmin, 1.2 dmax], view angle) hit;
  MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:342-420): equals np.sort-based
      medians with the first-row tie rule, N = 1 .. 700.

The GPU kernels are checked against this oracle in tests/test_gpu_frame.py.
"""
import numpy as np
import pytest

TUM1 = (517.306408, 516.469215, 318.643040, 255.313989, 0.262383, -0.953104, -0.005358,
        0.002628, 1.163314)                       # Examples/Monocular/TUM1.yaml
EUROC = (458.654, 457.296, 367.215, 248.375, -0.28340811, 0.07395907, 0.00019359,
         1.76187114e-05, 0.0)                    # Examples/Monocular/EuRoC.yaml
KITTI = (718.856, 718.856, 607.1928, 185.2157, 0.0, 0.0, 0.0, 0.0, 0.0)


def np_undistort(cam, xy):
    """float64 numpy restatement of cvUndistortPointsInternal (P = K, R = I, COUNT 5)."""
    fx, fy, cx, cy, k1, k2, p1, p2, k3 = (np.float64(np.float32(v)) for v in cam)
    x = np.asarray(xy, np.float32).astype(np.float64)
    u, v = x[:, 0].copy(), x[:, 1].copy()
    ifx, ify = 1.0 / fx, 1.0 / fy
    x = (u - cx) * ifx
    y = (v - cy) * ify
    x0, y0 = x.copy(), y.copy()
    z = 0.0
    for _ in range(5):
        r2 = x * x + y * y
        icdist = (1 + ((z * r2 + z) * r2 + z) * r2) / (1 + ((k3 * r2 + k2) * r2 + k1) * r2)
        dx = 2 * p1 * x * y + p2 * (r2 + 2 * x * x) + z * r2 + z * r2 * r2
        dy = p1 * (r2 + 2 * y * y) + 2 * p2 * x * y + z * r2 + z * r2 * r2
        x = (x0 - dx) * icdist
        y = (y0 - dy) * icdist
    xx = fx * x + 0.0 * y + cx
    yy = 0.0 * x + fy * y + cy
    ww = 1.0 / (0.0 * x + 0.0 * y + 1.0)
    return np.stack([(xx * ww).astype(np.float32), (yy * ww).astype(np.float32)], 1)


def distort(cam, xy):
    """OpenCV's forward model (projectPoints' distortion) of undistorted pixels."""
    fx, fy, cx, cy, k1, k2, p1, p2, k3 = (float(v) for v in cam)
    x = (xy[:, 0].astype(np.float64) - cx) / fx
    y = (xy[:, 1].astype(np.float64) - cy) / fy
    r2 = x * x + y * y
    rad = 1 + k1 * r2 + k2 * r2 * r2 + k3 * r2 * r2 * r2
    xd = x * rad + 2 * p1 * x * y + p2 * (r2 + 2 * x * x)
    yd = y * rad + p1 * (r2 + 2 * y * y) + 2 * p2 * x * y
    return np.stack([xd * fx + cx, yd * fy + cy], 1)


def _pts(n, w, h, seed):
    rng = np.random.default_rng(seed)
    xy = np.stack([rng.uniform(0, w, n), rng.uniform(0, h, n)], 1).astype(np.float32)
    corners = np.array([[0, 0], [w, 0], [0, h], [w, h], [w / 2, h / 2]], np.float32)
    return np.concatenate([corners, xy])


@pytest.mark.parametrize("cam,w,h", [(TUM1, 640, 480), (EUROC, 752, 480)])
def test_undistort_points_equal_numpy(oracle, cam, w, h):
    xy = _pts(4000, w, h, 1)
    got = oracle.undistort_points(oracle.camera(*cam), xy)
    ref = np_undistort(cam, xy)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


def test_undistort_inverts_forward_model(oracle):
    # EuRoC's mild barrel distortion: 5 iterations converge well inside the image
    cam = EUROC
    xy = _pts(2000, 752, 480, 2)
    un = oracle.undistort_points(oracle.camera(*cam), xy)
    back = distort(cam, un.astype(np.float64))
    err = np.abs(back - xy).max(1)
    r = np.hypot(xy[:, 0] - 367.2, xy[:, 1] - 248.4)
    assert err[r < 200].max() < 1e-3  # converged (2e-4 px); the corners are not (0.3 px)
    assert np.median(err) < 1e-2


def test_undistort_keypoints_copy_when_k1_zero(oracle):
    kp = np.zeros(50, oracle.KP_DTYPE)
    rng = np.random.default_rng(3)
    kp["x"], kp["y"] = rng.uniform(0, 640, 50), rng.uniform(0, 480, 50)
    kp["angle"], kp["octave"], kp["response"] = rng.uniform(0, 360, 50), rng.integers(0, 8, 50), 9
    # k1 == 0 with other nonzero coefficients: still mvKeysUn = mvKeys (Frame.cc:544)
    cam = oracle.camera(500, 500, 320, 240, 0.0, 0.5, 0.01, 0.01, 0.3)
    out = oracle.undistort_keypoints(cam, kp)
    assert out.tobytes() == kp.tobytes()
    assert oracle.image_bounds(cam, 640, 480) == (0.0, 640.0, 0.0, 480.0)
    cam = oracle.camera(*TUM1)
    out = oracle.undistort_keypoints(cam, kp)
    ref = np_undistort(TUM1, np.stack([kp["x"], kp["y"]], 1))
    assert np.array_equal(out["x"], ref[:, 0]) and np.array_equal(out["y"], ref[:, 1])
    for f in ("size", "angle", "response", "octave", "class_id"):
        assert np.array_equal(out[f], kp[f])


def test_image_bounds_tum1(oracle):
    b = oracle.image_bounds(oracle.camera(*TUM1), 640, 480)
    c = np_undistort(TUM1, np.array([[0, 0], [640, 0], [0, 480], [640, 480]], np.float32))
    assert b == (min(c[0, 0], c[2, 0]), max(c[1, 0], c[3, 0]), min(c[0, 1], c[1, 1]),
                 max(c[2, 1], c[3, 1]))


# ---------------------------------------------------------------- isInFrustum
def rot(rx, ry, rz):
    cx_, sx = np.cos(rx), np.sin(rx)
    cy_, sy = np.cos(ry), np.sin(ry)
    cz, sz = np.cos(rz), np.sin(rz)
    Rx = np.array([[1, 0, 0], [0, cx_, -sx], [0, sx, cx_]])
    Ry = np.array([[cy_, 0, sy], [0, 1, 0], [-sy, 0, cy_]])
    Rz = np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1]])
    return Rz @ Ry @ Rx


def frustum_case(oracle_or_lib, n, seed, nlevels=8, bf=386.1448):
    """A KITTI camera at a random pose and n local map points around its view (a mix of
    visible points and every early-out).  Returns (fcam, mps) as the module's records."""
    rng = np.random.default_rng(seed)
    R = rot(*rng.uniform(-0.3, 0.3, 3))
    Ow = rng.uniform(-50, 50, 3)
    t = -R @ Ow
    Tcw = np.concatenate([R, t[:, None]], 1).astype(np.float32)
    fx, fy, cx, cy = 718.856, 718.856, 607.1928, 185.2157
    lsf = np.float32(np.log(np.float64(np.float32(1.2))))
    fcam = np.zeros((), oracle_or_lib.FRUSTUM_DTYPE)
    fcam["Tcw"] = Tcw.reshape(12)
    for k, val in zip(("fx", "fy", "cx", "cy", "bf", "log_scale_factor"), (fx, fy, cx, cy, bf, lsf)):
        fcam[k] = val
    fcam["nlevels"] = nlevels
    fcam["min_x"], fcam["max_x"], fcam["min_y"], fcam["max_y"] = 0.0, 1241.0, 0.0, 376.0
    mps = np.zeros(n, oracle_or_lib.MAPPOINT_DTYPE)
    # camera-frame points: depth 0.5..80 m (some behind), pixel spread past the image
    z = rng.uniform(-5, 80, n)
    u = rng.uniform(-200, 1450, n)
    v = rng.uniform(-100, 480, n)
    pc = np.stack([(u - cx) * z / fx, (v - cy) * z / fy, z], 1)
    pw = (R.T @ (pc - t).T).T
    mps["x"], mps["y"], mps["z"] = pw[:, 0], pw[:, 1], pw[:, 2]
    # normals: the mean viewing direction, perturbed (some past 60 degrees)
    d = pw - Ow
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    nrm = d + rng.normal(0, 0.6, (n, 3))
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    mps["nx"], mps["ny"], mps["nz"] = nrm[:, 0], nrm[:, 1], nrm[:, 2]
    dist = np.linalg.norm(pw - Ow, axis=1)
    # the scale-invariance range around the true distance (some outside)
    mps["max_dist"] = dist * rng.uniform(0.7, 3.0, n)
    mps["min_dist"] = mps["max_dist"] / np.float32(1.2) ** 7 * rng.uniform(0.3, 5.0, n)
    mps["flags"] = np.where(rng.random(n) < 0.9, 1, 0) | np.where(rng.random(n) < 0.5, 2, 0)
    return Tcw, (fx, fy, cx, cy, bf, lsf, nlevels), fcam, mps


def np_frustum(Tcw, intr, bounds, mps, limit):
    """numpy restatement of Frame::isInFrustum (the oracle's pins): (in_view, u, v, ur,
    level, view_cos) per point."""
    fx, fy, cx, cy, bf, lsf, nlevels = intr
    T = Tcw.astype(np.float64)
    P = np.stack([mps["x"], mps["y"], mps["z"]], 1)
    tcw = Tcw[:, 3]
    Pc = np.zeros_like(P)
    Ow = np.zeros(3, np.float32)
    for r in range(3):
        acc = np.zeros(len(P))
        for k in range(3):
            acc = acc + T[r, k] * P[:, k].astype(np.float64)
        Pc[:, r] = (acc * 1.0 + np.float64(tcw[r])).astype(np.float32)
        o = 0.0
        for k in range(3):
            o = o + T[k, r] * np.float64(tcw[k])
        Ow[r] = np.float32(o * -1.0)
    f32 = np.float32
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        invz = f32(1.0) / Pc[:, 2]
        u = f32(fx) * Pc[:, 0] * invz + f32(cx)
        v = f32(fy) * Pc[:, 1] * invz + f32(cy)
        PO = (P - Ow).astype(np.float32)
        s = np.zeros(len(P))
        for k in range(3):
            s = s + PO[:, k].astype(np.float64) * PO[:, k].astype(np.float64)
        dist = np.sqrt(s).astype(np.float32)
        dot = np.zeros(len(P))
        for k, nm in enumerate(("nx", "ny", "nz")):
            dot = dot + PO[:, k].astype(np.float64) * mps[nm].astype(np.float64)
        vc = (dot / dist.astype(np.float64)).astype(np.float32)
        ratio = mps["max_dist"] / dist
        lvl = np.ceil(np.log(ratio.astype(np.float64)) / np.float64(np.float32(lsf)))
    ok = (mps["flags"] & 1) != 0
    ok &= ~(Pc[:, 2] < 0)
    ok &= ~((u < bounds[0]) | (u > bounds[1]) | (v < bounds[2]) | (v > bounds[3]))
    ok &= ~((dist < f32(0.8) * mps["min_dist"]) | (dist > f32(1.2) * mps["max_dist"]))
    ok &= ~(vc < f32(limit))
    lvl = np.clip(np.nan_to_num(lvl, nan=0, posinf=99, neginf=-99), 0, nlevels - 1).astype(np.int32)
    ur = u - f32(bf) * invz
    return ok, u, v, ur, lvl, vc


@pytest.mark.parametrize("seed", range(4))
def test_is_in_frustum_equals_numpy(oracle, seed):
    Tcw, intr, fcam, mps = frustum_case(oracle, 6000, seed)
    proj, nv = oracle.is_in_frustum(fcam, mps, 0.5)
    ok, u, v, ur, lvl, vc = np_frustum(Tcw, intr, (0.0, 1241.0, 0.0, 376.0), mps, 0.5)
    assert nv == ok.sum()
    assert np.array_equal((proj["flags"] & 1) != 0, ok)
    assert np.array_equal(proj["flags"] & 2, mps["flags"] & 2)
    for got, ref in ((proj["u"], u), (proj["v"], v), (proj["ur"], ur), (proj["view_cos"], vc)):
        assert np.array_equal(got[ok].view(np.uint32), ref[ok].view(np.uint32))
    assert np.array_equal(proj["level"][ok], lvl[ok])
    # a mix of outcomes: visible points at several levels and every early-out hit
    assert 200 < nv < 5000 and len(np.unique(proj["level"][ok])) >= 4


def test_is_in_frustum_keeps_stale_members(oracle):
    Tcw, intr, fcam, mps = frustum_case(oracle, 500, 9)
    before = np.zeros(len(mps), oracle.MP_DTYPE)
    before["u"], before["level"], before["flags"] = 12.5, 3, 1
    proj, nv = oracle.is_in_frustum(fcam, mps, 0.5, proj=before)
    out = (proj["flags"] & 1) == 0
    assert out.sum() > 0 and np.all(proj["u"][out] == 12.5) and np.all(proj["level"][out] == 3)


# ------------------------------------------------- ComputeDistinctiveDescriptors
def np_distinctive(desc):
    n = len(desc)
    if n == 0:
        return -1
    bits = np.unpackbits(desc, axis=1)
    D = (bits[:, None, :] != bits[None, :, :]).sum(2)
    med = np.sort(D, axis=1)[:, int(0.5 * (n - 1))]
    return int(np.argmin(med))  # the first minimum = strict < over rows in order


def distinctive_case(n, seed, near=True):
    """n observation descriptors of one map point: noisy copies of one descriptor (the
    realistic case) or unrelated ones."""
    rng = np.random.default_rng(seed)
    base = rng.integers(0, 256, 32, dtype=np.uint8)
    d = np.repeat(base[None], n, 0)
    if near:
        flips = rng.random((n, 256)) < rng.uniform(0.02, 0.2, (n, 1))
        d ^= np.packbits(flips, axis=1)
    else:
        d = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    return d


@pytest.mark.parametrize("n", [1, 2, 3, 4, 7, 33, 64, 65, 130, 513, 700])
def test_distinctive_equals_numpy(oracle, n):
    for seed in range(3):
        d = distinctive_case(n, seed + 10 * n, near=seed != 2)
        assert oracle.distinctive_descriptor(d) == np_distinctive(d)


def test_distinctive_ties_first_row(oracle):
    # all rows identical: every median 0, row 0 wins; two clusters of equal size: ties
    d = np.repeat(np.arange(32, dtype=np.uint8)[None], 5, 0)
    assert oracle.distinctive_descriptor(d) == 0
    a = np.zeros(32, np.uint8)
    b = np.full(32, 255, np.uint8)
    d = np.stack([b, a, b, a])  # medians: row 0: sort(0,256,0,256)[1] = 0 ... all 0 -> 0
    assert oracle.distinctive_descriptor(d) == np_distinctive(d) == 0
    assert oracle.distinctive_descriptor(np.zeros((0, 32), np.uint8)) == -1


def test_distinctive_pool_batch(oracle):
    rng = np.random.default_rng(5)
    pool = rng.integers(0, 256, (3000, 32), dtype=np.uint8)
    counts = rng.integers(0, 40, 200)
    off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)
    rows = rng.integers(0, 3000, off[-1]).astype(np.int32)
    best = oracle.distinctive_descriptors(pool, rows, off)
    for p in range(200):
        assert best[p] == np_distinctive(pool[rows[off[p]:off[p + 1]]])


# ------------------------------------------------------------------ ComputeStereoFromRGBD
TUM_MBF = 40.0  # TUM1.yaml Camera.bf
TUM_DEPTH_FACTOR = np.float32(1.0) / np.float32(5000.0)  # 1 / DepthMapFactor


def rgbd_case(mod, seed, kind="u16", n=1000, w=640, h=480):
    """a depth image (TUM-style raw uint16 with holes, or float metres with holes / NaN) and
    keypoints over the whole image incl. its last row / column and just outside it"""
    rng = np.random.default_rng(seed)
    if kind == "u16":
        depth = rng.integers(500, 40000, (h, w)).astype(np.uint16)
        depth[rng.random((h, w)) < 0.15] = 0
    else:
        depth = rng.uniform(0.3, 8.0, (h, w)).astype(np.float32)
        depth[rng.random((h, w)) < 0.1] = 0
        depth[rng.random((h, w)) < 0.02] = np.nan
        depth[rng.random((h, w)) < 0.02] = -1.0
    kps = np.zeros(n, mod.KP_DTYPE)
    kps["x"] = rng.uniform(0, w, n)
    kps["y"] = rng.uniform(0, h, n)
    kps["x"][:4] = [w - 0.25, 0.0, w + 0.5, -1.5]
    kps["y"][:4] = [h - 0.75, 0.0, 10.0, 10.0]
    kps["octave"] = rng.integers(0, 8, n)
    kun = kps.copy()
    kun["x"] = kps["x"] + rng.normal(0, 2, n)
    kun["y"] = kps["y"] + rng.normal(0, 2, n)
    return depth, kps, kun


def np_rgbd(depth, factor, kps, kun, mbf):
    h, w = depth.shape
    u = np.trunc(kps["x"]).astype(np.int64)
    v = np.trunc(kps["y"]).astype(np.int64)
    ok = (u >= 0) & (u < w) & (v >= 0) & (v < h)
    raw = np.zeros(len(kps), np.float32)
    raw[ok] = depth[v[ok], u[ok]].astype(np.float32)
    scale = depth.dtype == np.uint16 or abs(float(np.float32(factor) - np.float32(1.0))) > 1e-5
    with np.errstate(invalid="ignore"):
        d = (raw * np.float32(factor)).astype(np.float32) if scale else raw
        good = ok & (d > 0)
    ur = np.full(len(kps), -1, np.float32)
    dd = np.full(len(kps), -1, np.float32)
    dd[good] = d[good]
    ur[good] = kun["x"][good] - np.float32(mbf) / d[good]
    return ur, dd


@pytest.mark.parametrize("kind,factor", [("u16", TUM_DEPTH_FACTOR), ("u16", 1.0),
                                         ("f32", 1.0), ("f32", 0.5)])
def test_rgbd_stereo_equals_numpy(oracle, kind, factor):
    depth, kps, kun = rgbd_case(oracle, 3, kind)
    ur, dd = oracle.rgbd_stereo(depth, factor, kps, kun, TUM_MBF)
    rur, rdd = np_rgbd(depth, factor, kps, kun, TUM_MBF)
    assert np.array_equal(ur.view(np.uint32), rur.view(np.uint32))
    assert np.array_equal(dd.view(np.uint32), rdd.view(np.uint32))
    assert (dd > 0).sum() > len(kps) // 2 and (dd == -1).sum() > 20
    assert dd[2] == -1 and dd[3] == -1  # outside the image


def test_predict_scale_fast_path_logic():
    """csrc/frame_device.h predict_scale: the float quotient decides ceil(log(r) / L) unless it
    lies within 1e-3 of an integer (then the double expression runs).  Checked here with
    numpy's float32 log over a million ratios, dense around every level boundary 1.2^k."""
    rng = np.random.default_rng(7)
    L32 = np.float32(np.log(np.float64(np.float32(1.2))))
    k = rng.integers(-3, 12, 500000)
    near = (np.float64(1.2) ** k * (1 + rng.normal(0, 1e-6, k.size))).astype(np.float32)
    wide = np.exp(rng.uniform(-3, 4, 500000)).astype(np.float32)
    # |q| up to the fast path's limit of 64 (the float quotient's error grows with |q|: about
    # 1e-5 near 64, still far inside the 1e-3 margin)
    kf = rng.integers(-64, 64, 200000)
    far = (np.float64(1.2) ** kf * (1 + rng.normal(0, 1e-4, kf.size))).astype(np.float32)
    big = np.exp(rng.uniform(-64, 64, 200000) * np.float64(L32)).astype(np.float32)
    r = np.concatenate([near, wide, (np.float64(1.2) ** np.arange(-3, 12)).astype(np.float32),
                        far, big])
    qf = np.log(r) / L32
    fl = np.floor(qf)
    fast = (np.abs(qf) < 64) & (qf - fl > np.float32(1e-3)) & (qf - fl < np.float32(0.999))
    exact = np.ceil(np.log(r.astype(np.float64)) / np.float64(L32))
    assert np.array_equal((fl + 1)[fast], exact[fast])
    assert fast[near.size:near.size + wide.size].mean() > 0.99 and (~fast).sum() > 1000
