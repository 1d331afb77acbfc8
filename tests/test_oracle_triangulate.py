"""CPU: the oracle's CreateNewMapPoints triangulation (oracle/mapping_oracle.c, orc_triangulate
and orc_tri_geometry; src/LocalMapping.cc:293-560 and ComputeF12 :690-707) pinned against

  - the host libm for the float transcendental it restates (glibc atan2f: every sampled pair
    bit-equal; cosf is pinned in test_oracle_kats.py);
  - numpy for ComputeF12 (float64 K1^-T [t12]x R12 K2^-1, tolerance) and for the cv::SVD
    stand-in (the null vector of the 4x4 system vs numpy's SVD, up to sign, tolerance);
  - a second, pure-Python restatement of the triangulation loop (float32 scalars in the
    reference's evaluation order, the host libm's atan2f / cosf, the oracle's null vector):
    every status and every new point bit-equal;
  - and the reference's own geometry: a point triangulated from exact projections lands on the
    generating 3-D point (tolerance), each rejection branch fires on the pairs built for it.

cv::SVD::compute's own bits are not reproduced (OpenCV is not in this image): positions from
the linear triangulation are parity-unpinned against OpenCV, pinned here to numpy's SVD within
a float tolerance.  The GPU kernel is checked bit-exact against this oracle in
tests/test_gpu_mapping.py.
"""
import ctypes
import ctypes.util

import numpy as np
import pytest

KITTI_K = (718.856, 718.856, 607.1928, 185.2157)
BF = 386.1448
F32 = np.float32


def _libm():
    m = ctypes.CDLL(ctypes.util.find_library("m"))
    m.atan2f.argtypes = [ctypes.c_float, ctypes.c_float]
    m.atan2f.restype = ctypes.c_float
    m.cosf.argtypes = [ctypes.c_float]
    m.cosf.restype = ctypes.c_float
    return m


def _rot(rng, s):
    w = rng.normal(0, s, 3)
    th = np.linalg.norm(w)
    k = w / max(th, 1e-12)
    Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * Kx + (1 - np.cos(th)) * Kx @ Kx


def tri_pair_case(O, seed, n=1000, baseline=1.2, stereo=0.6, w=1241, h=376, noise=0.5,
                  distort=0.02):
    """O: a module with KP_DTYPE and KF_CAM_DTYPE / KF_CAMERA_DTYPE (the oracle or liborbg's
    _lib).  Two KeyFrames of one camera seeing n 3-D points and a matches12 list with the cases
    CreateNewMapPoints rejects: wrong matches (reprojection), far points (parallax), points
    behind KF2, octave jumps (scale consistency), monocular and stereo features, mvKeys !=
    mvKeysUn (UnprojectStereo reads mvKeys).  Returns (kf1, kf2, c1, c2, m12, sf, s2, Xw)."""
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy = KITTI_K
    sf = (F32(1.2) ** np.arange(8)).astype(F32)
    s2 = (sf * sf).astype(F32)
    R1w = _rot(rng, 0.3)
    t1w = rng.uniform(-10, 10, 3)
    R21 = _rot(rng, 0.05)
    base = np.array([baseline, rng.uniform(-0.1, 0.1), rng.uniform(-0.4, 0.4)])
    t21 = -R21 @ base
    R2w, t2w = R21 @ R1w, R21 @ t1w + t21
    z = np.where(rng.random(n) < 0.1, rng.uniform(300, 3000, n), rng.uniform(3, 60, n))
    u1 = rng.uniform(10, w - 10, n)
    v1 = rng.uniform(10, h - 10, n)
    X1 = np.stack([(u1 - cx) * z / fx, (v1 - cy) * z / fy, z], 1)
    Xw = (R1w.T @ (X1 - t1w).T).T
    X2 = (R2w @ Xw.T).T + t2w
    behind = X2[:, 2] <= 0.1
    X2[behind, 2] = 1.0
    u2 = fx * X2[:, 0] / X2[:, 2] + cx
    v2 = fy * X2[:, 1] / X2[:, 2] + cy
    oct1 = rng.integers(0, 8, n)
    jump = rng.random(n) < 0.05
    oct2 = np.where(jump, (oct1 + 4) % 8, np.clip(oct1 + rng.integers(-1, 2, n), 0, 7))
    nz = rng.normal(0, noise, (n, 4)) * np.sqrt(s2[oct2])[:, None]

    def kps(u, v, octv):
        k = np.zeros(n, O.KP_DTYPE)
        k["x"], k["y"], k["octave"] = u, v, octv
        k["size"], k["response"], k["angle"] = 31, 20, rng.uniform(0, 360, n)
        return k

    kp1 = kps(u1 + nz[:, 0], v1 + nz[:, 1], oct1)
    kp2 = kps(u2 + nz[:, 2], v2 + nz[:, 3], oct2)
    # mvKeys: the distorted positions (a small radial shift), mvKeysUn above
    raw1, raw2 = kp1.copy(), kp2.copy()
    for raw, u, v in ((raw1, u1, v1), (raw2, u2, v2)):
        r2 = ((u - cx) / fx) ** 2 + ((v - cy) / fy) ** 2
        raw["x"] = (u - cx) * (1 - distort * r2) + cx
        raw["y"] = (v - cy) * (1 - distort * r2) + cy
    # stereo: mvuRight = u - bf / z (a little disparity noise), mvDepth = bf / disparity
    def stereo_of(kp, zz):
        st = rng.random(n) < stereo
        disp = BF / zz + rng.normal(0, 0.6 * noise, n)
        st &= disp > 0.5
        ur = np.where(st, kp["x"] - disp, -1).astype(F32)
        dp = np.where(st, F32(BF) / disp.astype(F32), -1).astype(F32)
        return ur, dp

    ur1, d1 = stereo_of(kp1, z)
    ur2, d2 = stereo_of(kp2, X2[:, 2])
    # matches: KF2's order shuffled; 8% wrong partners, 10% unmatched
    perm = rng.permutation(n)
    inv = np.argsort(perm)
    kp2, raw2, ur2, d2 = kp2[perm], raw2[perm], ur2[perm], d2[perm]
    m12 = inv.astype(np.int32)
    wrong = rng.random(n) < 0.08
    m12[wrong] = rng.integers(0, n, wrong.sum())
    m12[rng.random(n) < 0.1] = -1
    kf1 = dict(kps=kp1, kps_raw=raw1, uright=ur1, depth=d1)
    kf2 = dict(kps=kp2, kps_raw=raw2, uright=ur2, depth=d2)
    mb = BF / fx
    c1 = kf_cam(O, np.concatenate([R1w, t1w[:, None]], 1), fx, fy, cx, cy, mb, BF)
    c2 = kf_cam(O, np.concatenate([R2w, t2w[:, None]], 1), fx, fy, cx, cy, mb, BF)
    return kf1, kf2, c1, c2, m12, sf, s2, Xw


def kf_cam(O, Tcw, fx, fy, cx, cy, mb, mbf):
    """the camera record (the oracle's KF_CAM_DTYPE or liborbg's KF_CAMERA_DTYPE: one layout)"""
    dt = getattr(O, "KF_CAM_DTYPE", None) or O.KF_CAMERA_DTYPE
    c = np.zeros((), dt)
    c["Tcw"] = np.asarray(Tcw, F32).reshape(-1)[:12]
    c["fx"], c["fy"], c["cx"], c["cy"] = fx, fy, cx, cy
    c["invfx"], c["invfy"] = F32(1.0) / F32(fx), F32(1.0) / F32(fy)
    c["mb"], c["mbf"] = mb, mbf
    return c


# ------------------------------------------------------------- pure-Python restatement
def _gemm_rows(M, x, alpha=1.0, c=None, transpose=False):
    """cv::gemm of a 3x3 float block with a float 3-vector: double sums, one rounding."""
    out = []
    for i in range(3):
        t = 0.0
        for k in range(3):
            t += float(M[k, i] if transpose else M[i, k]) * float(x[k])
        t *= alpha
        if c is not None:
            t += float(c[i])
        out.append(F32(t))
    return np.array(out, F32)


def _dot(a, b):
    s = 0.0
    for k in range(3):
        s += float(a[k]) * float(b[k])
    return s


def py_triangulate(O, kf1, kf2, c1, c2, m12, sf, s2, scale_factor):
    """CreateNewMapPoints' triangulation loop (LocalMapping.cc:395-560), float32 scalars."""
    m = _libm()
    T1 = c1["Tcw"].reshape(3, 4)
    T2 = c2["Tcw"].reshape(3, 4)
    Ow1 = _gemm_rows(T1[:, :3], T1[:, 3], -1.0, transpose=True)
    Ow2 = _gemm_rows(T2[:, :3], T2[:, 3], -1.0, transpose=True)
    ratio = F32(1.5) * F32(scale_factor)
    n = len(m12)
    X = np.zeros((n, 3), F32)
    st = np.zeros(n, np.int8)
    for i in range(n):
        j = int(m12[i])
        if j < 0:
            continue
        st[i], x = _tri_one(O, m, kf1, kf2, c1, c2, T1, T2, Ow1, Ow2, i, j, sf, s2, ratio)
        if st[i] == O.TRI_NEW:
            X[i] = x
    return int((st == O.TRI_NEW).sum()), X, st


def _tri_one(O, m, kf1, kf2, c1, c2, T1, T2, Ow1, Ow2, i, j, sf, s2, ratio):
    kp1, kp2 = kf1["kps"][i], kf2["kps"][j]
    ur1, ur2 = F32(kf1["uright"][i]), F32(kf2["uright"][j])
    st1, st2 = ur1 >= 0, ur2 >= 0
    xn1 = np.array([(kp1["x"] - c1["cx"]) * c1["invfx"], (kp1["y"] - c1["cy"]) * c1["invfy"], 1], F32)
    xn2 = np.array([(kp2["x"] - c2["cx"]) * c2["invfx"], (kp2["y"] - c2["cy"]) * c2["invfy"], 1], F32)
    ray1 = _gemm_rows(T1[:, :3], xn1, transpose=True)
    ray2 = _gemm_rows(T2[:, :3], xn2, transpose=True)
    cpr = F32(_dot(ray1, ray2) / (np.sqrt(_dot(ray1, ray1)) * np.sqrt(_dot(ray2, ray2))))
    cps = F32(cpr + F32(1))
    cps1 = cps2 = cps
    if st1:
        cps1 = F32(m.cosf(F32(2) * F32(m.atan2f(F32(c1["mb"]) / F32(2), F32(kf1["depth"][i])))))
    elif st2:
        cps2 = F32(m.cosf(F32(2) * F32(m.atan2f(F32(c2["mb"]) / F32(2), F32(kf2["depth"][j])))))
    cps = min(cps1, cps2)
    if cpr < cps and cpr > 0 and (st1 or st2 or cpr < 0.9998):
        A = np.zeros((4, 4), F32)
        for r, (T, xv) in enumerate(((T1, xn1[0]), (T1, xn1[1]), (T2, xn2[0]), (T2, xn2[1]))):
            row = r % 2
            A[r] = (T[2] * xv + T[row] * F32(-1)) + F32(0)
        v = O.tri_nullvec(A).astype(F32)
        if v[3] == 0:
            return O.TRI_W0, None
        a = F32(1.0 / float(v[3]))
        x3 = (v[:3] * a + F32(0)).astype(F32)
    elif st1 and cps1 < cps2:
        zz = F32(kf1["depth"][i])
        kr = kf1["kps_raw"][i]
        xc = np.array([(kr["x"] - c1["cx"]) * zz * c1["invfx"], (kr["y"] - c1["cy"]) * zz * c1["invfy"], zz], F32)
        x3 = _gemm_rows(T1[:, :3], xc, c=Ow1, transpose=True)
    elif st2 and cps2 < cps1:
        zz = F32(kf2["depth"][j])
        kr = kf2["kps_raw"][j]
        xc = np.array([(kr["x"] - c2["cx"]) * zz * c2["invfx"], (kr["y"] - c2["cy"]) * zz * c2["invfy"], zz], F32)
        x3 = _gemm_rows(T2[:, :3], xc, c=Ow2, transpose=True)
    else:
        return O.TRI_PARALLAX, None
    z1 = F32(_dot(T1[2, :3], x3) + float(T1[2, 3]))
    if z1 <= 0:
        return O.TRI_Z1, None
    z2 = F32(_dot(T2[2, :3], x3) + float(T2[2, 3]))
    if z2 <= 0:
        return O.TRI_Z2, None
    for (T, c, kp, ur, stv, zz, code) in ((T1, c1, kp1, ur1, st1, z1, O.TRI_REPROJ1),
                                         (T2, c2, kp2, ur2, st2, z2, O.TRI_REPROJ2)):
        sig = F32(s2[kp["octave"]])
        xx = F32(_dot(T[0, :3], x3) + float(T[0, 3]))
        yy = F32(_dot(T[1, :3], x3) + float(T[1, 3]))
        iz = F32(1.0 / float(zz))
        u = F32(c["fx"]) * xx * iz + F32(c["cx"])
        v = F32(c["fy"]) * yy * iz + F32(c["cy"])
        ex, ey = u - kp["x"], v - kp["y"]
        if not stv:
            if float(ex * ex + ey * ey) > 5.991 * float(sig):
                return code, None
        else:
            exr = (u - F32(c1["mbf"]) * iz) - ur  # both use the current KeyFrame's mbf (:528)
            if float(ex * ex + ey * ey + exr * exr) > 7.8 * float(sig):
                return code, None
    n1, n2 = (x3 - Ow1).astype(F32), (x3 - Ow2).astype(F32)
    d1, d2 = F32(np.sqrt(_dot(n1, n1))), F32(np.sqrt(_dot(n2, n2)))
    if d1 == 0 or d2 == 0:
        return O.TRI_DIST0, None
    rd = d2 / d1
    ro = F32(sf[kp1["octave"]]) / F32(sf[kp2["octave"]])
    if rd * ratio < ro or rd > ro * ratio:
        return O.TRI_SCALE, None
    return O.TRI_NEW, x3


# ------------------------------------------------------------------------------ tests
def test_atan2f_matches_libm(oracle):
    """orc_atan2f (glibc's fdlibm-derived atan2f, its |x| >= 2^25 bound of atanf) is the host
    libm bit for bit: 12M sampled pairs in C plus the special values."""
    for seed in (1, 7, 12345):
        assert oracle.atan2f_check(seed, 4_000_000) == 0
    m = _libm()
    sp = [0.0, -0.0, 1.0, -1.0, 1e-30, -1e-30, 1e30, 2.0 ** 25, 2.0 ** 26, float("inf"),
          float("-inf"), 3.4e38, 1.4e-45, 0.19345, 45.0]
    for y in sp:
        for x in sp:
            a, b = F32(m.atan2f(y, x)), F32(oracle.atan2f(y, x))
            assert a.tobytes() == b.tobytes(), (y, x, a, b)
    assert np.isnan(oracle.atan2f(float("nan"), 1.0))


@pytest.mark.parametrize("seed", range(4))
def test_compute_f12_matches_numpy(oracle, seed):
    kf1, kf2, c1, c2, m12, sf, s2, Xw = tri_pair_case(oracle, seed, n=50)
    g = oracle.tri_geometry(c1, c2)
    T1 = c1["Tcw"].reshape(3, 4).astype(np.float64)
    T2 = c2["Tcw"].reshape(3, 4).astype(np.float64)
    R12 = T1[:, :3] @ T2[:, :3].T
    t12 = -R12 @ T2[:, 3] + T1[:, 3]
    tx = np.array([[0, -t12[2], t12[1]], [t12[2], 0, -t12[0]], [-t12[1], t12[0], 0]])
    K1 = np.array([[c1["fx"], 0, c1["cx"]], [0, c1["fy"], c1["cy"]], [0, 0, 1]], np.float64)
    K2 = np.array([[c2["fx"], 0, c2["cx"]], [0, c2["fy"], c2["cy"]], [0, 0, 1]], np.float64)
    F = np.linalg.inv(K1.T) @ tx @ R12 @ np.linalg.inv(K2)
    assert np.allclose(g["F12"].reshape(3, 3), F, rtol=2e-5, atol=2e-5 * np.abs(F).max())
    assert np.allclose(g["Cw1"], -T1[:, :3].T @ T1[:, 3], atol=1e-4)
    assert np.array_equal(g["Tcw2"], c2["Tcw"])
    # epipolar constraint of the exact projections: x1^T F12 x2 ~ 0
    x1 = (K1 @ (T1[:, :3] @ Xw.T + T1[:, 3:])).T
    x2 = (K2 @ (T2[:, :3] @ Xw.T + T2[:, 3:])).T
    x1, x2 = x1 / x1[:, 2:], x2 / x2[:, 2:]
    e = np.einsum("ni,ij,nj->n", x1, g["F12"].reshape(3, 3).astype(np.float64), x2)
    line = x1 @ g["F12"].reshape(3, 3).astype(np.float64)
    assert np.all(np.abs(e) / np.hypot(line[:, 0], line[:, 1]) < 0.05)


def test_nullvec_matches_numpy_svd(oracle):
    """the cv::SVD stand-in vs numpy's SVD: the same null direction (sign and scale free)."""
    rng = np.random.default_rng(3)
    kf1, kf2, c1, c2, m12, sf, s2, Xw = tri_pair_case(oracle, 11, n=400)
    T1, T2 = c1["Tcw"].reshape(3, 4), c2["Tcw"].reshape(3, 4)
    worst = 0.0
    for i in rng.permutation(400)[:200]:
        j = m12[i]
        if j < 0:
            continue
        xn1 = [(kf1["kps"]["x"][i] - c1["cx"]) * c1["invfx"], (kf1["kps"]["y"][i] - c1["cy"]) * c1["invfy"]]
        xn2 = [(kf2["kps"]["x"][j] - c2["cx"]) * c2["invfx"], (kf2["kps"]["y"][j] - c2["cy"]) * c2["invfy"]]
        A = np.stack([T1[2] * xn1[0] - T1[0], T1[2] * xn1[1] - T1[1],
                      T2[2] * xn2[0] - T2[0], T2[2] * xn2[1] - T2[1]]).astype(F32)
        v = oracle.tri_nullvec(A)
        vt = np.linalg.svd(A.astype(np.float64))[2][3]
        assert abs(np.linalg.norm(v) - 1) < 1e-12
        d = min(np.abs(v - vt).max(), np.abs(v + vt).max())
        sv = np.linalg.svd(A.astype(np.float64), compute_uv=False)
        worst = max(worst, d * sv[2] / sv[0])  # conditioning-scaled
        assert d < 1e-9 * sv[0] / max(sv[2] - sv[3], 1e-300) + 1e-9
    assert worst < 1e-9


@pytest.mark.parametrize("seed,baseline,stereo", [(0, 1.2, 0.6), (1, 0.3, 0.0), (2, 2.5, 1.0),
                                                  (3, 0.05, 0.5)])
def test_triangulate_equals_python(oracle, seed, baseline, stereo):
    kf1, kf2, c1, c2, m12, sf, s2, Xw = tri_pair_case(oracle, seed, n=500, baseline=baseline,
                                                      stereo=stereo)
    n, X, st = oracle.triangulate(kf1, kf2, c1, c2, m12, sf, s2, 1.2)
    rn, rX, rst = py_triangulate(oracle, kf1, kf2, c1, c2, m12, sf, s2, 1.2)
    assert np.array_equal(st, rst)
    assert n == rn and np.array_equal(X.view(np.uint32), rX.view(np.uint32))
    assert np.all(st[m12 < 0] == oracle.TRI_NONE)


def test_triangulate_geometry_and_branches(oracle):
    """new points land on the generating 3-D points; each rejection branch of the reference
    fires where the case builds it."""
    O = oracle
    # noise-free observations: every new point is the generating one (float rounding)
    kf1, kf2, c1, c2, m12, sf, s2, Xw = tri_pair_case(O, 20, n=2000, noise=0.0, distort=0.0)
    n, X, st = O.triangulate(kf1, kf2, c1, c2, m12, sf, s2, 1.2)
    good = st == O.TRI_NEW
    T1 = c1["Tcw"].reshape(3, 4).astype(np.float64)
    depth = (T1[:, :3] @ Xw.T + T1[:, 3:])[2]
    err = np.linalg.norm(X[good] - Xw[good], axis=1) / depth[good]
    assert n > 1000 and np.median(err) < 1e-4 and np.percentile(err, 90) < 1e-3
    kf1, kf2, c1, c2, m12, sf, s2, Xw = tri_pair_case(O, 21, n=3000)
    n, X, st = O.triangulate(kf1, kf2, c1, c2, m12, sf, s2, 1.2)
    assert n > 1000
    codes = set(np.unique(st).tolist())
    for c in (O.TRI_NONE, O.TRI_NEW, O.TRI_PARALLAX, O.TRI_REPROJ1, O.TRI_REPROJ2, O.TRI_SCALE):
        assert c in codes, c
    # KF2 = KF1 (no baseline), monocular: no parallax anywhere -> nothing new
    kfm1 = dict(kf1, uright=np.full(3000, -1, F32))
    ident = np.arange(3000, dtype=np.int32)
    n0, _, st0 = O.triangulate(kfm1, kfm1, c1, c1, ident, sf, s2, 1.2)
    assert n0 == 0 and np.all(st0 == O.TRI_PARALLAX)
    # ... stereo in KF1: UnprojectStereo of KF1 for every pair with depth (cosParallaxStereo1
    # < cosParallaxStereo2 = cosParallaxRays + 1)
    n1, X1, st1 = O.triangulate(kf1, dict(kfm1), c1, c1, ident, sf, s2, 1.2)
    assert n1 > 0.5 * (kf1["uright"] >= 0).sum()
    assert np.all(st1[kf1["uright"] < 0] == O.TRI_PARALLAX)


def test_triangulate_empty(oracle):
    kf1, kf2, c1, c2, m12, sf, s2, Xw = tri_pair_case(oracle, 4, n=20)
    n, X, st = oracle.triangulate(kf1, kf2, c1, c2, np.full(20, -1, np.int32), sf, s2, 1.2)
    assert n == 0 and np.all(st == 0) and np.all(X == 0)
    e = {k: v[:0] for k, v in kf1.items()}
    n, X, st = oracle.triangulate(e, kf2, c1, c2, np.zeros(0, np.int32), sf, s2, 1.2)
    assert n == 0 and len(st) == 0
