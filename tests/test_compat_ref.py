"""The reference-facing drop-in layer: ORB_SLAM2::ORBextractor with the reference's OpenCV
signatures (lazy mvImagePyramid) and orb_slam2_test_amd/compat/orbg_reference.hpp's
ORBmatcher / Optimizer call sites over stand-ins of the reference's Frame / KeyFrame /
MapPoint, driven by tests/compat_ref_selftest.cpp.  OpenCV is absent here, so the program
compiles against tests/compat_stub/ (a test-only stand-in of the cv:: subset the layer uses).

CPU: the program and both headers compile (g++ -Wall -Werror).  GPU: it runs on two
synthetic KITTI-shaped frames and checks the drop-ins against the plain-buffer layer (same
matches, same prev positions, same H blocks) and the reference's invariants (matched map
points within TH_HIGH, hessian blocks in vertex-id order), and replays its SearchByBoW,
UndistortKeyPoints / ComputeImageBounds and SearchForTriangulation calls through the oracle;
the isInFrustum loop of SearchLocalPoints, Fuse with its sequential map update (Replace /
AddObservation, re-checks) and ComputeDistinctiveDescriptors are checked in the program.
"""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "orb_slam2_test_amd", "lib")
SRC = os.path.join(ROOT, "tests", "compat_ref_selftest.cpp")


def test_drop_in_layer_compiles(tmp_path):
    out = tmp_path / "compat_ref_selftest"
    cmd = ["g++", "-std=c++17", "-O1", "-Wall", "-Werror",
           "-I" + os.path.join(ROOT, "include"),
           "-I" + os.path.join(ROOT, "orb_slam2_test_amd", "compat"),
           "-I" + os.path.join(ROOT, "tests", "compat_stub"), SRC, "-L" + LIB, "-lorbg",
           "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]


@pytest.mark.gpu
def test_drop_in_layer_runs(tmp_path):
    from orb_slam2_test_amd import synthetic as S
    exe = os.path.join(LIB, "compat_ref_selftest")
    assert os.path.exists(exe), "built by orb_slam2_test_amd/csrc/Makefile (build())"
    fr = S.sequence(2, 376, 1241, seed=S.DEFAULT_SEED + 21)
    paths = []
    for i in range(2):
        p = tmp_path / ("f%d.raw" % i)
        np.ascontiguousarray(fr[i]).tofile(p)
        paths.append(str(p))
    out = tmp_path / "out"
    out.mkdir()
    r = subprocess.run([exe, paths[0], paths[1], "1241", "376", str(out)], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert "compat_ref ok" in r.stdout
    # SearchByBoW through the drop-in (KeyFrame / Frame stand-ins, grid FeatureVectors):
    # replayed through the oracle on the inputs the program wrote
    from oracle import pyoracle as O

    def rd(name, dt):
        return np.fromfile(str(out / name), dt)
    kd, fd = rd("bow_kd.u8", np.uint8).reshape(-1, 32), rd("bow_fd.u8", np.uint8).reshape(-1, 32)
    kfv = (rd("bow_kn.i32", np.int32), rd("bow_ko.i32", np.int32), rd("bow_kf.i32", np.int32))
    ffv = (rd("bow_fn.i32", np.int32), rd("bow_fo.i32", np.int32), rd("bow_ff.i32", np.int32))
    rn, ref = O.search_by_bow(kd, rd("bow_ka.f32", np.float32), rd("bow_kv.u8", np.uint8), kfv,
                              fd, rd("bow_fa.f32", np.float32), ffv, nnratio=0.7, check_ori=True)
    assert int(rd("bow_n.i32", np.int32)[0]) == rn
    assert np.array_equal(rd("bow_match.i32", np.int32), ref)
    # Frame::UndistortKeyPoints / ComputeImageBounds (TUM1.yaml's camera) through the drop-in
    cam = O.camera(517.306408, 516.469215, 318.643040, 255.313989, 0.262383, -0.953104,
                   -0.005358, 0.002628, 1.163314)
    und_in = rd("und_in.f32", np.float32).reshape(-1, 2)
    assert np.array_equal(rd("und_out.f32", np.float32).reshape(-1, 2),
                          O.undistort_points(cam, und_in))
    assert tuple(rd("und_bounds.f32", np.float32)) == O.image_bounds(cam, 640, 480)
    # SearchForTriangulation(KA, KB, F12) through the drop-in, replayed on its inputs
    akp, bkp = rd("tri_akp.bin", O.KP_DTYPE), rd("tri_bkp.bin", O.KP_DTYPE)
    kfa = dict(kps=akp, desc=kd, uright=rd("tri_aur.f32", np.float32),
               fv=(rd("tri_an.i32", np.int32), rd("tri_ao.i32", np.int32), rd("tri_af.i32", np.int32)))
    kfb = dict(kps=bkp, desc=fd, uright=rd("tri_bur.f32", np.float32),
               fv=(rd("tri_bn.i32", np.int32), rd("tri_bo.i32", np.int32), rd("tri_bf.i32", np.int32)))
    geo = np.zeros((), O.TRI_GEOM_DTYPE)
    gv = rd("tri_geom.f32", np.float32)
    geo["F12"], geo["Cw1"], geo["Tcw2"] = gv[:9], gv[9:12], gv[12:24]
    geo["fx2"], geo["fy2"], geo["cx2"], geo["cy2"] = gv[24:28]
    p = O.params(nfeatures=2000)
    tn, tm = O.search_for_triangulation(kfa, kfb, geo, np.array(p.scale[:8], np.float32),
                                        np.array(p.sigma2[:8], np.float32), False, False)
    pairs = rd("tri_pairs.i32", np.int32).reshape(-1, 2)
    assert len(pairs) == tn and tn > 20
    assert np.array_equal(pairs[:, 0], np.nonzero(tm >= 0)[0])
    assert np.array_equal(pairs[:, 1], tm[tm >= 0])


def _lba_scene(rng):
    """A LocalBundleAdjustment scene of the reference's shapes: 4 local key frames (one with
    mnId 0, fixed by Optimizer.cc:714), 2 fixed cameras, one bad key frame in neither list that
    still observes points (its edges are dropped, :788), ids out of list order, mono and
    stereo keypoints, world coordinates offset by ~400 m."""
    fx = fy = 718.856
    cx, cy, bf = 607.1928, 185.2157, 386.1448
    ids = [12, 0, 7, 30, 3, 21, 9]
    lists = [1, 1, 1, 1, 0, 0, -1]
    bad = [0, 0, 0, 0, 0, 0, 1]
    nkf, K, nmp = len(ids), 500, 260
    origin = np.array([400.0, -20.0, 150.0])
    Ts = []
    for i in range(nkf):
        ax = rng.normal(size=3)
        ax /= np.linalg.norm(ax)
        ang = rng.uniform(0, 0.1)
        Kx = np.array([[0, -ax[2], ax[1]], [ax[2], 0, -ax[0]], [-ax[1], ax[0], 0]])
        R = np.eye(3) + np.sin(ang) * Kx + (1 - np.cos(ang)) * Kx @ Kx
        C = origin + np.array([rng.normal(0, 0.5), 0, 1.2 * i])
        T = np.zeros((3, 4))
        T[:, :3] = R
        T[:, 3] = -R @ C
        Ts.append(T.astype(np.float32))
    inv2 = np.array([1.0 / np.float32(1.2) ** (2 * l) for l in range(8)], np.float32)
    kp = np.zeros((nkf, K, 4), np.float32)
    kp[:, :, 0] = rng.uniform(0, 1241, (nkf, K))
    kp[:, :, 1] = rng.uniform(0, 376, (nkf, K))
    kp[:, :, 2] = rng.integers(0, 8, (nkf, K))
    kp[:, :, 3] = -1
    used = np.zeros(nkf, int)
    mp = np.zeros((nmp, 4))
    mp[:, 0] = rng.permutation(np.arange(1000, 1000 + 4 * nmp))[:nmp]  # ids out of order
    obs = []
    for j in range(nmp):
        T0 = Ts[rng.integers(0, nkf)].astype(np.float64)
        z = rng.uniform(6, 50)
        xc = np.array([(rng.uniform(50, 1190) - cx) / fx * z, (rng.uniform(20, 356) - cy) / fy * z, z])
        X = T0[:, :3].T @ (xc - T0[:, 3])
        mp[j, 1:] = X.astype(np.float32)
        for i in sorted(rng.choice(nkf, size=int(rng.integers(2, 6)), replace=False)):
            T = Ts[i].astype(np.float64)
            c = T[:, :3] @ mp[j, 1:] + T[:, 3]
            if c[2] <= 0.5:
                continue
            k = used[i]
            used[i] += 1
            noise = rng.normal(0, 1.5, 3) * (8 if rng.random() < 0.1 else 1)
            kp[i, k, 0] = fx * c[0] / c[2] + cx + noise[0]
            kp[i, k, 1] = fy * c[1] / c[2] + cy + noise[1]
            if rng.random() < 0.5:
                kp[i, k, 3] = kp[i, k, 0] - bf / c[2] + noise[2]
            obs.append((j, i, k))
    kf = np.zeros((nkf, 20))
    for i in range(nkf):
        kf[i, :8] = [ids[i], fx, fy, cx, cy, bf, bad[i], lists[i]]
        kf[i, 8:] = Ts[i].reshape(-1)
    return dict(kf=kf, kp=kp, inv2=inv2, mp=mp, obs=np.array(obs, np.int32), K=K)


def _expected_window(oracle, sc):
    """Optimizer::LocalBundleAdjustment's vertices and edges (Optimizer.cc:708-851), built
    here from the scene directly: poses = local key frames then fixed cameras (list order),
    fixed iff fixed camera or mnId == 0; an edge per observation (map point order, then key
    frame order = the std::map<KeyFrame*, size_t> order of the stand-ins) by a listed key frame
    that is not bad; mono iff uRight < 0; Omega = mvInvLevelSigma2[octave]; Huber delta =
    (float)sqrt(5.991) / (float)sqrt(7.815)."""
    from orb_slam2_test_amd import _lib
    kf, kp = sc["kf"], sc["kp"]
    order = [i for i in range(len(kf)) if kf[i, 7] > 0] + [i for i in range(len(kf)) if kf[i, 7] == 0]
    pose_of = {i: n for n, i in enumerate(order)}
    poses = np.zeros(len(order), _lib.POSE_DTYPE)
    for n, i in enumerate(order):
        q, t = oracle.se3_from_tcw(kf[i, 8:].astype(np.float32))
        poses[n]["q"], poses[n]["t"] = q, t
        poses[n]["fixed"] = 1 if (kf[i, 7] == 0 or kf[i, 0] == 0) else 0
    points = sc["mp"][:, 1:].astype(np.float32).astype(np.float64)
    edges = []
    for j in range(len(sc["mp"])):
        for (_, i, k) in sorted([tuple(o) for o in sc["obs"] if o[0] == j], key=lambda o: o[1]):
            if kf[i, 6] or i not in pose_of:
                continue
            e = np.zeros((), _lib.EDGE_DTYPE)
            e["point"], e["pose"] = j, pose_of[i]
            st = kp[i, k, 3] >= 0
            e["stereo"], e["robust"], e["active"] = int(st), 1, 1
            e["obs"][0], e["obs"][1] = kp[i, k, 0], kp[i, k, 1]
            e["obs"][2] = kp[i, k, 3] if st else 0.0
            e["inv_sigma2"] = sc["inv2"][int(kp[i, k, 2])]
            e["fx"], e["fy"], e["cx"], e["cy"], e["bf"] = [np.float32(v) for v in kf[i, 1:6]]
            e["huber_delta"] = np.float32(np.sqrt(7.815 if st else 5.991))
            edges.append(e)
    return order, poses, points, np.array(edges, _lib.EDGE_DTYPE)


@pytest.mark.gpu
def test_lba_window_against_an_independent_window_and_the_oracle(tmp_path, oracle):
    """build_lba_window (vertex order, fixed flags, mono / stereo choice, Omega, Huber delta,
    intrinsics) equals a window built here from the scene, and linearize_lba_window's
    BlockSolver<6,3> layout (block_solver.hpp:502-560: hessian blocks in vertex-id order,
    column-major, g2o's b sign, per (pose, point) H_pl sums, activeRobustChi2) equals the
    oracle's linearisation of that independent window, rearranged here into g2o's order."""
    from orb_slam2_test_amd import _lib
    exe = os.path.join(LIB, "compat_ref_selftest")
    sc = _lba_scene(np.random.default_rng(2026))
    d = tmp_path
    np.array([len(sc["kf"]), sc["K"], len(sc["mp"]), len(sc["obs"])], np.int32).tofile(d / "lba_meta.i32")
    sc["kf"].astype(np.float64).tofile(d / "lba_kf.f64")
    sc["kp"].astype(np.float32).tofile(d / "lba_kp.f32")
    sc["inv2"].tofile(d / "lba_inv2.f32")
    sc["mp"].astype(np.float64).tofile(d / "lba_mp.f64")
    sc["obs"].astype(np.int32).tofile(d / "lba_obs.i32")
    r = subprocess.run([exe, "lba", str(d)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    order, poses, points, edges = _expected_window(oracle, sc)
    got_poses = np.fromfile(d / "win_poses.bin", _lib.POSE_DTYPE)
    got_edges = np.fromfile(d / "win_edges.bin", _lib.EDGE_DTYPE)
    assert list(np.fromfile(d / "win_kf.i32", np.int32)) == order
    assert np.array_equal(got_poses.view(np.uint8), poses.view(np.uint8))
    assert np.array_equal(np.fromfile(d / "win_points.f64").reshape(-1, 3), points)
    assert len(got_edges) == len(edges) and len(edges) > 600
    for f in _lib.EDGE_DTYPE.names:
        assert np.array_equal(got_edges[f], edges[f]), f
    assert edges["stereo"].sum() > 100 and (edges["stereo"] == 0).sum() > 100
    assert poses["fixed"].tolist() == [0, 1, 0, 0, 1, 1]  # mnId 0 and the fixed cameras
    # the oracle's linearisation of the independent window, in g2o's hessian order
    eo, hpose, bpose, hpoint, bpoint = oracle.ba_linearize(poses, points, edges)
    ids = sc["kf"][order, 0]
    free = [n for n in range(len(order)) if not poses["fixed"][n]]
    hp_order = sorted(free, key=lambda n: ids[n])
    pt_order = list(np.argsort(sc["mp"][:, 0], kind="stable"))
    ph = {n: h for h, n in enumerate(hp_order)}
    qh = {j: h for h, j in enumerate(pt_order)}
    assert list(np.fromfile(d / "g2o_pose_hidx.i32", np.int32)) == [ph.get(n, -1) for n in range(len(order))]
    assert list(np.fromfile(d / "g2o_point_hidx.i32", np.int32)) == [qh[j] for j in range(len(points))]
    nf = len(hp_order)
    exp_hpp = np.concatenate([hpose[n].T.reshape(-1) for n in hp_order])  # column-major
    exp_hll = np.concatenate([hpoint[j].T.reshape(-1) for j in pt_order])
    exp_b = np.concatenate([bpose[n] for n in hp_order] + [bpoint[j] for j in pt_order])
    hpl = {}
    for e, o in zip(edges, eo):
        if poses["fixed"][e["pose"]]:
            continue
        key = (ph[e["pose"]], qh[e["point"]])
        hpl[key] = hpl.get(key, 0) + o["hpl"].T  # (pose row, point col) = hpl[c][r]
    got_hpl = np.fromfile(d / "g2o_Hpl.f64").reshape(-1, 20)
    assert len(got_hpl) == len(hpl)

    def rel(a, b):
        return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))

    assert rel(np.fromfile(d / "g2o_Hpp.f64"), exp_hpp) < 1e-9
    assert rel(np.fromfile(d / "g2o_Hll.f64"), exp_hll) < 1e-9
    assert rel(np.fromfile(d / "g2o_b.f64"), exp_b) < 1e-9
    for row in got_hpl:
        blk = hpl[(int(row[0]), int(row[1]))]
        assert rel(row[2:].reshape(3, 6).T, blk) < 1e-9  # column-major 6x3
    # activeRobustChi2 (sparse_optimizer.cpp:100-114) over the oracle's per-edge chi2
    dsq = (edges["huber_delta"] ** 2).astype(np.float32).astype(np.float64)
    rho0 = np.where(eo["chi2"] <= dsq, eo["chi2"], 2 * np.sqrt(eo["chi2"]) * edges["huber_delta"] - dsq)
    chi = float(np.fromfile(d / "g2o_chi2.f64")[0])
    assert abs(chi - rho0.sum()) <= 1e-9 * abs(rho0.sum())
    assert nf == 3
