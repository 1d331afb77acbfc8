"""Seeded synthetic grayscale sequences (SURVEY.md 8d "Synthetic inputs").

There is no network and no dataset in this environment, so benches and tests use
KITTI/TUM-shaped synthetic frames: value-noise texture (4 octaves of bilinearly
up-sampled uniform noise) plus random rectangles and line edges, so FAST finds
corners in every 30-px cell.  Frame t+1 is the same canvas panned by a seeded
(dx, dy) of at most 8 px plus +-2 intensity noise, so frame-to-frame matching has
true correspondences.  Everything is numpy with ``np.random.Generator(PCG64)``.
"""
import numpy as np

DEFAULT_SEED = 20261015


def _value_noise(rng, h, w, cell):
    gh, gw = h // cell + 2, w // cell + 2
    grid = rng.random((gh, gw), dtype=np.float32)
    ys = np.arange(h, dtype=np.float32) / cell
    xs = np.arange(w, dtype=np.float32) / cell
    y0 = np.floor(ys).astype(np.int64)
    x0 = np.floor(xs).astype(np.int64)
    fy = (ys - y0)[:, None]
    fx = (xs - x0)[None, :]
    g00 = grid[y0][:, x0]
    g01 = grid[y0][:, x0 + 1]
    g10 = grid[y0 + 1][:, x0]
    g11 = grid[y0 + 1][:, x0 + 1]
    return (g00 * (1 - fx) + g01 * fx) * (1 - fy) + (g10 * (1 - fx) + g11 * fx) * fy


def canvas(h, w, seed=DEFAULT_SEED, n_rects=None, n_lines=None):
    """A textured float32 canvas in [0, 255]."""
    rng = np.random.Generator(np.random.PCG64(seed))
    img = np.zeros((h, w), np.float32)
    for cell, amp in ((32, 0.35), (12, 0.25), (5, 0.2), (2, 0.2)):
        img += amp * _value_noise(rng, h, w, cell)
    img = img * 255.0
    area = h * w
    n_rects = n_rects if n_rects is not None else max(8, area // 6000)
    for _ in range(n_rects):
        rh, rw = rng.integers(6, 60, size=2)
        y, x = rng.integers(0, max(1, h - rh)), rng.integers(0, max(1, w - rw))
        img[y:y + rh, x:x + rw] = img[y:y + rh, x:x + rw] * 0.3 + rng.uniform(0, 255) * 0.7
    n_lines = n_lines if n_lines is not None else max(4, area // 20000)
    for _ in range(n_lines):
        if rng.random() < 0.5:
            y = rng.integers(0, h)
            x0, x1 = sorted(rng.integers(0, w, size=2))
            img[y:y + 2, x0:x1] = rng.uniform(0, 255)
        else:
            x = rng.integers(0, w)
            y0, y1 = sorted(rng.integers(0, h, size=2))
            img[y0:y1, x:x + 2] = rng.uniform(0, 255)
    return np.clip(img, 0, 255)


def frame(h, w, seed=DEFAULT_SEED):
    """A single synthetic u8 frame."""
    return np.rint(canvas(h, w, seed)).astype(np.uint8)


def sequence(n, h, w, seed=DEFAULT_SEED, max_step=8, noise=2):
    """n frames (n, h, w) u8 panning over one canvas with seeded (dx, dy) <= max_step."""
    rng = np.random.Generator(np.random.PCG64(seed + 1))
    steps = rng.integers(-max_step, max_step + 1, size=(n, 2))
    steps[0] = 0
    pos = np.cumsum(steps, axis=0)
    pos -= pos.min(axis=0)
    ch = h + int(pos[:, 0].max()) + 1
    cw = w + int(pos[:, 1].max()) + 1
    base = canvas(ch, cw, seed)
    out = np.empty((n, h, w), np.uint8)
    for t in range(n):
        y, x = pos[t]
        crop = base[y:y + h, x:x + w]
        jitter = rng.integers(-noise, noise + 1, size=(h, w)).astype(np.float32)
        out[t] = np.clip(np.rint(crop + jitter), 0, 255).astype(np.uint8)
    return out


def sequence_block(n_total, lo, hi, h, w, seed=DEFAULT_SEED, max_step=8, noise=2):
    """Frames [(lo - 1) mod n_total, lo, ..., hi - 1] -- a rank's block of the cyclic
    batched-sequence partition plus its 1-frame halo (sequence.local_indices) -- of an
    n_total-frame sequence panning over one canvas like sequence().  Each frame's pixel
    jitter comes from its own generator (seed, t), so a rank materialises only its block."""
    from .sequence import local_indices
    rng = np.random.Generator(np.random.PCG64(seed + 1))
    steps = rng.integers(-max_step, max_step + 1, size=(n_total, 2))
    steps[0] = 0
    pos = np.cumsum(steps, axis=0)
    pos -= pos.min(axis=0)
    base = canvas(h + int(pos[:, 0].max()) + 1, w + int(pos[:, 1].max()) + 1, seed)
    idx = local_indices(n_total, lo, hi)
    out = np.empty((len(idx), h, w), np.uint8)
    for j, t in enumerate(idx):
        y, x = pos[t]
        crop = base[y:y + h, x:x + w]
        jr = np.random.Generator(np.random.PCG64([seed + 7, int(t)]))
        jitter = jr.integers(-noise, noise + 1, size=(h, w)).astype(np.float32)
        out[j] = np.clip(np.rint(crop + jitter), 0, 255).astype(np.uint8)
    return out


def sequence_blocks(n_total, ranges, h, w, seed=DEFAULT_SEED, max_step=8, noise=2):
    """sequence_block for several blocks [(lo, hi), ...] of one n_total-frame sequence,
    with the canvas built once: a list of [hi - lo + 1, h, w] arrays (halo first)."""
    from .sequence import local_indices
    rng = np.random.Generator(np.random.PCG64(seed + 1))
    steps = rng.integers(-max_step, max_step + 1, size=(n_total, 2))
    steps[0] = 0
    pos = np.cumsum(steps, axis=0)
    pos -= pos.min(axis=0)
    base = canvas(h + int(pos[:, 0].max()) + 1, w + int(pos[:, 1].max()) + 1, seed)
    blocks = []
    for lo, hi in ranges:
        idx = local_indices(n_total, lo, hi)
        out = np.empty((len(idx), h, w), np.uint8)
        for j, t in enumerate(idx):
            y, x = pos[t]
            crop = base[y:y + h, x:x + w]
            jr = np.random.Generator(np.random.PCG64([seed + 7, int(t)]))
            jitter = jr.integers(-noise, noise + 1, size=(h, w)).astype(np.float32)
            out[j] = np.clip(np.rint(crop + jitter), 0, 255).astype(np.uint8)
        blocks.append(out)
    return blocks


def bench_block_ranges(B, world, rank, nblocks):
    """The blocks bench.py streams through on rank `rank`: block k = frames
    [(k world + rank) B, (k world + rank + 1) B) of one cyclic nblocks * world * B-frame
    sequence, so consecutive steps read different frames (different HBM) and every rank's
    block k is disjoint from every other rank's.  Returns (n_total, [(lo, hi), ...])."""
    n_total = nblocks * world * B
    return n_total, [((k * world + rank) * B, (k * world + rank + 1) * B) for k in range(nblocks)]


def stereo_pair(h, w, seed=DEFAULT_SEED, noise=2, d_min=4.0, d_max=60.0, n_objects=6):
    """A rectified synthetic stereo pair (left, right) u8 and the true disparity map.

    Disparity d(x, y) is a road-like plane growing from d_min at the top row to ~d_max/2 at
    the bottom, with n_objects nearer fronto-parallel boxes up to d_max.  The right image
    samples the left canvas at x + d (linear interpolation): a left pixel at column x sees
    the same scene point at x - d in the right image, as for KITTI's rectified cameras.
    Occlusions are ignored.  Noise is +-noise independently per image."""
    rng = np.random.Generator(np.random.PCG64(seed + 31))
    pad = int(np.ceil(d_max)) + 2
    base = canvas(h, w + pad, seed)
    ys = np.arange(h, dtype=np.float32)[:, None]
    disp = np.broadcast_to(d_min + (d_max / 2 - d_min) * ys / max(h - 1, 1), (h, w)).copy()
    for _ in range(n_objects):
        oh, ow = rng.integers(h // 8, h // 3), rng.integers(w // 16, w // 5)
        oy, ox = rng.integers(0, h - oh), rng.integers(0, w - ow)
        disp[oy:oy + oh, ox:ox + ow] = rng.uniform(d_max / 3, d_max)
    left = base[:, :w]
    xs = np.arange(w, dtype=np.float32)[None, :]
    # right(x) = scene point whose left column is x + d: sample the left canvas at x + d
    src = np.clip(xs + disp, 0, w + pad - 2)
    x0 = np.floor(src).astype(np.int64)
    fx = src - x0
    rows = np.arange(h)[:, None]
    right = base[rows, x0] * (1 - fx) + base[rows, x0 + 1] * fx
    jl = rng.integers(-noise, noise + 1, size=(h, w)).astype(np.float32)
    jr = rng.integers(-noise, noise + 1, size=(h, w)).astype(np.float32)
    L = np.clip(np.rint(left + jl), 0, 255).astype(np.uint8)
    R = np.clip(np.rint(right + jr), 0, 255).astype(np.uint8)
    return L, R, disp


def stereo_sequence(n, h, w, seed=DEFAULT_SEED, noise=2, d_min=4.0, d_max=60.0):
    """n rectified stereo frames: left = sequence(n, h, w, seed), right[t](x) = left[t](x + d)
    (linear interpolation, clamped at the right edge) with one disparity map d(x, y) of the
    stereo_pair kind, plus +-noise.  Returns (lefts, rights, disparity)."""
    lefts = sequence(n, h, w, seed=seed)
    _, _, disp = stereo_pair(h, w, seed=seed, noise=0, d_min=d_min, d_max=d_max)
    rng = np.random.Generator(np.random.PCG64(seed + 57))
    xs = np.arange(w, dtype=np.float32)[None, :]
    src = np.clip(xs + disp, 0, w - 1.001)
    x0 = np.floor(src).astype(np.int64)
    fx = (src - x0).astype(np.float32)
    rows = np.arange(h)[:, None]
    rights = np.empty_like(lefts)
    for t in range(n):
        a = lefts[t].astype(np.float32)
        r = a[rows, x0] * (1 - fx) + a[rows, x0 + 1] * fx
        r += rng.integers(-noise, noise + 1, size=(h, w)).astype(np.float32)
        rights[t] = np.clip(np.rint(r), 0, 255).astype(np.uint8)
    return lefts, rights, disp


def sequence_positions(n, seed=DEFAULT_SEED, max_step=8):
    """(n, 2) canvas offsets (y, x) of sequence(n, ..., seed, max_step): frame t's pixel
    (x, y) is canvas (x + pos[t, 1], y + pos[t, 0])."""
    rng = np.random.Generator(np.random.PCG64(seed + 1))
    steps = rng.integers(-max_step, max_step + 1, size=(n, 2))
    steps[0] = 0
    pos = np.cumsum(steps, axis=0)
    return pos - pos.min(axis=0)


def constant(h, w, value=128):
    return np.full((h, w), value, np.uint8)


def pure_noise(h, w, seed=DEFAULT_SEED):
    rng = np.random.Generator(np.random.PCG64(seed + 7))
    return rng.integers(0, 256, size=(h, w), dtype=np.uint8)


# ---------------------------------------------------------------------------
# Local-BA windows (SURVEY.md 8d "BA"): KITTI00 intrinsics (Stereo/KITTI00-02.yaml)
# ---------------------------------------------------------------------------
KITTI_FX = 718.856
KITTI_FY = 718.856
KITTI_CX = 607.1928
KITTI_CY = 185.2157
KITTI_BF = 386.1448


def _quat_from_axis_angle(axis, ang):
    axis = axis / np.linalg.norm(axis)
    s = np.sin(ang / 2)
    q = np.array([axis[0] * s, axis[1] * s, axis[2] * s, np.cos(ang / 2)])
    if q[3] < 0:
        q = -q
    return q


def _rot(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def ba_window(n_local=10, n_fixed=10, n_points=6000, obs_per_point=4.5, stereo_frac=0.6,
              outlier_frac=0.1, seed=DEFAULT_SEED, world_offset=500.0, robust=True,
              scale_factor=1.2, nlevels=8):
    """A synthetic LocalBundleAdjustment window.  Returns (poses, points, edges) as
    structured arrays with the dtypes of orb_slam2_test_amd._lib (pose/edge records)."""
    from ._lib import EDGE_DTYPE, POSE_DTYPE
    rng = np.random.Generator(np.random.PCG64(seed + 99))
    npose = n_local + n_fixed
    origin = rng.uniform(-world_offset, world_offset, size=3)
    poses = np.zeros(npose, POSE_DTYPE)
    cams = []
    for i in range(npose):
        # cameras driving forward along +z in world, small rotations
        q = _quat_from_axis_angle(rng.normal(size=3), rng.uniform(0, 0.15))
        Rcw = _rot(q)
        center = origin + np.array([rng.normal(0, 1.0), rng.normal(0, 0.2), 1.5 * i])
        t = -Rcw @ center
        poses[i]["q"] = q
        poses[i]["t"] = t
        poses[i]["fixed"] = 1 if i >= n_local else 0
        cams.append((Rcw, t))
    # points in front of the cameras at depth 5-60 m
    pts = np.zeros((n_points, 3))
    for j in range(n_points):
        Rcw, t = cams[rng.integers(0, npose)]
        depth = rng.uniform(5, 60)
        u = rng.uniform(0, 1241)
        v = rng.uniform(0, 376)
        xc = np.array([(u - KITTI_CX) / KITTI_FX * depth, (v - KITTI_CY) / KITTI_FY * depth, depth])
        pts[j] = Rcw.T @ (xc - t)
    inv_sigma2 = [1.0 / float(np.float32(np.float32(scale_factor) ** (2 * l))) for l in range(nlevels)]
    edges = []
    for j in range(n_points):
        k = max(1, int(rng.poisson(obs_per_point - 1)) + 1)
        kfs = rng.choice(npose, size=min(k, npose), replace=False)
        for i in kfs:
            Rcw, t = cams[i]
            xc = Rcw @ pts[j] + t
            if xc[2] <= 0.1:
                continue
            e = np.zeros((), EDGE_DTYPE)
            e["point"] = j
            e["pose"] = i
            octave = int(rng.integers(0, nlevels))
            e["inv_sigma2"] = float(np.float32(inv_sigma2[octave]))
            e["fx"], e["fy"], e["cx"], e["cy"], e["bf"] = (KITTI_FX, KITTI_FY, KITTI_CX, KITTI_CY,
                                                           KITTI_BF)
            u = KITTI_FX * xc[0] / xc[2] + KITTI_CX
            v = KITTI_FY * xc[1] / xc[2] + KITTI_CY
            noise = rng.normal(0, 1.0, size=3)
            if rng.random() < outlier_frac:
                noise *= 25
            stereo = rng.random() < stereo_frac
            # observations are float keypoint coordinates (cv::KeyPoint pt, f32 -> double)
            e["obs"][0] = float(np.float32(u + noise[0]))
            e["obs"][1] = float(np.float32(v + noise[1]))
            if stereo:
                e["stereo"] = 1
                e["obs"][2] = float(np.float32(u - KITTI_BF / xc[2] + noise[2]))
                e["huber_delta"] = float(np.float32(np.sqrt(7.815)))
            else:
                e["huber_delta"] = float(np.float32(np.sqrt(5.991)))
            e["robust"] = 1 if robust else 0
            e["active"] = 1
            edges.append(e)
    return poses, pts, np.array(edges, dtype=EDGE_DTYPE)


# ---------------------------------------------------------------------------
# Tracking-matcher scenes (ORBmatcher::SearchByProjection): map points back-projected
# from frame t-1's keypoints at a common depth, so a pure camera translation reproduces
# the sequence's pan (u' = u + fx tx / z) and the matches have a ground truth.
# ---------------------------------------------------------------------------
MP_VALID, MP_HAS_OBS = 1, 2
LF_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("octave", "<i4"),
                     ("angle", "<f4"), ("flags", "<i4")])
MP_DTYPE = np.dtype([("u", "<f4"), ("v", "<f4"), ("ur", "<f4"), ("level", "<i4"),
                     ("view_cos", "<f4"), ("flags", "<i4")])


def tracking_scene(kps_last, shift_xy, seed=DEFAULT_SEED, depth=10.0, fx=KITTI_FX, fy=KITTI_FY,
                   cx=KITTI_CX, cy=KITTI_CY, bf=KITTI_BF, tz=0.0, valid_frac=0.9,
                   obs_frac=0.8):
    """LastFrame points and camera poses for SearchByProjection(CurrentFrame, LastFrame).

    kps_last: frame t-1 keypoints (KP_DTYPE); shift_xy: image motion (dx, dy) of the scene
    from t-1 to t.  World = camera t-1 (Tlw = [I | 0]); Tcw = [I | t] with
    t = (dx z / fx, dy z / fy, tz).  Returns (points LF_DTYPE, Tcw (3, 4), Tlw (3, 4))."""
    rng = np.random.Generator(np.random.PCG64(seed + 31))
    n = len(kps_last)
    z = np.float32(depth)
    pts = np.zeros(n, LF_DTYPE)
    pts["x"] = (kps_last["x"] - np.float32(cx)) * z / np.float32(fx)
    pts["y"] = (kps_last["y"] - np.float32(cy)) * z / np.float32(fy)
    pts["z"] = z
    pts["octave"] = kps_last["octave"]
    pts["angle"] = kps_last["angle"]
    fl = np.where(rng.random(n) < valid_frac, MP_VALID, 0)
    fl |= np.where(rng.random(n) < obs_frac, MP_HAS_OBS, 0)
    pts["flags"] = fl
    Tlw = np.zeros((3, 4), np.float32)
    Tlw[:, :3] = np.eye(3)
    Tcw = Tlw.copy()
    Tcw[0, 3] = shift_xy[0] * depth / fx
    Tcw[1, 3] = shift_xy[1] * depth / fy
    Tcw[2, 3] = tz
    return pts, Tcw, Tlw


def map_projections(kps_src, shift_xy, seed=DEFAULT_SEED, depth=10.0, bf=KITTI_BF, jitter=0.7,
                    valid_frac=0.9, obs_frac=0.9):
    """Local-map projections (Frame::isInFrustum outputs) of map points seen at kps_src,
    moved by shift_xy plus up to +-jitter px: MP_DTYPE records."""
    rng = np.random.Generator(np.random.PCG64(seed + 37))
    n = len(kps_src)
    mp = np.zeros(n, MP_DTYPE)
    mp["u"] = kps_src["x"] + np.float32(shift_xy[0]) + rng.uniform(-jitter, jitter, n).astype(np.float32)
    mp["v"] = kps_src["y"] + np.float32(shift_xy[1]) + rng.uniform(-jitter, jitter, n).astype(np.float32)
    mp["ur"] = mp["u"] - np.float32(bf / depth)
    mp["level"] = kps_src["octave"]
    mp["view_cos"] = np.where(rng.random(n) < 0.5, 0.9995, 0.99).astype(np.float32)
    fl = np.where(rng.random(n) < valid_frac, MP_VALID, 0)
    fl |= np.where(rng.random(n) < obs_frac, MP_HAS_OBS, 0)
    mp["flags"] = fl
    return mp


# ---------------------------------------------------------------------------
# PoseOptimization frames: map points seen by one frame with a perturbed initial pose
# ---------------------------------------------------------------------------
PEDGE_DTYPE = np.dtype([("obs", "<f4", 3), ("xw", "<f4", 3), ("inv_sigma2", "<f4"),
                        ("stereo", "<i4")])


def pose_frame(n=1500, stereo_frac=0.5, outlier_frac=0.1, seed=DEFAULT_SEED, noise=1.0,
               rot_err=0.01, trans_err=0.1, world_offset=50.0):
    """One Tracking frame for Optimizer::PoseOptimization: n map points at 4-60 m with their
    keypoint observations (pixel noise `noise` scaled per octave, stereo u_r for
    stereo_frac, outlier_frac replaced by random pixels), the true pose Tcw and a perturbed
    initial pose (the motion-model prediction).  Returns (edges, Tcw_true (3, 4),
    Tcw_init (3, 4)), float32 poses."""
    rng = np.random.Generator(np.random.PCG64(seed + 41))
    q = _quat_from_axis_angle(rng.normal(size=3), rng.uniform(0, 0.3))
    R = _rot(q)
    t = rng.uniform(-world_offset, world_offset, 3)
    Tcw = np.zeros((3, 4))
    Tcw[:, :3] = R
    Tcw[:, 3] = t
    # points in front of the camera, then to world
    depth = rng.uniform(4, 60, n)
    u = rng.uniform(0, 1241, n)
    v = rng.uniform(0, 376, n)
    xc = np.stack([(u - KITTI_CX) * depth / KITTI_FX, (v - KITTI_CY) * depth / KITTI_FY, depth], 1)
    xw = (xc - t) @ R  # R^T (xc - t)
    octave = rng.integers(0, 8, n)
    scale = 1.2 ** octave
    e = np.zeros(n, PEDGE_DTYPE)
    obs_u = u + rng.normal(0, noise, n) * scale
    obs_v = v + rng.normal(0, noise, n) * scale
    ur = obs_u - KITTI_BF / depth + rng.normal(0, noise, n) * scale
    out = rng.random(n) < outlier_frac
    obs_u[out] = rng.uniform(0, 1241, out.sum())
    obs_v[out] = rng.uniform(0, 376, out.sum())
    e["obs"][:, 0] = obs_u
    e["obs"][:, 1] = obs_v
    st = rng.random(n) < stereo_frac
    e["obs"][:, 2] = np.where(st, ur, -1.0)
    e["stereo"] = st
    e["xw"] = xw
    e["inv_sigma2"] = (1.0 / (scale * scale)).astype(np.float32)
    dq = _quat_from_axis_angle(rng.normal(size=3), rot_err)
    R0 = _rot(dq) @ R
    T0 = np.zeros((3, 4))
    T0[:, :3] = R0
    T0[:, 3] = t + rng.normal(0, trans_err, 3)
    return e, Tcw.astype(np.float32), T0.astype(np.float32)


# ---------------------------------------------------------------------------
# DBoW2 vocabularies (ORBvoc.txt is not shipped with the reference checkout; these stand in
# for it with the same text format, sizes and weighting)
# ---------------------------------------------------------------------------
def _flip_mask(rng, n, depth):
    """random 32-byte masks whose bits are set with probability 2^-depth"""
    m = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    for _ in range(depth - 1):
        m &= rng.integers(0, 256, (n, 32), dtype=np.uint8)
    return m


def vocabulary(k=10, L=6, seed=DEFAULT_SEED, stop_frac=0.01, scoring=0, weighting=0):
    """A full k-ary tree of depth L in breadth-first node order (node 0 the root, parent
    (i - 1) // k), the node list loadFromTextFile builds (TemplatedVocabulary.h:1376-1417).
    Children descend from their parent's descriptor with 2^-level bit flips (level 1 fully
    random), so a descriptor's path is decided by real distance gaps and ties as in a
    k-means tree.  Leaves carry idf weights in (0.5, 10), stop_frac of them 0 (stopped);
    ORBvoc.txt's header is "10 6 0 0" (TF_IDF, L1_NORM)."""
    rng = np.random.default_rng(seed)
    n = (k ** (L + 1) - 1) // (k - 1)
    parent = np.zeros(n, np.int32)
    parent[1:] = (np.arange(1, n) - 1) // k
    desc = np.zeros((n, 32), np.uint8)
    lo = 1
    for lvl in range(1, L + 1):
        hi = lo + k ** lvl
        if lvl == 1:
            desc[lo:hi] = rng.integers(0, 256, (hi - lo, 32), dtype=np.uint8)
        else:
            desc[lo:hi] = desc[parent[lo:hi]] ^ _flip_mask(rng, hi - lo, min(lvl, 4))
        lo = hi
    is_leaf = np.zeros(n, np.uint8)
    first_leaf = (k ** L - 1) // (k - 1)
    is_leaf[first_leaf:] = 1
    weight = np.zeros(n)
    nl = n - first_leaf
    w = rng.uniform(0.5, 10.0, nl)
    w[rng.random(nl) < stop_frac] = 0.0
    weight[first_leaf:] = w
    return dict(k=k, L=L, scoring=scoring, weighting=weighting, parent=parent,
                is_leaf=is_leaf, desc=desc, weight=weight)


def ragged_vocabulary(k=10, L=5, seed=DEFAULT_SEED, leaf_prob=0.25, stop_frac=0.05,
                      scoring=0, weighting=0, max_nodes=60000):
    """A ragged tree in DBoW2's creation order (each node's children appended together,
    then each child expanded -- HKmeansStep): k root children, 1..k per inner node, leaves at
    depths 2..L (a node below L becomes a leaf with probability leaf_prob), duplicate sibling
    descriptors (exact distance ties) and some stopped words."""
    rng = np.random.default_rng(seed)
    parent, leaf, desc, depth = [0], [0], [np.zeros(32, np.uint8)], [0]
    stack = [0]
    while stack:
        p = stack.pop(0)
        if len(parent) + k > max_nodes:
            break
        nc = int(rng.integers(1, k + 1)) if p else k
        kids = []
        for j in range(nc):
            d = (desc[p] ^ _flip_mask(rng, 1, min(depth[p] + 1, 4))[0]) if p else \
                rng.integers(0, 256, 32, dtype=np.uint8)
            if j > 0 and rng.random() < 0.1:
                d = desc[kids[-1]].copy()         # sibling duplicate: exact tie
            nid = len(parent)
            parent.append(p)
            desc.append(d)
            depth.append(depth[p] + 1)
            is_leaf = depth[p] + 1 >= L or (depth[p] >= 1 and rng.random() < leaf_prob)
            leaf.append(1 if is_leaf else 0)
            kids.append(nid)
            if not is_leaf:
                stack.append(nid)
    # inner nodes left unexpanded by max_nodes become leaves (isLeaf() = no children)
    has_child = np.zeros(len(parent), bool)
    has_child[np.asarray(parent[1:], np.int64)] = True
    leaf = np.where(has_child, 0, 1).astype(np.uint8)
    leaf[0] = 0
    n = len(parent)
    weight = np.where(leaf > 0, rng.uniform(0.5, 10.0, n), 0.0)
    weight[(leaf > 0) & (rng.random(n) < stop_frac)] = 0.0
    return dict(k=k, L=L, scoring=scoring, weighting=weighting,
                parent=np.asarray(parent, np.int32), is_leaf=leaf, desc=np.asarray(desc),
                weight=weight)


def write_vocabulary_text(path, voc, weight_fmt="%.17g"):
    """TemplatedVocabulary::saveToTextFile's format (TemplatedVocabulary.h:1429-1447):
    "k L scoring weighting", then "parent isLeaf d0 .. d31 weight" per node 1..n-1
    (saveToTextFile streams the weight with the default 6 significant digits; pass
    weight_fmt="%g" for that)."""
    n = len(voc["parent"])
    with open(path, "w") as f:
        f.write("%d %d %d %d\n" % (voc["k"], voc["L"], voc["scoring"], voc["weighting"]))
        for i in range(1, n):
            f.write("%d %d %s %s\n" % (voc["parent"][i], voc["is_leaf"][i],
                                       " ".join(str(int(b)) for b in voc["desc"][i]),
                                       weight_fmt % voc["weight"][i]))
