"""ctypes front-end of the CPU oracle -- TEST INFRASTRUCTURE ONLY.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg may
import this module.  The product (``orb_slam2_test_amd``) never does.

The oracle restates the reference algorithms (see oracle/orb_oracle.h for the
file:line map) in plain C; this module builds ``oracle/_build/liborbg_oracle.so``
on demand (gcc) and exposes numpy-friendly wrappers.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liborbg_oracle.so")

MAX_LEVELS = 16

KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
POSE_DTYPE = np.dtype([("q", "<f8", 4), ("t", "<f8", 3), ("fixed", "<i4"), ("pad", "<i4")])
EDGE_DTYPE = np.dtype([("point", "<i4"), ("pose", "<i4"), ("stereo", "<i4"), ("robust", "<i4"),
                       ("active", "<i4"), ("pad", "<i4"), ("obs", "<f8", 3),
                       ("inv_sigma2", "<f8"), ("fx", "<f8"), ("fy", "<f8"), ("cx", "<f8"),
                       ("cy", "<f8"), ("bf", "<f8"), ("huber_delta", "<f8")])
EDGE_OUT_DTYPE = np.dtype([("err", "<f8", 3), ("chi2", "<f8"), ("rho1", "<f8"),
                           ("jp", "<f8", (3, 3)), ("jt", "<f8", (3, 6)), ("hpl", "<f8", (3, 6))])

RESIZE_SCALAR, RESIZE_SSE2_16_4, RESIZE_SIMD_16_8 = 0, 4, 8
# cosf/sinf of the rBRIEF rotation (orb_oracle.h ORC_SINCOS_*)
SINCOS_GLIBC, SINCOS_PINNED, SINCOS_HOST = 0, 1, 2

# tracking matcher records (orb_oracle.h: orc_lf_point, orc_map_proj)
MP_VALID, MP_HAS_OBS = 1, 2
LF_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("octave", "<i4"),
                     ("angle", "<f4"), ("flags", "<i4")])
MP_DTYPE = np.dtype([("u", "<f4"), ("v", "<f4"), ("ur", "<f4"), ("level", "<i4"),
                     ("view_cos", "<f4"), ("flags", "<i4")])


# Frame / MapPoint geometry records (orb_oracle.h: orc_camera, orc_map_point, orc_frustum_cam)
CAMERA_DTYPE = np.dtype([("fx", "<f4"), ("fy", "<f4"), ("cx", "<f4"), ("cy", "<f4"),
                         ("k1", "<f4"), ("k2", "<f4"), ("p1", "<f4"), ("p2", "<f4"),
                         ("k3", "<f4")])
MAPPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("nx", "<f4"),
                           ("ny", "<f4"), ("nz", "<f4"), ("min_dist", "<f4"),
                           ("max_dist", "<f4"), ("flags", "<i4")])
RELOC_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("min_dist", "<f4"),
                        ("max_dist", "<f4"), ("angle", "<f4"), ("flags", "<i4")])
SIM3_PAIR_DTYPE = np.dtype([("T1w", "<f4", 12), ("T2w", "<f4", 12), ("R12", "<f4", 9),
                            ("t12", "<f4", 3), ("s12", "<f4"), ("fx", "<f4"), ("fy", "<f4"),
                            ("cx", "<f4"), ("cy", "<f4"), ("log_scale_factor", "<f4"),
                            ("nlevels", "<i4"), ("min_x", "<f4"), ("max_x", "<f4"),
                            ("min_y", "<f4"), ("max_y", "<f4")])
FRUSTUM_DTYPE = np.dtype([("Tcw", "<f4", 12), ("fx", "<f4"), ("fy", "<f4"), ("cx", "<f4"),
                          ("cy", "<f4"), ("bf", "<f4"), ("log_scale_factor", "<f4"),
                          ("nlevels", "<i4"), ("min_x", "<f4"), ("max_x", "<f4"),
                          ("min_y", "<f4"), ("max_y", "<f4")])


# SearchForTriangulation pair geometry (orb_oracle.h orc_tri_geom)
TRI_GEOM_DTYPE = np.dtype([("F12", "<f4", 9), ("Cw1", "<f4", 3), ("Tcw2", "<f4", 12),
                           ("fx2", "<f4"), ("fy2", "<f4"), ("cx2", "<f4"), ("cy2", "<f4")])


# CreateNewMapPoints camera record (orb_oracle.h orc_kf_cam) and status codes (ORC_TRI_*)
KF_CAM_DTYPE = np.dtype([("Tcw", "<f4", 12), ("fx", "<f4"), ("fy", "<f4"), ("cx", "<f4"),
                         ("cy", "<f4"), ("invfx", "<f4"), ("invfy", "<f4"), ("mb", "<f4"),
                         ("mbf", "<f4")])
TRI_NONE, TRI_NEW, TRI_PARALLAX, TRI_W0, TRI_Z1, TRI_Z2 = 0, 1, -1, -2, -3, -4
TRI_REPROJ1, TRI_REPROJ2, TRI_DIST0, TRI_SCALE = -5, -6, -7, -8


class KFTri(C.Structure):
    _fields_ = [("kps", C.c_void_p), ("kps_raw", C.c_void_p), ("uright", C.c_void_p),
                ("depth", C.c_void_p), ("n", C.c_int32)]


class TriKF(C.Structure):
    _fields_ = [("kps", C.c_void_p), ("desc", C.c_void_p), ("uright", C.c_void_p),
                ("has_mp", C.c_void_p), ("n", C.c_int32), ("fv_nodes", C.c_void_p),
                ("fv_off", C.c_void_p), ("fv_feats", C.c_void_p), ("nfv", C.c_int32)]


class Params(C.Structure):
    _fields_ = [("nfeatures", C.c_int32), ("scale_factor", C.c_float), ("nlevels", C.c_int32),
                ("ini_th_fast", C.c_int32), ("min_th_fast", C.c_int32),
                ("scale", C.c_float * MAX_LEVELS), ("inv_scale", C.c_float * MAX_LEVELS),
                ("sigma2", C.c_float * MAX_LEVELS), ("inv_sigma2", C.c_float * MAX_LEVELS),
                ("features_per_level", C.c_int32 * MAX_LEVELS), ("umax", C.c_int32 * 16),
                ("resize_mode", C.c_int32), ("gauss_k", C.c_int32 * 7), ("brief_fma", C.c_int32),
                ("sincos_mode", C.c_int32)]


PEDGE_DTYPE = np.dtype([("obs", "<f4", 3), ("xw", "<f4", 3), ("inv_sigma2", "<f4"),
                        ("stereo", "<i4")])


class PoseCam(C.Structure):
    _fields_ = [("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float),
                ("bf", C.c_float), ("pad", C.c_float)]


class TrackCam(C.Structure):
    _fields_ = [("Tcw", C.c_float * 12), ("Tlw", C.c_float * 12), ("fx", C.c_float),
                ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float), ("bf", C.c_float),
                ("b", C.c_float), ("mono", C.c_int32), ("pad", C.c_int32)]


def track_cam(Tcw, Tlw, fx, fy, cx, cy, bf, b, mono):
    c = TrackCam()
    for i, v in enumerate(np.asarray(Tcw, np.float32).reshape(12)):
        c.Tcw[i] = float(v)
    for i, v in enumerate(np.asarray(Tlw, np.float32).reshape(12)):
        c.Tlw[i] = float(v)
    c.fx, c.fy, c.cx, c.cy, c.bf, c.b = (float(np.float32(v)) for v in (fx, fy, cx, cy, bf, b))
    c.mono = 1 if mono else 0
    return c


class OrcVocab(C.Structure):
    _fields_ = [("k", C.c_int32), ("L", C.c_int32), ("scoring", C.c_int32),
                ("weighting", C.c_int32), ("nnodes", C.c_int32), ("nwords", C.c_int32),
                ("desc", C.c_void_p), ("weight", C.c_void_p), ("word_id", C.c_void_p),
                ("child_off", C.c_void_p), ("child_idx", C.c_void_p)]


class Bounds(C.Structure):
    _fields_ = [("min_x", C.c_float), ("max_x", C.c_float), ("min_y", C.c_float),
                ("max_y", C.c_float)]


_lib = None


def build(force=False):
    """Compile the oracle with its Makefile (gcc).  Returns the .so path."""
    srcs = [os.path.join(HERE, f) for f in os.listdir(HERE)
            if f.endswith((".c", ".h", ".inc")) or f == "Makefile"]
    if force or not os.path.exists(LIB_PATH) or any(
            os.path.getmtime(s) > os.path.getmtime(LIB_PATH) for s in srcs if os.path.exists(s)):
        subprocess.check_call(["make", "-s", "-C", HERE])
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        P = C.POINTER
        vp = C.c_void_p
        L.orc_init_params.argtypes = [P(Params), C.c_int, C.c_float, C.c_int, C.c_int, C.c_int]
        L.orc_extract.argtypes = [P(Params), vp, C.c_int, C.c_int, C.c_int, vp, vp, C.c_int, vp,
                                  vp, vp]
        L.orc_level_candidates.argtypes = [P(Params), vp, C.c_int, C.c_int, C.c_int, C.c_int, vp,
                                           C.c_int]
        L.orc_distribute_octree.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                            C.c_int, vp, C.c_int]
        L.orc_resize_linear_u8.argtypes = [vp, C.c_int, C.c_int, C.c_int, vp, C.c_int, C.c_int,
                                           C.c_int, C.c_int]
        L.orc_gauss7_u8.argtypes = [vp, C.c_int, C.c_int, C.c_int, vp, C.c_int, vp]
        L.orc_fast_score.argtypes = [vp, C.c_int]
        L.orc_fast_window.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.c_int, vp, C.c_int]
        L.orc_fast_atan2.argtypes = [C.c_float, C.c_float]
        L.orc_fast_atan2.restype = C.c_float
        L.orc_ic_angle.argtypes = [vp, C.c_int, C.c_float, C.c_float, vp]
        L.orc_ic_angle.restype = C.c_float
        L.orc_pinned_sincos_deg.argtypes = [C.c_float, P(C.c_float), P(C.c_float)]
        L.orc_brief_sincos_deg.argtypes = [C.c_float, C.c_int, P(C.c_float), P(C.c_float)]
        L.orc_glibc_sinf.argtypes = [C.c_float]
        L.orc_glibc_sinf.restype = C.c_float
        L.orc_glibc_cosf.argtypes = [C.c_float]
        L.orc_glibc_cosf.restype = C.c_float
        L.orc_sincosf_check.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32]
        L.orc_sincosf_check.restype = C.c_long
        L.orc_descriptor_distance.argtypes = [vp, vp]
        L.orc_knn2.argtypes = [vp, C.c_int, vp, C.c_int, vp, vp, vp]
        L.orc_search_for_initialization.argtypes = [vp, vp, C.c_int, vp, vp, C.c_int,
                                                    P(Bounds), vp, vp, C.c_int, C.c_float,
                                                    C.c_int]
        L.orc_frames_batch.argtypes = [P(Params), vp, C.c_int, C.c_int, C.c_int, C.c_int,
                                       C.c_int, C.c_float, vp, vp]
        L.orc_frames_full.argtypes = [P(Params), vp, C.c_int, C.c_int, C.c_int, C.c_int,
                                      C.c_int, C.c_float, vp, vp, C.c_int, vp, vp, vp, vp]
        L.orc_extract_batch.argtypes = [P(Params), vp, C.c_int, C.c_int, C.c_int, C.c_int, vp]
        L.orc_extract_batch.restype = C.c_long
        L.orc_ba_linearize.argtypes = [vp, C.c_int, vp, C.c_int, vp, C.c_int, vp, vp, vp, vp, vp]
        L.orc_ba_numeric_jacobian.argtypes = [vp, vp, vp, vp, vp]
        L.orc_ba_errors.argtypes = [vp, vp, vp, C.c_int, vp, vp, vp, vp]
        L.orc_ba_update.argtypes = [vp, C.c_int, vp, C.c_int, vp, vp]
        L.orc_ba_optimize.argtypes = [vp, C.c_int, vp, C.c_int, vp, C.c_int, C.c_int, vp]
        L.orc_ba_optimize.restype = C.c_int
        L.orc_ba_optimize_ctl.argtypes = [vp, C.c_int, vp, C.c_int, vp, C.c_int, C.c_int,
                                          C.c_int, C.c_int, vp, vp]
        L.orc_ba_optimize_ctl.restype = C.c_int
        L.orc_ba_errors.restype = C.c_double
        L.orc_ba_schur_solve.argtypes = [vp, C.c_int, C.c_int, vp, C.c_int, vp, vp, vp, vp, vp,
                                         C.c_double, vp, vp]
        L.orc_stereo_matches.argtypes = [P(Params), vp, vp, C.c_int, vp, vp, C.c_int, vp, vp,
                                         C.c_int, C.c_int, C.c_float, C.c_float, vp, vp]
        L.orc_track_direction.argtypes = [vp, vp, vp]
        L.orc_pose_optimization.argtypes = [vp, C.c_int, vp, vp, vp, vp, vp, vp]
        L.orc_se3_from_tcw.argtypes = [vp, vp, vp]
        L.orc_se3_to_tcw.argtypes = [vp, vp, vp]
        L.orc_match_pose.argtypes = [vp, C.c_int, vp, C.c_int, vp, vp, C.c_float, vp, vp, vp]
        L.orc_search_by_projection_lastframe.argtypes = [vp, vp, vp, C.c_int, vp, vp, vp, vp,
                                                         vp, C.c_int, vp, C.c_float, C.c_int,
                                                         vp]
        L.orc_search_by_projection_local.argtypes = [vp, vp, vp, C.c_int, vp, vp, vp, vp, vp,
                                                     C.c_int, C.c_float, C.c_float, vp]
        L.orc_bow_transform.argtypes = [P(OrcVocab), vp, C.c_int, C.c_int, vp, vp, P(C.c_int), vp,
                                        vp, vp, P(C.c_int)]
        L.orc_bow_word.argtypes = [P(OrcVocab), vp, C.c_int, P(C.c_int32), P(C.c_double),
                                   P(C.c_int32)]
        L.orc_search_by_bow.restype = C.c_int
        L.orc_search_by_bow.argtypes = [vp, vp, vp, C.c_int, vp, vp, vp, C.c_int, vp, vp, C.c_int,
                                        vp, vp, vp, C.c_int, C.c_float, C.c_int, vp]
        L.orc_search_for_triangulation.argtypes = [P(TriKF), P(TriKF), vp, vp, vp, C.c_int,
                                                   C.c_int, vp]
        L.orc_search_for_triangulation.restype = C.c_int
        L.orc_atan2f.argtypes = [C.c_float, C.c_float]
        L.orc_atan2f.restype = C.c_float
        L.orc_atan2f_check.argtypes = [C.c_uint32, C.c_long]
        L.orc_atan2f_check.restype = C.c_long
        L.orc_tri_geometry.argtypes = [vp, vp, vp]
        L.orc_tri_nullvec.argtypes = [vp, vp]
        L.orc_triangulate.argtypes = [P(KFTri), P(KFTri), vp, vp, vp, vp, vp, C.c_float, vp, vp]
        L.orc_triangulate.restype = C.c_int
        L.orc_fuse_search.argtypes = [P(TriKF), vp, vp, vp, C.c_int, C.c_float, vp, vp, vp, vp]
        L.orc_fuse_search.restype = C.c_int
        L.orc_fuse_sim3_search.argtypes = [P(TriKF), vp, vp, vp, C.c_int, C.c_float, vp, vp, vp]
        L.orc_fuse_sim3_search.restype = C.c_int
        L.orc_sim3_decompose.argtypes = [vp, vp]
        L.orc_search_by_projection_reloc.argtypes = [vp, vp, C.c_int, vp, vp, vp, vp, vp,
                                                     C.c_int, C.c_float, C.c_int, C.c_int, vp]
        L.orc_search_by_projection_reloc.restype = C.c_int
        L.orc_search_by_projection_sim3.argtypes = [vp, vp, C.c_int, vp, vp, vp, vp, vp,
                                                    C.c_int, C.c_int, vp]
        L.orc_search_by_projection_sim3.restype = C.c_int
        L.orc_search_by_sim3.argtypes = [vp, vp, C.c_int, vp, vp, vp, vp, vp, C.c_int, vp, vp,
                                         vp, vp, C.c_float, vp, vp]
        L.orc_search_by_sim3.restype = C.c_int
        L.orc_rgbd_stereo.argtypes = [vp, C.c_int, C.c_float, C.c_int, C.c_int, C.c_size_t, vp,
                                      vp, C.c_int, C.c_float, vp, vp]
        L.orc_rgbd_stereo.restype = None
        L.orc_sim3_decompose.restype = None
        L.orc_search_by_bow_kf.restype = C.c_int
        L.orc_search_by_bow_kf.argtypes = [vp, vp, vp, C.c_int, vp, vp, vp, C.c_int, vp, vp, vp,
                                           C.c_int, vp, vp, vp, C.c_int, C.c_float, C.c_int, vp]
        L.orc_undistort_points.argtypes = [vp, vp, C.c_int, vp]
        L.orc_undistort_keypoints.argtypes = [vp, vp, C.c_int, vp]
        L.orc_image_bounds.argtypes = [vp, C.c_int, C.c_int, P(Bounds)]
        L.orc_log_scale_factor.argtypes = [C.c_float]
        L.orc_log_scale_factor.restype = C.c_float
        L.orc_is_in_frustum_n.argtypes = [vp, vp, C.c_int, C.c_float, vp]
        L.orc_is_in_frustum_n.restype = C.c_int
        L.orc_distinctive_descriptor.argtypes = [vp, C.c_int]
        L.orc_distinctive_descriptor.restype = C.c_int
        L.orc_distinctive_descriptors_n.argtypes = [vp, vp, vp, C.c_int, vp]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


def params(nfeatures=2000, scale_factor=1.2, nlevels=8, ini_th_fast=20, min_th_fast=7,
           resize_mode=RESIZE_SIMD_16_8, gauss_k=None, brief_fma=0, sincos_mode=SINCOS_GLIBC):
    p = Params()
    rc = lib().orc_init_params(C.byref(p), nfeatures, scale_factor, nlevels, ini_th_fast,
                               min_th_fast)
    if rc != 0:
        raise ValueError("orc_init_params: %d" % rc)
    p.resize_mode = resize_mode
    if gauss_k is not None:
        for i in range(7):
            p.gauss_k[i] = int(gauss_k[i])
    p.brief_fma = brief_fma
    p.sincos_mode = sincos_mode
    return p


def level_sizes(p, w, h):
    out = []
    for l in range(p.nlevels):
        s = np.float32(p.inv_scale[l])
        out.append((int(np.rint(np.float32(w) * s)), int(np.rint(np.float32(h) * s))))
    return out


def extract(p, img, with_pyramid=False, with_desc=True):
    """ORBextractor::operator() restated.  Returns dict(kps, desc, level_counts[, pyramid])."""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    cap = p.nfeatures * 2 + 8 * 70
    kps = np.zeros(cap, KP_DTYPE)
    desc = np.zeros((cap, 32), np.uint8) if with_desc else None
    lc = np.zeros(MAX_LEVELS, np.int32)
    cc = np.zeros(MAX_LEVELS, np.int32)
    sizes = level_sizes(p, w, h)
    pyr = np.zeros(sum(a * b for a, b in sizes), np.uint8) if with_pyramid else None
    n = lib().orc_extract(C.byref(p), _p(img), w, h, w, _p(kps), _p(desc), cap, _p(lc), _p(pyr),
                          _p(cc))
    if n < 0:
        raise RuntimeError("orc_extract failed: %d" % n)
    out = {"kps": kps[:n].copy(), "level_counts": lc[:p.nlevels].copy(),
           "cand_counts": cc[:p.nlevels].copy()}
    if with_desc:
        out["desc"] = desc[:n].copy()
    if with_pyramid:
        levels, o = [], 0
        for (lw, lh) in sizes:
            levels.append(pyr[o:o + lw * lh].reshape(lh, lw).copy())
            o += lw * lh
        out["pyramid"] = levels
    return out


def level_candidates(p, lvl, level):
    lvl = np.ascontiguousarray(lvl, dtype=np.uint8)
    lh, lw = lvl.shape
    cap = lw * lh // 2 + 16
    out = np.zeros(cap, KP_DTYPE)
    n = lib().orc_level_candidates(C.byref(p), _p(lvl), lw, lh, lw, level, _p(out), cap)
    if n < 0:
        raise RuntimeError("orc_level_candidates failed: %d" % n)
    return out[:n].copy()


def resize_linear(src, dw, dh, mode=RESIZE_SIMD_16_8):
    src = np.ascontiguousarray(src, dtype=np.uint8)
    sh, sw = src.shape
    dst = np.zeros((dh, dw), np.uint8)
    lib().orc_resize_linear_u8(_p(src), sw, sh, sw, _p(dst), dw, dh, dw, mode)
    return dst


def gauss7(src, k=(18, 34, 48, 56, 48, 34, 18)):
    src = np.ascontiguousarray(src, dtype=np.uint8)
    h, w = src.shape
    dst = np.zeros_like(src)
    kk = np.asarray(k, np.int32)
    lib().orc_gauss7_u8(_p(src), w, h, w, _p(dst), w, _p(kk))
    return dst


def fast_atan2(y, x):
    return lib().orc_fast_atan2(float(y), float(x))


def sincos_deg(a, mode=SINCOS_PINNED):
    """(cos, sin) of the rBRIEF rotation for an angle in degrees (ORBextractor.cc:120-122)."""
    c, s = C.c_float(), C.c_float()
    lib().orc_brief_sincos_deg(float(a), int(mode), C.byref(c), C.byref(s))
    return c.value, s.value


def glibc_sinf(y):
    return lib().orc_glibc_sinf(float(y))


def glibc_cosf(y):
    return lib().orc_glibc_cosf(float(y))


def sincosf_check(lo, hi, stride):
    """Mismatches of the glibc sinf/cosf restatement against the linked libm over every
    `stride`-th float bit pattern in [lo, hi)."""
    return int(lib().orc_sincosf_check(int(lo), int(hi), int(stride)))


def descriptor_distance(a, b):
    a = np.ascontiguousarray(a, np.uint8)
    b = np.ascontiguousarray(b, np.uint8)
    return lib().orc_descriptor_distance(_p(a), _p(b))


def knn2(qdesc, tdesc):
    qdesc = np.ascontiguousarray(qdesc, np.uint8)
    tdesc = np.ascontiguousarray(tdesc, np.uint8)
    nq, nt = len(qdesc), len(tdesc)
    bi = np.zeros(nq, np.int32)
    bd = np.zeros(nq, np.int32)
    sd = np.zeros(nq, np.int32)
    lib().orc_knn2(_p(qdesc), nq, _p(tdesc), nt, _p(bi), _p(bd), _p(sd))
    return bi, bd, sd


def search_for_initialization(kps1, desc1, kps2, desc2, prev_xy, bounds, window=100,
                              nnratio=0.9, check_ori=True):
    kps1 = np.ascontiguousarray(kps1, KP_DTYPE)
    kps2 = np.ascontiguousarray(kps2, KP_DTYPE)
    desc1 = np.ascontiguousarray(desc1, np.uint8)
    desc2 = np.ascontiguousarray(desc2, np.uint8)
    prev = np.ascontiguousarray(prev_xy, np.float32).copy()
    m12 = np.zeros(len(kps1), np.int32)
    b = Bounds(*[float(v) for v in bounds])
    n = lib().orc_search_for_initialization(_p(kps1), _p(desc1), len(kps1), _p(kps2), _p(desc2),
                                            len(kps2), C.byref(b), _p(prev), _p(m12), window,
                                            nnratio, 1 if check_ori else 0)
    return n, m12, prev


def stereo_matches(p, left, right, w, h, bf, min_z):
    """Frame::ComputeStereoMatches restated (oracle/stereo_oracle.c).  left / right are
    extract(..., with_pyramid=True) results of the two images.  Returns (uRight, depth)
    float32 arrays over the left keypoints (-1 where unmatched)."""
    def packed(r):
        return np.ascontiguousarray(np.concatenate([lv.reshape(-1) for lv in r["pyramid"]]))
    kl = np.ascontiguousarray(left["kps"], KP_DTYPE)
    kr = np.ascontiguousarray(right["kps"], KP_DTYPE)
    dl = np.ascontiguousarray(left["desc"], np.uint8)
    dr = np.ascontiguousarray(right["desc"], np.uint8)
    ur = np.zeros(max(len(kl), 1), np.float32)
    dp = np.zeros(max(len(kl), 1), np.float32)
    pl, pr = packed(left), packed(right)
    lib().orc_stereo_matches(C.byref(p), _p(kl), _p(dl), len(kl), _p(kr), _p(dr), len(kr),
                             _p(pl), _p(pr), w, h, float(bf), float(min_z), _p(ur), _p(dp))
    return ur[:len(kl)].copy(), dp[:len(kl)].copy()


def _frame_args(kps, desc, uright, taken0):
    kps = np.ascontiguousarray(kps, KP_DTYPE)
    desc = np.ascontiguousarray(desc, np.uint8)
    ur = None if uright is None else np.ascontiguousarray(uright, np.float32)
    tk = None if taken0 is None else np.ascontiguousarray(taken0, np.uint8)
    return kps, desc, ur, tk


def track_direction(cam):
    f, b = C.c_int(), C.c_int()
    lib().orc_track_direction(C.byref(cam), C.byref(f), C.byref(b))
    return f.value, b.value


def search_by_projection_lastframe(kps, desc, uright, taken0, bounds, scale_factors, pts, pdesc,
                                   cam, th, check_ori=True):
    """ORBmatcher::SearchByProjection(CurrentFrame, LastFrame, th, bMono) restated
    (oracle/track_oracle.c).  Returns (nmatches, match[n]: LastFrame point index or -1)."""
    kps, desc, ur, tk = _frame_args(kps, desc, uright, taken0)
    pts = np.ascontiguousarray(pts, LF_DTYPE)
    pdesc = np.ascontiguousarray(pdesc, np.uint8)
    sf = np.ascontiguousarray(scale_factors, np.float32)
    match = np.zeros(max(len(kps), 1), np.int32)
    b = Bounds(*[float(v) for v in bounds])
    n = lib().orc_search_by_projection_lastframe(_p(kps), _p(desc), _p(ur), len(kps), _p(tk),
                                                 C.byref(b), _p(sf), _p(pts), _p(pdesc),
                                                 len(pts), C.byref(cam), float(th),
                                                 1 if check_ori else 0, _p(match))
    return n, match[:len(kps)].copy()


def search_by_projection_local(kps, desc, uright, taken0, bounds, scale_factors, mps, mdesc,
                               th=1.0, nnratio=0.8):
    """ORBmatcher(nnratio).SearchByProjection(F, vpMapPoints, th) restated.  Returns
    (nmatches, match[n]: map point index written by the call or -1)."""
    kps, desc, ur, tk = _frame_args(kps, desc, uright, taken0)
    mps = np.ascontiguousarray(mps, MP_DTYPE)
    mdesc = np.ascontiguousarray(mdesc, np.uint8)
    sf = np.ascontiguousarray(scale_factors, np.float32)
    match = np.zeros(max(len(kps), 1), np.int32)
    b = Bounds(*[float(v) for v in bounds])
    n = lib().orc_search_by_projection_local(_p(kps), _p(desc), _p(ur), len(kps), _p(tk),
                                             C.byref(b), _p(sf), _p(mps), _p(mdesc), len(mps),
                                             float(th), float(nnratio), _p(match))
    return n, match[:len(kps)].copy()


def frames_batch(p, imgs, nthreads=1, window=100, nnratio=0.9):
    imgs = np.ascontiguousarray(imgs, np.uint8)
    nf, h, w = imgs.shape
    nkp = np.zeros(nf, np.int32)
    nm = np.zeros(nf, np.int32)
    lib().orc_frames_batch(C.byref(p), _p(imgs), nf, w, h, nthreads, window, nnratio, _p(nkp),
                           _p(nm))
    return nkp, nm


def frames_full(p, imgs, nthreads=1, window=100, nnratio=0.9):
    """The bench unit on every frame of `imgs`, every output kept (orc_frames_full): frame f
    is extracted and matched against frame f-1 (cyclic: frame 0 against the last).  Returns
    (nkp[f], nmatches[f], kps[f] (list of KP_DTYPE arrays), desc[f], knn[f] (nkp[f] x 3:
    best idx, best, second over frame f-1), m12[f] (vnMatches12 of pair (f-1, f), nkp[f-1]
    entries))."""
    imgs = np.ascontiguousarray(imgs, np.uint8)
    nf, h, w = imgs.shape
    cap = 2 * p.nfeatures + 256
    nkp = np.zeros(nf, np.int32)
    nm = np.zeros(nf, np.int32)
    kps = np.zeros((nf, cap), KP_DTYPE)
    desc = np.zeros((nf, cap, 32), np.uint8)
    knn = np.zeros((nf, cap, 3), np.int32)
    m12 = np.zeros((nf, cap), np.int32)
    lib().orc_frames_full(C.byref(p), _p(imgs), nf, w, h, nthreads, window, nnratio, _p(nkp),
                          _p(nm), cap, _p(kps), _p(desc), _p(knn), _p(m12))
    return (nkp, nm, [kps[f, :nkp[f]] for f in range(nf)], [desc[f, :nkp[f]] for f in range(nf)],
            [knn[f, :nkp[f]] for f in range(nf)],
            [m12[f, :nkp[(f - 1) % nf]] for f in range(nf)])


def ba_linearize(poses, points, edges):
    poses = np.ascontiguousarray(poses, POSE_DTYPE)
    points = np.ascontiguousarray(points, np.float64)
    edges = np.ascontiguousarray(edges, EDGE_DTYPE)
    npose, npoint, nedge = len(poses), len(points), len(edges)
    eout = np.zeros(nedge, EDGE_OUT_DTYPE)
    hpose = np.zeros((npose, 6, 6))
    bpose = np.zeros((npose, 6))
    hpoint = np.zeros((npoint, 3, 3))
    bpoint = np.zeros((npoint, 3))
    lib().orc_ba_linearize(_p(poses), npose, _p(points), npoint, _p(edges), nedge, _p(eout),
                           _p(hpose), _p(bpose), _p(hpoint), _p(bpoint))
    return eout, hpose, bpose, hpoint, bpoint


def ba_errors(poses, points, edges):
    """computeActiveErrors + activeRobustChi2 + isDepthPositive restated (orc_ba_errors):
    returns (err (n, 3), chi2 (n,), rho0 (n,), depth_ok (n,) bool, active robust chi2 sum)."""
    poses = np.ascontiguousarray(poses, POSE_DTYPE)
    points = np.ascontiguousarray(points, np.float64)
    edges = np.ascontiguousarray(edges, EDGE_DTYPE)
    n = len(edges)
    err = np.zeros((max(n, 1), 3))
    chi2 = np.zeros(max(n, 1))
    rho0 = np.zeros(max(n, 1))
    dok = np.zeros(max(n, 1), np.uint8)
    tot = lib().orc_ba_errors(_p(poses), _p(points), _p(edges), n, _p(err), _p(chi2), _p(rho0),
                              _p(dok))
    return err[:n], chi2[:n], rho0[:n], dok[:n].astype(bool), tot


def match_pose(p, kps1, kps2, m12, cam, depth):
    """The batched-sequence per-frame pose (orc_match_pose): PoseOptimization of frame 2 over
    vnMatches12 with F1's keypoints back-projected at `depth`.  cam = (fx, fy, cx, cy, bf).
    Returns (ninliers, q (x, y, z, w), t)."""
    k1 = np.ascontiguousarray(kps1, KP_DTYPE)
    k2 = np.ascontiguousarray(kps2, KP_DTYPE)
    m = np.ascontiguousarray(m12, np.int32)
    c = PoseCam(*[float(np.float32(v)) for v in cam], 0.0)
    inv2 = np.ascontiguousarray(np.asarray(p.inv_sigma2[:p.nlevels], np.float32))
    q = np.zeros(4)
    t = np.zeros(3)
    n = lib().orc_match_pose(_p(k1), len(k1), _p(k2), len(k2), _p(m), C.byref(c),
                             float(depth), _p(inv2), _p(q), _p(t))
    return n, q, t


def se3_to_tcw(q, t):
    """Converter::toCvMat(SE3Quat) restated (orc_se3_to_tcw): rows 0..2 of the float pose."""
    q = np.ascontiguousarray(q, np.float64)
    t = np.ascontiguousarray(t, np.float64)
    T = np.zeros(12, np.float32)
    lib().orc_se3_to_tcw(_p(q), _p(t), _p(T))
    return T


def se3_from_tcw(Tcw):
    """Converter::toSE3Quat restated (orc_se3_from_tcw): rows 0..2 of a float pose ->
    (q (x, y, z, w) normalised, t)."""
    T = np.ascontiguousarray(np.asarray(Tcw, np.float32).reshape(-1)[:12])
    q = np.zeros(4)
    t = np.zeros(3)
    lib().orc_se3_from_tcw(_p(T), _p(q), _p(t))
    return q, t


def ba_numeric_jacobian(pose, xyz, edge):
    pose = np.ascontiguousarray(np.asarray(pose, POSE_DTYPE).reshape(1))
    xyz = np.ascontiguousarray(xyz, np.float64)
    edge = np.ascontiguousarray(np.asarray(edge, EDGE_DTYPE).reshape(1))
    jp = np.zeros((3, 3))
    jt = np.zeros((3, 6))
    lib().orc_ba_numeric_jacobian(_p(pose), _p(xyz), _p(edge), _p(jp), _p(jt))
    return jp, jt


def pose_optimization(edges, cam, Tcw):
    """Optimizer::PoseOptimization restated (oracle/pose_oracle.c).  edges: PEDGE_DTYPE,
    cam: (fx, fy, cx, cy, bf), Tcw: (3, 4) float32.  Returns (ninliers, q (x,y,z,w),
    t, Tcw_out (3, 4) float32, outlier (n,) bool)."""
    e = np.ascontiguousarray(edges, PEDGE_DTYPE)
    c = PoseCam(*[float(np.float32(v)) for v in cam], 0.0)
    T = np.ascontiguousarray(np.asarray(Tcw, np.float32).reshape(12))
    q = np.zeros(4)
    t = np.zeros(3)
    To = np.zeros(12, np.float32)
    out = np.zeros(max(len(e), 1), np.uint8)
    n = lib().orc_pose_optimization(_p(e), len(e), C.byref(c), _p(T), _p(q), _p(t), _p(To),
                                    _p(out))
    return n, q, t, To.reshape(3, 4), out[:len(e)].astype(bool)


def ba_schur_solve(poses, npoint, edges, eout, hpose, bpose, hpoint, bpoint, lam):
    """g2o BlockSolver_6_3::solve (Schur) after setLambda(lam) on ba_linearize's outputs.
    Returns (ok, dx_pose (npose, 6), dx_point (npoint, 3))."""
    poses = np.ascontiguousarray(poses, POSE_DTYPE)
    edges = np.ascontiguousarray(edges, EDGE_DTYPE)
    eout = np.ascontiguousarray(eout, EDGE_OUT_DTYPE)
    hp, bp = np.ascontiguousarray(hpose, np.float64), np.ascontiguousarray(bpose, np.float64)
    hq, bq = np.ascontiguousarray(hpoint, np.float64), np.ascontiguousarray(bpoint, np.float64)
    dp = np.zeros((max(len(poses), 1), 6))
    dq = np.zeros((max(npoint, 1), 3))
    ok = lib().orc_ba_schur_solve(_p(poses), len(poses), npoint, _p(edges), len(edges), _p(eout),
                                  _p(hp), _p(bp), _p(hq), _p(bq), float(lam), _p(dp), _p(dq))
    return bool(ok), dp[:len(poses)], dq[:npoint]


def ba_update(poses, points, dx_pose, dx_point):
    """SparseOptimizer::update restated (orc_ba_update): returns updated copies."""
    poses = np.array(poses, POSE_DTYPE)
    points = np.array(points, np.float64)
    dp = np.ascontiguousarray(dx_pose, np.float64)
    dq = np.ascontiguousarray(dx_point, np.float64)
    lib().orc_ba_update(_p(poses), len(poses), _p(points), len(points), _p(dp), _p(dq))
    return poses, points


def ba_optimize(poses, points, edges, iterations):
    """optimizer.optimize(iterations) with g2o's Levenberg-Marquardt restated
    (orc_ba_optimize): returns (poses, points, report dict)."""
    poses = np.array(poses, POSE_DTYPE)
    points = np.array(points, np.float64)
    edges = np.ascontiguousarray(edges, EDGE_DTYPE)
    rep = np.zeros(6)
    lib().orc_ba_optimize(_p(poses), len(poses), _p(points), len(points), _p(edges), len(edges),
                          int(iterations), _p(rep))
    return poses, points, dict(iterations=int(rep[0]), trials=int(rep[1]),
                               terminated=int(rep[2]), initial_chi2=rep[3], final_chi2=rep[4],
                               **{"lambda": rep[5]})


def ba_optimize_ctl(poses, points, edges, iterations, stop_it=-1, stop_trial=-1, last_chi2=None):
    """optimize(iterations) with g2o's force-stop flag raised after trial `stop_trial` of
    iteration `stop_it` (-1: after that iteration; stop_it -1: never, -2: before the call),
    restated (orc_ba_optimize_ctl).  `last_chi2` (float64 [nedge], updated in place when an
    iteration ran): the chi2 g2o's edges hold afterwards.  Returns (poses, points, report)."""
    poses = np.array(poses, POSE_DTYPE)
    points = np.array(points, np.float64)
    edges = np.ascontiguousarray(edges, EDGE_DTYPE)
    rep = np.zeros(6)
    if last_chi2 is not None:
        assert last_chi2.dtype == np.float64 and last_chi2.flags.c_contiguous
        assert len(last_chi2) == len(edges)
    lib().orc_ba_optimize_ctl(_p(poses), len(poses), _p(points), len(points), _p(edges),
                              len(edges), int(iterations), int(stop_it), int(stop_trial),
                              _p(last_chi2), _p(rep))
    return poses, points, dict(iterations=int(rep[0]), trials=int(rep[1]),
                               terminated=int(rep[2]), initial_chi2=rep[3], final_chi2=rep[4],
                               **{"lambda": rep[5]})


class Vocab:
    """Flat vocabulary for oracle/bow_oracle.c, built from the loadFromTextFile node list
    (TemplatedVocabulary.h:1376-1417): children in node order, leaves numbered in order."""

    def __init__(self, k, L, scoring, weighting, parent, is_leaf, desc, weight):
        parent = np.asarray(parent, np.int64)
        n = len(parent)
        is_leaf = np.asarray(is_leaf).astype(bool)
        is_leaf[0] = False
        self.desc = np.ascontiguousarray(np.asarray(desc, np.uint8).reshape(n, 32))
        self.weight = np.ascontiguousarray(weight, np.float64)
        self.word_id = np.zeros(n, np.int32)
        self.word_id[is_leaf] = np.arange(int(is_leaf.sum()), dtype=np.int32)
        cnt = np.bincount(parent[1:], minlength=n) if n > 1 else np.zeros(n, np.int64)
        self.child_off = np.zeros(n + 1, np.int32)
        self.child_off[1:] = np.cumsum(cnt)
        order = np.argsort(parent[1:], kind="stable") + 1
        self.child_idx = np.ascontiguousarray(order, np.int32) if n > 1 else np.zeros(1, np.int32)
        self.s = OrcVocab(k, L, scoring, weighting, n, int(is_leaf.sum()), _p(self.desc),
                          _p(self.weight), _p(self.word_id), _p(self.child_off),
                          _p(self.child_idx))


def bow_word(voc, feat, levelsup):
    """single-feature transform (TemplatedVocabulary.h:1220-1259): (word, weight, nid)"""
    w, x, nid = C.c_int32(), C.c_double(), C.c_int32(-7)
    f = np.ascontiguousarray(feat, np.uint8)
    lib().orc_bow_word(C.byref(voc.s), _p(f), levelsup, C.byref(w), C.byref(x), C.byref(nid))
    return w.value, x.value, nid.value


def bow_transform(voc, desc, levelsup):
    """transform(features, BowVector, FeatureVector, levelsup) -> (bow_words, bow_weights,
    fv_nodes, fv_off, fv_feats)."""
    d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
    n = len(d)
    cap = max(n, 1)
    bw, bx = np.zeros(cap, np.int32), np.zeros(cap)
    vn, vo, vf = np.zeros(cap, np.int32), np.zeros(cap + 1, np.int32), np.zeros(cap, np.int32)
    nb, nf = C.c_int(), C.c_int()
    lib().orc_bow_transform(C.byref(voc.s), _p(d), n, levelsup, _p(bw), _p(bx), C.byref(nb),
                            _p(vn), _p(vo), _p(vf), C.byref(nf))
    nb, nf = nb.value, nf.value
    return bw[:nb], bx[:nb], vn[:nf], vo[:nf + 1], vf[:vo[nf]]


def search_by_bow(kf_desc, kf_angle, kf_valid, kf_fv, f_desc, f_angle, f_fv, nnratio=0.75,
                  check_ori=True):
    """ORBmatcher::SearchByBoW(KeyFrame*, Frame&, ...) restated (orc_search_by_bow,
    bow_oracle.c).  kf_fv / f_fv = (fv_nodes, fv_off, fv_feats) as bow_transform returns them;
    kf_valid[i] = pMP && !pMP->isBad() (None: all).  Returns (nmatches, match[n_f]) with
    match[i] = the KF feature whose MapPoint matched F's feature i, -1 if none."""
    kd = np.ascontiguousarray(kf_desc, np.uint8).reshape(-1, 32)
    fd = np.ascontiguousarray(f_desc, np.uint8).reshape(-1, 32)
    ka = np.ascontiguousarray(kf_angle, np.float32)
    fa = np.ascontiguousarray(f_angle, np.float32)
    kv = (np.ones(len(kd), np.uint8) if kf_valid is None
          else np.ascontiguousarray(kf_valid, np.uint8))
    kn, ko, kfe = [np.ascontiguousarray(a, np.int32) for a in kf_fv]
    fn, fo, ffe = [np.ascontiguousarray(a, np.int32) for a in f_fv]
    match = np.zeros(max(len(fd), 1), np.int32)
    n = lib().orc_search_by_bow(_p(kd), _p(ka), _p(kv), len(kd), _p(kn), _p(ko), _p(kfe), len(kn),
                                _p(fd), _p(fa), len(fd), _p(fn), _p(fo), _p(ffe), len(fn),
                                float(nnratio), int(bool(check_ori)), _p(match))
    return n, match[:len(fd)].copy()


def search_by_bow_kf(desc1, angle1, valid1, fv1, desc2, angle2, valid2, fv2, nnratio=0.75,
                     check_ori=True):
    """ORBmatcher::SearchByBoW(KeyFrame*, KeyFrame*, vpMatches12) restated
    (orc_search_by_bow_kf): valid = pMP && !pMP->isBad() per side (None: all).  Returns
    (nmatches, match12[n1]) with match12[i] = the KF2 feature matched to KF1 feature i, -1."""
    d1 = np.ascontiguousarray(desc1, np.uint8).reshape(-1, 32)
    d2 = np.ascontiguousarray(desc2, np.uint8).reshape(-1, 32)
    a1 = np.ascontiguousarray(angle1, np.float32)
    a2 = np.ascontiguousarray(angle2, np.float32)
    v1 = np.ones(len(d1), np.uint8) if valid1 is None else np.ascontiguousarray(valid1, np.uint8)
    v2 = np.ones(len(d2), np.uint8) if valid2 is None else np.ascontiguousarray(valid2, np.uint8)
    n1, o1, f1 = [np.ascontiguousarray(a, np.int32) for a in fv1]
    n2, o2, f2 = [np.ascontiguousarray(a, np.int32) for a in fv2]
    m = np.zeros(max(len(d1), 1), np.int32)
    n = lib().orc_search_by_bow_kf(_p(d1), _p(a1), _p(v1), len(d1), _p(n1), _p(o1), _p(f1),
                                   len(n1), _p(d2), _p(a2), _p(v2), len(d2), _p(n2), _p(o2),
                                   _p(f2), len(n2), float(nnratio), int(bool(check_ori)), _p(m))
    return n, m[:len(d1)].copy()


# ---- Frame / MapPoint geometry (frame_oracle.c) ----
def camera(fx, fy, cx, cy, k1=0.0, k2=0.0, p1=0.0, p2=0.0, k3=0.0):
    c = np.zeros((), CAMERA_DTYPE)
    for k, v in zip(CAMERA_DTYPE.names, (fx, fy, cx, cy, k1, k2, p1, p2, k3)):
        c[k] = v
    return c


def undistort_points(cam, xy):
    """cv::undistortPoints(xy, K, D, noArray(), K): xy (n, 2) float32."""
    cam = np.ascontiguousarray(cam, CAMERA_DTYPE)
    xy = np.ascontiguousarray(xy, np.float32).reshape(-1, 2)
    out = np.zeros_like(xy)
    lib().orc_undistort_points(_p(cam), _p(xy), len(xy), _p(out))
    return out


def undistort_keypoints(cam, kps):
    """Frame::UndistortKeyPoints: mvKeysUn."""
    cam = np.ascontiguousarray(cam, CAMERA_DTYPE)
    kps = np.ascontiguousarray(kps, KP_DTYPE)
    out = np.zeros_like(kps)
    lib().orc_undistort_keypoints(_p(cam), _p(kps), len(kps), _p(out))
    return out


def image_bounds(cam, w, h):
    """Frame::ComputeImageBounds: (min_x, max_x, min_y, max_y)."""
    cam = np.ascontiguousarray(cam, CAMERA_DTYPE)
    b = Bounds()
    lib().orc_image_bounds(_p(cam), int(w), int(h), C.byref(b))
    return (b.min_x, b.max_x, b.min_y, b.max_y)


def log_scale_factor(sf):
    return lib().orc_log_scale_factor(float(sf))


def is_in_frustum(fcam, mps, viewing_cos_limit=0.5, proj=None):
    """Frame::isInFrustum over map points: (MP_DTYPE projections, number in view).  proj:
    the records' values before the call (only the flags of a point out of view change)."""
    fcam = np.ascontiguousarray(fcam, FRUSTUM_DTYPE)
    mps = np.ascontiguousarray(mps, MAPPOINT_DTYPE)
    out = np.zeros(len(mps), MP_DTYPE) if proj is None else np.array(proj, MP_DTYPE)
    n = lib().orc_is_in_frustum_n(_p(fcam), _p(mps), len(mps), float(viewing_cos_limit), _p(out))
    return out, n


def distinctive_descriptor(desc):
    """MapPoint::ComputeDistinctiveDescriptors over one point's observation rows: BestIdx."""
    desc = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
    return lib().orc_distinctive_descriptor(_p(desc), len(desc))


def distinctive_descriptors(pool, rows, off):
    pool = np.ascontiguousarray(pool, np.uint8).reshape(-1, 32)
    rows = np.ascontiguousarray(rows, np.int32)
    off = np.ascontiguousarray(off, np.int32)
    best = np.zeros(len(off) - 1, np.int32)
    lib().orc_distinctive_descriptors_n(_p(pool), _p(rows), _p(off), len(off) - 1, _p(best))
    return best


# ---- LocalMapping matchers (mapping_oracle.c) ----
def _tri_kf(kf, keep):
    """kf: dict(kps, desc, uright, has_mp, fv=(nodes, off, feats)) -> TriKF (arrays kept alive
    in `keep`)."""
    kps = np.ascontiguousarray(kf["kps"], KP_DTYPE)
    n = len(kps)
    desc = np.ascontiguousarray(kf["desc"], np.uint8).reshape(-1, 32)
    ur = kf.get("uright")
    ur = np.full(max(n, 1), -1.0, np.float32) if ur is None else np.ascontiguousarray(ur, np.float32)
    mp = kf.get("has_mp")
    mp = np.zeros(max(n, 1), np.uint8) if mp is None else np.ascontiguousarray(mp, np.uint8)
    nodes, off, feats = (np.ascontiguousarray(a, np.int32) for a in kf["fv"])
    keep += [kps, desc, ur, mp, nodes, off, feats]
    return TriKF(_p(kps), _p(desc), _p(ur), _p(mp), n, _p(nodes), _p(off), _p(feats), len(nodes))


def search_for_triangulation(kf1, kf2, geom, scale_factors, sigma2, only_stereo=False,
                             check_ori=False):
    """ORBmatcher(0.6, check_ori).SearchForTriangulation -> (nmatches, vMatches12)."""
    keep = []
    a, b = _tri_kf(kf1, keep), _tri_kf(kf2, keep)
    g = np.ascontiguousarray(geom, TRI_GEOM_DTYPE)
    sf = np.ascontiguousarray(scale_factors, np.float32)
    s2 = np.ascontiguousarray(sigma2, np.float32)
    m = np.zeros(max(a.n, 1), np.int32)
    n = lib().orc_search_for_triangulation(C.byref(a), C.byref(b), _p(g), _p(sf), _p(s2),
                                           int(only_stereo), int(check_ori), _p(m))
    return n, m[:a.n]


def atan2f(y, x):
    """glibc atan2f restated (orc_atan2f)."""
    return lib().orc_atan2f(float(y), float(x))


def atan2f_check(seed, n):
    """Bit mismatches of orc_atan2f vs the host libm's atan2f over n sampled pairs."""
    return lib().orc_atan2f_check(int(seed), int(n))


def kf_cam(Tcw, fx, fy, cx, cy, mb=0.0, mbf=0.0):
    """orc_kf_cam of a KeyFrame: Tcw (3x4 float32), intrinsics, invfx = 1/fx (Frame.cc
    float division), mb, mbf."""
    c = np.zeros((), KF_CAM_DTYPE)
    c["Tcw"] = np.asarray(Tcw, np.float32).reshape(-1)[:12]
    c["fx"], c["fy"], c["cx"], c["cy"] = fx, fy, cx, cy
    c["invfx"] = np.float32(1.0) / np.float32(fx)
    c["invfy"] = np.float32(1.0) / np.float32(fy)
    c["mb"], c["mbf"] = mb, mbf
    return c


def tri_geometry(c1, c2):
    """LocalMapping::ComputeF12(pKF1, pKF2) + the SearchForTriangulation geometry record."""
    a = np.ascontiguousarray(c1, KF_CAM_DTYPE)
    b = np.ascontiguousarray(c2, KF_CAM_DTYPE)
    g = np.zeros((), TRI_GEOM_DTYPE)
    lib().orc_tri_geometry(_p(a), _p(b), _p(g))
    return g


def tri_nullvec(A):
    """The oracle's cv::SVD stand-in: null vector (double) of a 4x4 float matrix."""
    a = np.ascontiguousarray(A, np.float32).reshape(16)
    v = np.zeros(4, np.float64)
    lib().orc_tri_nullvec(_p(a), _p(v))
    return v


def _kf_tri(kf, keep):
    kps = np.ascontiguousarray(kf["kps"], KP_DTYPE)
    raw = kf.get("kps_raw")
    raw = None if raw is None else np.ascontiguousarray(raw, KP_DTYPE)
    ur = kf.get("uright")
    ur = None if ur is None else np.ascontiguousarray(ur, np.float32)
    dp = kf.get("depth")
    dp = None if dp is None else np.ascontiguousarray(dp, np.float32)
    keep += [kps, raw, ur, dp]
    return KFTri(_p(kps), _p(raw), _p(ur), _p(dp), len(kps))


def triangulate(kf1, kf2, c1, c2, matches12, scale_factors, sigma2, scale_factor):
    """CreateNewMapPoints' triangulation of the matched pairs -> (nnew, x3d[n1, 3], status[n1]).
    kf: dict(kps = mvKeysUn, kps_raw = mvKeys, uright, depth)."""
    keep = []
    a, b = _kf_tri(kf1, keep), _kf_tri(kf2, keep)
    ca = np.ascontiguousarray(c1, KF_CAM_DTYPE)
    cb = np.ascontiguousarray(c2, KF_CAM_DTYPE)
    m = np.ascontiguousarray(matches12, np.int32)
    assert len(m) == a.n
    sf = np.ascontiguousarray(scale_factors, np.float32)
    s2 = np.ascontiguousarray(sigma2, np.float32)
    x = np.zeros((max(a.n, 1), 3), np.float32)
    st = np.zeros(max(a.n, 1), np.int8)
    n = lib().orc_triangulate(C.byref(a), C.byref(b), _p(ca), _p(cb), _p(m), _p(sf), _p(s2),
                              float(scale_factor), _p(x), _p(st))
    return n, x[:a.n], st[:a.n]


def fuse_search(kf, fcam, mps, mdesc, th, scale_factors, inv_sigma2):
    """ORBmatcher::Fuse(pKF, vpMapPoints, th)'s search -> (nfused, best_idx, best_dist).
    kf: dict(kps, desc, uright) (mvKeysUn, mDescriptors, mvuRight)."""
    keep = []
    k = _tri_kf(dict(kf, fv=(np.zeros(0), np.zeros(1), np.zeros(0))), keep)
    fcam = np.ascontiguousarray(fcam, FRUSTUM_DTYPE)
    mps = np.ascontiguousarray(mps, MAPPOINT_DTYPE)
    md = np.ascontiguousarray(mdesc, np.uint8).reshape(-1, 32)
    sf = np.ascontiguousarray(scale_factors, np.float32)
    isg = np.ascontiguousarray(inv_sigma2, np.float32)
    bi = np.zeros(max(len(mps), 1), np.int32)
    bd = np.zeros(max(len(mps), 1), np.int32)
    n = lib().orc_fuse_search(C.byref(k), _p(fcam), _p(mps), _p(md), len(mps), float(th),
                              _p(sf), _p(isg), _p(bi), _p(bd))
    return n, bi[:len(mps)], bd[:len(mps)]


def sim3_decompose(Scw):
    """Rcw | tcw (3x4 float32) of Fuse(pKF, Scw, ...)'s decomposition (ORBmatcher.cc:1143-1148)."""
    S = np.ascontiguousarray(np.asarray(Scw, np.float32).reshape(-1)[:12])
    T = np.zeros(12, np.float32)
    lib().orc_sim3_decompose(_p(S), _p(T))
    return T.reshape(3, 4)


def fuse_sim3_search(kf, fcam, mps, mdesc, th, scale_factors):
    """ORBmatcher::Fuse(pKF, Scw, vpPoints, th, vpReplacePoint)'s search -> (nfused, best_idx,
    best_dist); fcam["Tcw"] holds Scw's rows 0..2.  kf: dict(kps, desc)."""
    keep = []
    kf = dict(kf, fv=(np.zeros(0), np.zeros(1), np.zeros(0)))
    if kf.get("uright") is None:
        kf["uright"] = np.full(len(kf["kps"]), -1, np.float32)
    k = _tri_kf(kf, keep)
    fcam = np.ascontiguousarray(fcam, FRUSTUM_DTYPE)
    mps = np.ascontiguousarray(mps, MAPPOINT_DTYPE)
    md = np.ascontiguousarray(mdesc, np.uint8).reshape(-1, 32)
    sf = np.ascontiguousarray(scale_factors, np.float32)
    bi = np.zeros(max(len(mps), 1), np.int32)
    bd = np.zeros(max(len(mps), 1), np.int32)
    n = lib().orc_fuse_sim3_search(C.byref(k), _p(fcam), _p(mps), _p(md), len(mps), float(th),
                                   _p(sf), _p(bi), _p(bd))
    return n, bi[:len(mps)], bd[:len(mps)]


def search_by_projection_reloc(kps, desc, taken0, fcam, scale_factors, pts, pdesc, th, orb_dist,
                               check_ori=True):
    """ORBmatcher::SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist)
    (oracle/loop_oracle.c).  fcam: CurrentFrame's FRUSTUM_DTYPE state; pts RELOC_DTYPE.
    Returns (nmatches, match[n]: pKF point index written, -1, or -2 NULLed by the rotation
    filter)."""
    kps, desc, _, tk = _frame_args(kps, desc, None, taken0)
    fcam = np.ascontiguousarray(fcam, FRUSTUM_DTYPE)
    pts = np.ascontiguousarray(pts, RELOC_DTYPE)
    pdesc = np.ascontiguousarray(pdesc, np.uint8)
    sf = np.ascontiguousarray(scale_factors, np.float32)
    match = np.zeros(max(len(kps), 1), np.int32)
    n = lib().orc_search_by_projection_reloc(_p(kps), _p(desc), len(kps), _p(tk), _p(fcam),
                                             _p(sf), _p(pts), _p(pdesc), len(pts), float(th),
                                             int(orb_dist), 1 if check_ori else 0, _p(match))
    return n, match[:len(kps)].copy()


def search_by_projection_sim3(kps, desc, taken0, fcam, scale_factors, mps, mdesc, th):
    """ORBmatcher::SearchByProjection(pKF, Scw, vpPoints, vpMatched, th) (oracle/loop_oracle.c):
    fcam["Tcw"] = Scw rows 0..2.  Returns (nmatches, match[n]: vpPoints index written, -1)."""
    kps, desc, _, tk = _frame_args(kps, desc, None, taken0)
    fcam = np.ascontiguousarray(fcam, FRUSTUM_DTYPE)
    mps = np.ascontiguousarray(mps, MAPPOINT_DTYPE)
    mdesc = np.ascontiguousarray(mdesc, np.uint8)
    sf = np.ascontiguousarray(scale_factors, np.float32)
    match = np.zeros(max(len(kps), 1), np.int32)
    n = lib().orc_search_by_projection_sim3(_p(kps), _p(desc), len(kps), _p(tk), _p(fcam),
                                            _p(sf), _p(mps), _p(mdesc), len(mps), int(th),
                                            _p(match))
    return n, match[:len(kps)].copy()


def search_by_sim3(kf1, mp1, md1, matched1, kf2, mp2, md2, matched2, g, th, scale_factors):
    """ORBmatcher::SearchBySim3 (oracle/loop_oracle.c) -> (nFound, matches12).  kf1 / kf2:
    dict(kps, desc); mp* MAPPOINT_DTYPE per KeyFrame slot; matched* uint8 or None; g a
    SIM3_PAIR_DTYPE record."""
    k1, d1, _, a1 = _frame_args(kf1["kps"], kf1["desc"], None, matched1)
    k2, d2, _, a2 = _frame_args(kf2["kps"], kf2["desc"], None, matched2)
    mp1 = np.ascontiguousarray(mp1, MAPPOINT_DTYPE)
    mp2 = np.ascontiguousarray(mp2, MAPPOINT_DTYPE)
    md1 = np.ascontiguousarray(md1, np.uint8)
    md2 = np.ascontiguousarray(md2, np.uint8)
    g = np.ascontiguousarray(g, SIM3_PAIR_DTYPE)
    sf = np.ascontiguousarray(scale_factors, np.float32)
    m = np.zeros(max(len(k1), 1), np.int32)
    n = lib().orc_search_by_sim3(_p(k1), _p(d1), len(k1), _p(mp1), _p(md1), _p(a1), _p(k2),
                                 _p(d2), len(k2), _p(mp2), _p(md2), _p(a2), _p(g), float(th),
                                 _p(sf), _p(m))
    return n, m[:len(k1)].copy()


def rgbd_stereo(depth, factor, kps, kps_un, mbf):
    """Frame::ComputeStereoFromRGBD after GrabImageRGBD's depth conversion (oracle/
    frame_oracle.c): depth a (h, w) uint16 or float32 image -> (uright, depth) per keypoint."""
    depth = np.ascontiguousarray(depth)
    assert depth.dtype in (np.uint16, np.float32)
    kps = np.ascontiguousarray(kps, KP_DTYPE)
    kun = np.ascontiguousarray(kps_un, KP_DTYPE)
    ur = np.zeros(max(len(kps), 1), np.float32)
    dd = np.zeros(max(len(kps), 1), np.float32)
    h, w = depth.shape
    lib().orc_rgbd_stereo(_p(depth), 1 if depth.dtype == np.uint16 else 0, float(factor), w, h,
                          depth.strides[0], _p(kps), _p(kun), len(kps), float(mbf), _p(ur), _p(dd))
    return ur[:len(kps)].copy(), dd[:len(kps)].copy()
