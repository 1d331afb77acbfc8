"""ctypes binding of liborbg.so (include/orbg.h).

The product path has no CPU fallback: if the HIP library is missing or no GPU is
visible, the calls below raise.  ``lib()`` loads ``orb_slam2_test_amd/lib/liborbg.so``
(built in-tree by ``csrc/Makefile`` / ``__graft_entry__.build()``).
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "liborbg.so")
if os.environ.get("ORBG_LIB_VARIANT"):  # developer A/B: a build in lib/<variant>/ (csrc make OUT=)
    LIB_PATH = os.path.join(HERE, "lib", os.environ["ORBG_LIB_VARIANT"], "liborbg.so")
MAX_LEVELS = 16

ORBG_OK = 0
ORBG_EIO = -5
ORBG_ENOMEM = -12
ORBG_EINVAL = -22
ORBG_ERANGE = -34
ORBG_ENOTSUP = -95

RESIZE_SCALAR, RESIZE_SSE2_16_4, RESIZE_SIMD_16_8 = 0, 4, 8
SINCOS_GLIBC, SINCOS_PINNED = 0, 1

# cv::KeyPoint layout (orbg_keypoint)
KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
POSE_DTYPE = np.dtype([("q", "<f8", 4), ("t", "<f8", 3), ("fixed", "<i4"), ("pad", "<i4")])
EDGE_DTYPE = np.dtype([("point", "<i4"), ("pose", "<i4"), ("stereo", "<i4"), ("robust", "<i4"),
                       ("active", "<i4"), ("pad", "<i4"), ("obs", "<f8", 3),
                       ("inv_sigma2", "<f8"), ("fx", "<f8"), ("fy", "<f8"), ("cx", "<f8"),
                       ("cy", "<f8"), ("bf", "<f8"), ("huber_delta", "<f8")])
EDGE_OUT_DTYPE = np.dtype([("err", "<f8", 3), ("chi2", "<f8"), ("rho1", "<f8"),
                           ("jp", "<f8", (3, 3)), ("jt", "<f8", (3, 6)), ("hpl", "<f8", (3, 6))])


# tracking matcher records (orbg_lastframe_point, orbg_map_projection)
MP_VALID, MP_HAS_OBS = 1, 2
TRACK_LASTFRAME, TRACK_LOCAL, TRACK_RELOC, TRACK_LOOP = 0, 1, 2, 3
DEPTH_F32, DEPTH_U16 = 0, 1
LF_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("octave", "<i4"),
                     ("angle", "<f4"), ("flags", "<i4")])
MP_DTYPE = np.dtype([("u", "<f4"), ("v", "<f4"), ("ur", "<f4"), ("level", "<i4"),
                     ("view_cos", "<f4"), ("flags", "<i4")])


# Frame / MapPoint geometry records (orbg_camera, orbg_map_point, orbg_frustum_camera)
CAMERA_DTYPE = np.dtype([("fx", "<f4"), ("fy", "<f4"), ("cx", "<f4"), ("cy", "<f4"),
                         ("k1", "<f4"), ("k2", "<f4"), ("p1", "<f4"), ("p2", "<f4"),
                         ("k3", "<f4")])
SIM3_PAIR_DTYPE = np.dtype([("T1w", "<f4", 12), ("T2w", "<f4", 12), ("R12", "<f4", 9),
                            ("t12", "<f4", 3), ("s12", "<f4"), ("fx", "<f4"), ("fy", "<f4"),
                            ("cx", "<f4"), ("cy", "<f4"), ("log_scale_factor", "<f4"),
                            ("nlevels", "<i4"), ("min_x", "<f4"), ("max_x", "<f4"),
                            ("min_y", "<f4"), ("max_y", "<f4")])
RELOC_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("min_dist", "<f4"),
                        ("max_dist", "<f4"), ("angle", "<f4"), ("flags", "<i4")])
MAPPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("nx", "<f4"),
                           ("ny", "<f4"), ("nz", "<f4"), ("min_dist", "<f4"),
                           ("max_dist", "<f4"), ("flags", "<i4")])
FRUSTUM_DTYPE = np.dtype([("Tcw", "<f4", 12), ("fx", "<f4"), ("fy", "<f4"), ("cx", "<f4"),
                          ("cy", "<f4"), ("bf", "<f4"), ("log_scale_factor", "<f4"),
                          ("nlevels", "<i4"), ("min_x", "<f4"), ("max_x", "<f4"),
                          ("min_y", "<f4"), ("max_y", "<f4")])


TRI_GEOM_DTYPE = np.dtype([("F12", "<f4", 9), ("Cw1", "<f4", 3), ("Tcw2", "<f4", 12),
                           ("fx2", "<f4"), ("fy2", "<f4"), ("cx2", "<f4"), ("cy2", "<f4")])


# CreateNewMapPoints (include/orbg.h orbg_kf_camera, ORBG_TRI_*)
KF_CAMERA_DTYPE = np.dtype([("Tcw", "<f4", 12), ("fx", "<f4"), ("fy", "<f4"), ("cx", "<f4"),
                            ("cy", "<f4"), ("invfx", "<f4"), ("invfy", "<f4"), ("mb", "<f4"),
                            ("mbf", "<f4")])
TRI_NONE, TRI_NEW, TRI_PARALLAX, TRI_W0, TRI_Z1, TRI_Z2 = 0, 1, -1, -2, -3, -4
TRI_REPROJ1, TRI_REPROJ2, TRI_DIST0, TRI_SCALE = -5, -6, -7, -8


class KeyFrameGeo(C.Structure):
    """orbg_keyframe_geo (include/orbg.h): one KeyFrame's triangulation inputs, host arrays."""
    _fields_ = [("kps", C.c_void_p), ("kps_raw", C.c_void_p), ("uright", C.c_void_p),
                ("depth", C.c_void_p), ("n", C.c_int32)]


class LmReport(C.Structure):
    """orbg_lm_report (include/orbg.h)."""
    _fields_ = [("iterations", C.c_int32), ("trials", C.c_int32), ("terminated", C.c_int32),
                ("pad", C.c_int32), ("initial_chi2", C.c_double), ("final_chi2", C.c_double),
                ("lam", C.c_double)]


LM_POST_ITERATION = C.CFUNCTYPE(None, C.c_void_p, C.c_int)
LM_POST_TRIAL = C.CFUNCTYPE(None, C.c_void_p, C.c_int, C.c_int)


class LmControl(C.Structure):
    """orbg_lm_control (include/orbg.h): g2o's force-stop flag and iteration actions."""
    _fields_ = [("force_stop", C.c_void_p), ("post_iteration", LM_POST_ITERATION),
                ("post_trial", LM_POST_TRIAL), ("user", C.c_void_p),
                ("d_last_chi2", C.c_void_p)]


class KeyFrames(C.Structure):
    """orbg_keyframes (include/orbg.h): a set of KeyFrames in device memory."""
    _fields_ = [("desc", C.c_void_p), ("kps", C.c_void_p), ("uright", C.c_void_p),
                ("has_mp", C.c_void_p), ("counts", C.c_void_p), ("fv_nodes", C.c_void_p),
                ("fv_off", C.c_void_p), ("fv_feats", C.c_void_p), ("nfv", C.c_void_p)]


class KeyFrame(C.Structure):
    """orbg_keyframe (include/orbg.h): one KeyFrame from host arrays."""
    _fields_ = [("kps", C.c_void_p), ("desc", C.c_void_p), ("uright", C.c_void_p),
                ("has_mp", C.c_void_p), ("n", C.c_int32), ("fv_nodes", C.c_void_p),
                ("fv_off", C.c_void_p), ("fv_feats", C.c_void_p), ("nfv", C.c_int32)]


PEDGE_DTYPE = np.dtype([("obs", "<f4", 3), ("xw", "<f4", 3), ("inv_sigma2", "<f4"),
                        ("stereo", "<i4")])


class PoseCamera(C.Structure):
    _fields_ = [("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float),
                ("bf", C.c_float), ("pad", C.c_float)]


class TrackCamera(C.Structure):
    _fields_ = [("Tcw", C.c_float * 12), ("Tlw", C.c_float * 12), ("fx", C.c_float),
                ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float), ("bf", C.c_float),
                ("b", C.c_float), ("mono", C.c_int32), ("pad", C.c_int32)]


class TrackBatch(C.Structure):
    _fields_ = [("kps", C.c_void_p), ("desc", C.c_void_p), ("uright", C.c_void_p),
                ("taken0", C.c_void_p), ("counts", C.c_void_p), ("bounds", C.c_void_p),
                ("frame_cap", C.c_int32), ("queries", C.c_void_p), ("qdesc", C.c_void_p),
                ("qcounts", C.c_void_p), ("query_cap", C.c_int32), ("cams", C.c_void_p),
                ("th", C.c_float), ("nnratio", C.c_float), ("check_ori", C.c_int32),
                ("match", C.c_void_p), ("nmatches", C.c_void_p), ("fcams", C.c_void_p),
                ("orb_dist", C.c_int32)]


def track_camera(Tcw, Tlw, fx, fy, cx, cy, bf, b, mono):
    c = TrackCamera()
    for i, v in enumerate(np.asarray(Tcw, np.float32).reshape(12)):
        c.Tcw[i] = float(v)
    for i, v in enumerate(np.asarray(Tlw, np.float32).reshape(12)):
        c.Tlw[i] = float(v)
    c.fx, c.fy, c.cx, c.cy, c.bf, c.b = (float(np.float32(v)) for v in (fx, fy, cx, cy, bf, b))
    c.mono = 1 if mono else 0
    return c


class Params(C.Structure):
    _fields_ = [("nfeatures", C.c_int32), ("scale_factor", C.c_float), ("nlevels", C.c_int32),
                ("ini_th_fast", C.c_int32), ("min_th_fast", C.c_int32),
                ("resize_mode", C.c_int32), ("gauss_k", C.c_int32 * 7),
                ("brief_fma", C.c_int32), ("max_batch", C.c_int32), ("sincos_mode", C.c_int32)]


class Bounds(C.Structure):
    _fields_ = [("min_x", C.c_float), ("max_x", C.c_float), ("min_y", C.c_float),
                ("max_y", C.c_float)]


class OrbgError(RuntimeError):
    def __init__(self, code, what):
        super().__init__("%s failed (%d): %s" % (what, code, last_error()))
        self.code = code


class BowFrames(C.Structure):
    """orbg_bow_frames (include/orbg.h): one side of SearchByBoW pairs, device pointers."""
    _fields_ = [("desc", C.c_void_p), ("kps", C.c_void_p), ("counts", C.c_void_p),
                ("fv_nodes", C.c_void_p), ("fv_off", C.c_void_p), ("fv_feats", C.c_void_p),
                ("nfv", C.c_void_p), ("valid", C.c_void_p)]


_lib = None


def lib():
    """Load liborbg.so; raises if it is absent (no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError("liborbg.so not built at %s: run __graft_entry__.build() "
                           "(the product has no CPU fallback)" % LIB_PATH)
    # One HIP runtime per process: torch ships libamdhip64 / libhsa-runtime64 with the
    # same SONAMEs as /opt/rocm (libamdhip64.so.7, libhsa-runtime64.so.1).  Importing
    # torch first makes liborbg's DT_NEEDED entries bind to the copies torch loaded, so
    # torch (RCCL, tensors) and liborbg share one runtime and one device context.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    vp, P, i32, f32 = C.c_void_p, C.POINTER, C.c_int, C.c_float
    sz = C.c_size_t
    sig = {
        "orbg_params_default": (None, [P(Params)]),
        "orbg_create": (i32, [i32, P(Params), P(vp)]),
        "orbg_destroy": (None, [vp]),
        "orbg_last_error": (C.c_char_p, []),
        "orbg_abi_version": (i32, []),
        "orbg_get_scale_tables": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, vp]),
        "orbg_get_pattern": (i32, [vp]),
        "orbg_extract": (i32, [vp, vp, i32, i32, sz, vp, vp, i32, P(i32)]),
        "orbg_get_level": (i32, [vp, i32, i32, vp, sz, P(i32), P(i32)]),
        "orbg_get_blurred_level": (i32, [vp, i32, i32, vp, sz, P(i32), P(i32)]),
        "orbg_extract_batch_device": (i32, [vp, vp, i32, i32, i32, sz, sz]),
        "orbg_batch_outputs": (i32, [vp, P(vp), P(vp), P(vp), P(C.c_int32)]),
        "orbg_download_frame": (i32, [vp, i32, vp, vp, i32, P(i32)]),
        "orbg_match_batch_device": (i32, [vp, vp, vp, i32, i32, f32, i32]),
        "orbg_match_outputs": (i32, [vp, P(vp), P(vp), P(vp), P(C.c_int32)]),
        "orbg_download_matches": (i32, [vp, i32, vp, vp, i32, vp]),
        "orbg_sync": (i32, [vp]),
        "orbg_check_errors": (i32, [vp]),
        "orbg_stream": (vp, [vp]),
        "orbg_set_stream": (i32, [vp, vp]),
        "orbg_set_pipeline": (i32, [vp, i32]),
        "orbg_set_serial": (i32, [vp, i32]),
        "orbg_get_pipeline": (i32, [vp]),
        "orbg_batch_summary": (i32, [vp, vp]),
        "orbg_batch_matches": (i32, [vp, vp, vp]),
        "orbg_batch_acquire": (i32, [vp, vp]),
        "orbg_match_pose_batch_device": (i32, [vp, P(PoseCamera), f32, vp, vp, vp]),
        "orbg_batch_release": (i32, [vp, vp]),
        "orbg_stereo_batch_device": (i32, [vp, vp, vp, i32, f32, f32]),
        "orbg_stereo_outputs": (i32, [vp, vp, vp, vp, vp]),
        "orbg_stereo_summary": (i32, [vp, vp]),
        "orbg_stereo_frame": (i32, [vp, vp, vp, i32, i32, C.c_size_t, f32, f32, vp, vp, i32, vp,
                                    vp, vp, i32, vp, vp, vp]),
        "orbg_download_stereo": (i32, [vp, i32, vp, vp, i32, vp]),
        "orbg_match_stream": (vp, [vp]),
        "orbg_batch_stats": (i32, [vp, P(C.c_int64), P(C.c_int64)]),
        "orbg_get_quadtree_caps": (i32, [vp, P(i32), P(i32), P(i32)]),
        "orbg_get_blur_plan": (i32, [vp, P(i32), P(C.c_int64), P(C.c_int64)]),
        "orbg_get_blur_layout": (i32, [vp, P(i32)]),
        "orbg_profile_enable": (i32, [vp, i32]),
        "orbg_profile_read": (i32, [vp, i32, P(C.c_char_p), P(C.c_double), P(C.c_int64)]),
        "orbg_profile_reset": (i32, [vp]),
        "orbg_descriptor_distance": (i32, [vp, vp]),
        "orbg_hamming_knn2": (i32, [vp, vp, i32, vp, i32, vp, vp, vp]),
        "orbg_search_for_initialization": (i32, [vp, vp, vp, i32, vp, vp, i32, P(Bounds), vp, vp,
                                                 i32, f32, i32, P(i32)]),
        "orbg_search_by_projection_lastframe": (i32, [vp, vp, vp, vp, i32, vp, P(Bounds), vp, vp,
                                                      i32, P(TrackCamera), f32, i32, vp, P(i32)]),
        "orbg_search_by_projection_local": (i32, [vp, vp, vp, vp, i32, vp, P(Bounds), vp, vp, i32,
                                                  f32, f32, vp, P(i32)]),
        "orbg_search_by_projection_batch_device": (i32, [vp, i32, P(TrackBatch), i32]),
        "orbg_pose_optimization": (i32, [vp, vp, i32, P(PoseCamera), vp, vp, vp, vp, vp, P(i32)]),
        "orbg_pose_optimization_batch_device": (i32, [vp, vp, vp, i32, vp, vp, vp, vp, vp, vp, vp,
                                                      i32]),
        "orbg_ba_schur_solve": (i32, [vp, vp, i32, i32, vp, i32, vp, vp, vp, vp, vp, C.c_double, vp,
                                      vp, P(i32)]),
        "orbg_vocab_create": (i32, [vp, i32, i32, i32, i32, i32, vp, vp, vp, vp, P(vp)]),
        "orbg_vocab_load_text": (i32, [vp, C.c_char_p, P(vp)]),
        "orbg_vocab_destroy": (None, [vp]),
        "orbg_vocab_info": (i32, [vp, P(i32), P(i32), P(i32), P(i32), P(i32), P(i32)]),
        "orbg_bow_transform": (i32, [vp, vp, vp, i32, i32, vp, vp, P(i32), vp, vp, vp, P(i32)]),
        "orbg_bow_transform_batch_device": (i32, [vp, vp, vp, vp, i32, i32, i32, vp, vp, vp, vp,
                                                  vp, vp, vp, vp, vp]),
        "orbg_search_by_bow": (i32, [vp, vp, vp, vp, i32, vp, vp, vp, i32, vp, vp, i32, vp, vp, vp,
                                     i32, f32, i32, vp, P(i32)]),
        "orbg_search_by_bow_batch_device": (i32, [vp, P(BowFrames), P(BowFrames), i32, vp, vp, i32,
                                                  f32, i32, vp, vp]),
        "orbg_ba_linearize": (i32, [vp, vp, i32, vp, i32, vp, i32, vp, vp, vp, vp, vp]),
        "orbg_ba_set_jacobians": (i32, [vp, i32]),
        "orbg_ba_set_edge_errors": (i32, [vp, i32]),
        "orbg_ba_errors": (i32, [vp, vp, i32, vp, i32, vp, i32, vp, vp, vp, vp, P(C.c_double)]),
        "orbg_ba_errors_device": (i32, [vp, vp, vp, vp, i32, vp, vp, vp, vp]),
        "orbg_ba_linearize_device": (i32, [vp, vp, i32, vp, i32, vp, i32, vp, vp, vp, vp, vp, vp,
                                           vp, vp, vp]),
        "orbg_ba_build_system_device": (i32, [vp, vp, i32, vp, i32, vp, i32, vp, vp, vp, vp, vp,
                                              vp, vp, vp, vp]),
        "orbg_ba_graph_create": (i32, [vp, vp, i32, i32, i32, P(vp)]),
        "orbg_ba_graph_destroy": (i32, [vp]),
        "orbg_ba_graph_set_active": (i32, [vp, vp, vp]),
        "orbg_ba_graph_build_system": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, vp]),
        "orbg_ba_graph_errors": (i32, [vp, vp, vp, vp, vp, vp, vp, vp]),
        "orbg_ba_graph_schur_plan": (i32, [vp, vp, vp]),
        "orbg_ba_graph_schur_solve": (i32, [vp, vp, C.c_double, vp, vp, vp, vp, vp, vp, vp, vp]),
        "orbg_ba_graph_set_robust": (i32, [vp, vp, vp]),
        "orbg_ba_update_device": (i32, [vp, vp, i32, vp, i32, vp, vp, vp, vp]),
        "orbg_ba_graph_optimize": (i32, [vp, vp, vp, vp, i32, P(LmReport)]),
        "orbg_ba_graph_optimize_ctl": (i32, [vp, vp, vp, vp, i32, P(LmControl), P(LmReport)]),
        "orbg_search_for_triangulation": (i32, [vp, P(KeyFrame), P(KeyFrame), vp, i32, i32, vp,
                                                P(i32)]),
        "orbg_search_for_triangulation_batch_device": (i32, [vp, P(KeyFrames), i32, vp, vp, vp,
                                                             i32, i32, i32, vp, vp]),
        "orbg_triangulation_geometry": (i32, [vp, vp, vp, vp]),
        "orbg_triangulation_geometry_batch_device": (i32, [vp, vp, vp, vp, i32, vp]),
        "orbg_triangulate": (i32, [vp, P(KeyFrameGeo), P(KeyFrameGeo), vp, vp, vp, vp, vp,
                                   P(i32)]),
        "orbg_triangulate_batch_device": (i32, [vp, P(KeyFrames), vp, vp, i32, vp, vp, vp, vp,
                                                i32, vp, vp, vp]),
        "orbg_search_by_bow_kf": (i32, [vp, vp, vp, vp, i32, vp, vp, vp, i32, vp, vp, vp, i32, vp, vp,
                                        vp, i32, f32, i32, vp, P(i32)]),
        "orbg_search_by_bow_kf_batch_device": (i32, [vp, P(BowFrames), P(BowFrames), i32, vp, vp,
                                                     i32, f32, i32, vp, vp]),
        "orbg_fuse": (i32, [vp, P(KeyFrame), vp, vp, vp, i32, f32, vp, vp, P(i32)]),
        "orbg_fuse_batch_device": (i32, [vp, P(KeyFrames), i32, vp, vp, vp, vp, vp, i32, i32, f32,
                                         vp, vp, vp]),
        "orbg_search_by_projection_reloc": (i32, [vp, vp, vp, i32, vp, vp, vp, vp, i32, f32, i32,
                                                  i32, vp, P(i32)]),
        "orbg_search_by_projection_sim3": (i32, [vp, vp, vp, i32, vp, vp, vp, vp, i32, i32, vp,
                                                 P(i32)]),
        "orbg_rgbd_stereo": (i32, [vp, vp, i32, f32, i32, i32, C.c_size_t, vp, vp, i32, f32, vp,
                                   vp]),
        "orbg_rgbd_stereo_batch_device": (i32, [vp, vp, i32, f32, i32, i32, C.c_size_t,
                                                C.c_size_t, vp, vp, vp, i32, i32, f32, vp, vp]),
        "orbg_search_by_sim3": (i32, [vp, P(KeyFrame), vp, vp, vp, P(KeyFrame), vp, vp, vp, vp,
                                      f32, vp, P(i32)]),
        "orbg_search_by_sim3_batch_device": (i32, [vp, P(KeyFrames), i32, vp, vp, vp, vp, vp, vp,
                                                   vp, i32, f32, vp, vp]),
        "orbg_fuse_sim3": (i32, [vp, P(KeyFrame), vp, vp, vp, i32, f32, vp, vp, P(i32)]),
        "orbg_fuse_sim3_batch_device": (i32, [vp, P(KeyFrames), i32, vp, vp, vp, vp, vp, i32, i32, f32,
                                         vp, vp, vp]),
        "orbg_undistort_keypoints": (i32, [vp, vp, vp, i32, vp]),
        "orbg_undistort_batch_device": (i32, [vp, vp, vp, vp, i32, i32, vp]),
        "orbg_compute_image_bounds": (i32, [vp, i32, i32, P(Bounds)]),
        "orbg_set_camera": (i32, [vp, vp]),
        "orbg_batch_keys_un": (i32, [vp, P(vp), P(C.c_int32)]),
        "orbg_is_in_frustum": (i32, [vp, vp, vp, i32, f32, vp, P(i32)]),
        "orbg_is_in_frustum_batch_device": (i32, [vp, vp, vp, vp, i32, i32, f32, vp, vp]),
        "orbg_distinctive_descriptor": (i32, [vp, vp, i32, P(C.c_int32)]),
        "orbg_distinctive_descriptors_batch_device": (i32, [vp, vp, vp, vp, i32, vp, vp]),
    }
    for name, (res, args) in sig.items():
        if os.environ.get("ORBG_LIB_VARIANT") and not hasattr(L, name):
            continue  # developer A/B of an older build: entry points it predates stay unbound
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def last_error():
    if _lib is None:
        return ""
    m = _lib.orbg_last_error()
    return m.decode() if m else ""


def check(rc, what):
    if rc != ORBG_OK:
        raise OrbgError(rc, what)
    return rc


def ptr(a):
    """data pointer of a numpy array (or None)."""
    if a is None:
        return None
    return C.c_void_p(a.ctypes.data)


def default_params(**kw):
    p = Params()
    lib().orbg_params_default(C.byref(p))
    for k, v in kw.items():
        if k == "gauss_k":
            for i in range(7):
                p.gauss_k[i] = int(v[i])
        else:
            setattr(p, k, v)
    return p


class Context:
    """Owns one orbg_ctx (device buffers + one HIP stream)."""

    def __init__(self, device=0, params=None):
        self._L = lib()
        self.params = params if params is not None else default_params()
        h = C.c_void_p()
        check(self._L.orbg_create(int(device), C.byref(self.params), C.byref(h)), "orbg_create")
        self.handle = h
        self.device = device

    def close(self):
        if getattr(self, "handle", None):
            self._L.orbg_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # profiling (HIP events on the context stream)
    def profile(self, enable=True):
        check(self._L.orbg_profile_enable(self.handle, 1 if enable else 0), "profile_enable")

    def profile_reset(self):
        check(self._L.orbg_profile_reset(self.handle), "profile_reset")

    def profile_read(self):
        n = self._L.orbg_profile_read(self.handle, -1, None, None, None)
        out = {}
        for i in range(n):
            name, ms, cnt = C.c_char_p(), C.c_double(), C.c_int64()
            self._L.orbg_profile_read(self.handle, i, C.byref(name), C.byref(ms), C.byref(cnt))
            out[name.value.decode()] = (ms.value, cnt.value)
        return out

    def sync(self):
        """Drain the context's streams; raises OrbgError(ORBG_ENOTSUP) if a batch since the
        last check overflowed a quadtree capacity (sticky device flag)."""
        check(self._L.orbg_sync(self.handle), "orbg_sync")

    def check_errors(self):
        """Same check as sync(): read and clear the sticky device error flag."""
        check(self._L.orbg_check_errors(self.handle), "orbg_check_errors")

    def set_stream(self, stream_ptr):
        """Launch on a caller-owned hipStream_t (int pointer) or the own stream (None)."""
        check(self._L.orbg_set_stream(self.handle, C.c_void_p(stream_ptr) if stream_ptr else None),
              "orbg_set_stream")

    def set_pipeline(self, enable=True):
        """Pipelined batches: the image half of batch k+1 beside the keypoint half of batch k
        (orbg_set_pipeline; the batch's input images must stay unchanged until its outputs
        are complete)."""
        check(self._L.orbg_set_pipeline(self.handle, 1 if enable else 0), "orbg_set_pipeline")

    def set_serial(self, enable=True):
        """Every extraction kernel on the context stream, one after the other
        (orbg_set_serial): per-kernel event times without overlap."""
        check(self._L.orbg_set_serial(self.handle, 1 if enable else 0), "orbg_set_serial")

    def pipelined(self):
        return bool(self._L.orbg_get_pipeline(self.handle))

    def batch_stats(self):
        a, b = C.c_int64(), C.c_int64()
        check(self._L.orbg_batch_stats(self.handle, C.byref(a), C.byref(b)), "orbg_batch_stats")
        return a.value, b.value

    def quadtree_caps(self):
        """(first_cap, level0_cap, upper_cap) of the planned image size
        (orbg_get_quadtree_caps): the k_octree_lds candidate caps; past them, k_octree."""
        a, b, c = C.c_int32(), C.c_int32(), C.c_int32()
        check(self._L.orbg_get_quadtree_caps(self.handle, C.byref(a), C.byref(b), C.byref(c)),
              "orbg_get_quadtree_caps")
        return a.value, b.value, c.value

    def blur_plan(self):
        """(fused, interior px per frame, border px per frame) of the planned image size
        (orbg_get_blur_plan)."""
        a, b, c = C.c_int32(), C.c_int64(), C.c_int64()
        check(self._L.orbg_get_blur_plan(self.handle, C.byref(a), C.byref(b), C.byref(c)),
              "orbg_get_blur_plan")
        return bool(a.value), b.value, c.value

    def blur_tiled(self):
        """True when the blurred levels are stored as 16 x 8-px tiles (orbg_get_blur_layout)."""
        a = C.c_int32()
        check(self._L.orbg_get_blur_layout(self.handle, C.byref(a)), "orbg_get_blur_layout")
        return bool(a.value)

    def stereo_summary(self, d_out_ptr):
        check(self._L.orbg_stereo_summary(self.handle, C.c_void_p(d_out_ptr)),
              "orbg_stereo_summary")

    def match_stream(self):
        """hipStream_t (int) of batch matching and the summary."""
        return self._L.orbg_match_stream(self.handle)

    def batch_matches(self, d_out_ptr=None):
        """vnMatches12 of every pair of the last match batch into a device buffer of
        npairs x frame_cap int32 (orbg_batch_matches); returns frame_cap."""
        fc = C.c_int32()
        check(self._L.orbg_batch_matches(self.handle, C.c_void_p(d_out_ptr) if d_out_ptr else None,
                                         C.byref(fc)), "orbg_batch_matches")
        return fc.value

    def batch_acquire(self, stream_ptr=None):
        """Make `stream` (None: the match stream) wait until the last batch's device
        outputs (and stereo outputs) are written (orbg_batch_acquire)."""
        check(self._L.orbg_batch_acquire(self.handle, C.c_void_p(stream_ptr) if stream_ptr else None),
              "orbg_batch_acquire")

    def batch_release(self, stream_ptr=None):
        """Reads of those outputs enqueued on `stream` so far finish before liborbg
        overwrites them (orbg_batch_release)."""
        check(self._L.orbg_batch_release(self.handle, C.c_void_p(stream_ptr) if stream_ptr else None),
              "orbg_batch_release")

    def batch_summary(self, d_out_ptr):
        check(self._L.orbg_batch_summary(self.handle, C.c_void_p(d_out_ptr)), "orbg_batch_summary")
