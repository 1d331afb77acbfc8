"""ORBextractor -- drop-in mirror of ORB_SLAM2::ORBextractor over liborbg (HIP, gfx950).

Reference interface: include/ORBextractor.h:55-135, src/ORBextractor.cc:432-1443.

    ext = ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST)
    keypoints, descriptors = ext(image, mask)      # operator()(image, mask, kps, desc)
    ext.GetLevels(); ext.GetScaleFactor(); ext.GetScaleFactors(); ...
    ext.mvImagePyramid[level]                      # public std::vector<cv::Mat>

keypoints is a numpy structured array with cv::KeyPoint's fields (x, y, size, angle,
response, octave, class_id); descriptors is an (N, 32) uint8 array.  As in the
reference, an empty image returns immediately (here: ``(None, None)``: outputs
untouched), the mask is ignored, and zero keypoints give an empty descriptor matrix.

``extract_batch_device`` runs the same kernels on a batch of device-resident frames
(the batched-sequence mode); results stay in HBM.
"""
import ctypes as C

import numpy as np

from . import _lib as L


class ORBextractor:
    HARRIS_SCORE = 0
    FAST_SCORE = 1

    def __init__(self, nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST, device=0,
                 max_batch=1, resize_mode=L.RESIZE_SIMD_16_8, gauss_k=None, brief_fma=0,
                 sincos_mode=L.SINCOS_GLIBC):
        kw = dict(nfeatures=int(nfeatures), scale_factor=float(scaleFactor),
                  nlevels=int(nlevels), ini_th_fast=int(iniThFAST), min_th_fast=int(minThFAST),
                  resize_mode=int(resize_mode), brief_fma=int(brief_fma),
                  max_batch=int(max_batch), sincos_mode=int(sincos_mode))
        if gauss_k is not None:
            kw["gauss_k"] = gauss_k
        self.ctx = L.Context(device, L.default_params(**kw))
        self._tables()
        self._pyr_cache = None
        self._frame_cap = 0

    def _tables(self):
        nl = C.c_int32()
        sf = C.c_float()
        arrs = [np.zeros(L.MAX_LEVELS, np.float32) for _ in range(4)]
        fpl = np.zeros(L.MAX_LEVELS, np.int32)
        umax = np.zeros(16, np.int32)
        L.check(L.lib().orbg_get_scale_tables(self.ctx.handle, C.byref(nl), C.byref(sf),
                                              *[L.ptr(a) for a in arrs], L.ptr(fpl),
                                              L.ptr(umax)), "orbg_get_scale_tables")
        self.nlevels = nl.value
        self.scaleFactor = sf.value
        k = self.nlevels
        self.mvScaleFactor, self.mvInvScaleFactor, self.mvLevelSigma2, self.mvInvLevelSigma2 = \
            [a[:k].copy() for a in arrs]
        self.mnFeaturesPerLevel = fpl[:k].copy()
        self.umax = umax.copy()

    # --- getters, ORBextractor.h:78-98 ---
    def GetLevels(self):
        return self.nlevels

    def GetScaleFactor(self):
        return float(np.float32(self.scaleFactor))

    def GetScaleFactors(self):
        return list(self.mvScaleFactor)

    def GetInverseScaleFactors(self):
        return list(self.mvInvScaleFactor)

    def GetScaleSigmaSquares(self):
        return list(self.mvLevelSigma2)

    def GetInverseScaleSigmaSquares(self):
        return list(self.mvInvLevelSigma2)

    # --- operator(), ORBextractor.cc:1330-1397 ---
    def __call__(self, image, mask=None):
        if image is None or getattr(image, "size", 0) == 0:
            return None, None  # _image.empty(): return, outputs untouched
        img = np.asarray(image)
        if img.dtype != np.uint8 or img.ndim != 2:
            raise ValueError("ORBextractor expects a CV_8UC1 image (2-D uint8)")
        img = np.ascontiguousarray(img)
        h, w = img.shape
        cap = self.ctx.params.nfeatures + 16 * (self.nlevels + 4) + 64
        while True:
            kps = np.zeros(cap, L.KP_DTYPE)
            desc = np.zeros((cap, 32), np.uint8)
            n = C.c_int()
            rc = L.lib().orbg_extract(self.ctx.handle, L.ptr(img), w, h, img.strides[0],
                                      L.ptr(kps), L.ptr(desc), cap, C.byref(n))
            if rc == L.ORBG_ERANGE:
                cap = n.value
                continue
            L.check(rc, "orbg_extract")
            break
        self._pyr_cache = None
        n = n.value
        return kps[:n].copy(), desc[:n].copy()

    @property
    def mvImagePyramid(self):
        """Host copies of the pyramid levels of the last extracted frame (frame 0)."""
        if self._pyr_cache is None:
            self._pyr_cache = [self.get_level(0, l) for l in range(self.nlevels)]
        return self._pyr_cache

    def get_level(self, frame, level):
        return self._level("orbg_get_level", frame, level)

    def get_blurred_level(self, frame, level):
        """The GaussianBlur of pyramid level `level` (the image rBRIEF samples,
        ORBextractor.cc:1375-1377); a parity accessor (orbg_get_blurred_level)."""
        return self._level("orbg_get_blurred_level", frame, level)

    def _level(self, fn, frame, level):
        lw, lh = C.c_int(), C.c_int()
        f = getattr(L.lib(), fn)
        L.check(f(self.ctx.handle, frame, level, None, 0, C.byref(lw), C.byref(lh)), fn)
        out = np.zeros((lh.value, lw.value), np.uint8)
        L.check(f(self.ctx.handle, frame, level, L.ptr(out), lw.value, C.byref(lw),
                  C.byref(lh)), fn)
        return out

    # --- batched, device-resident ---
    def extract_batch_device(self, d_ptr, nframes, w, h, step=None, frame_stride=None):
        step = w if step is None else step
        frame_stride = step * h if frame_stride is None else frame_stride
        L.check(L.lib().orbg_extract_batch_device(self.ctx.handle, C.c_void_p(d_ptr), nframes,
                                                  w, h, step, frame_stride),
                "orbg_extract_batch_device")
        self._pyr_cache = None

    def batch_outputs(self):
        k, d, c, fc = C.c_void_p(), C.c_void_p(), C.c_void_p(), C.c_int32()
        L.check(L.lib().orbg_batch_outputs(self.ctx.handle, C.byref(k), C.byref(d), C.byref(c),
                                           C.byref(fc)), "orbg_batch_outputs")
        return k.value, d.value, c.value, fc.value

    def download_frame(self, frame):
        n = C.c_int()
        rc = L.lib().orbg_download_frame(self.ctx.handle, frame, None, None, 0, C.byref(n))
        if rc not in (L.ORBG_OK, L.ORBG_ERANGE):
            L.check(rc, "orbg_download_frame")
        kps = np.zeros(max(n.value, 1), L.KP_DTYPE)
        desc = np.zeros((max(n.value, 1), 32), np.uint8)
        L.check(L.lib().orbg_download_frame(self.ctx.handle, frame, L.ptr(kps), L.ptr(desc),
                                            n.value, C.byref(n)), "orbg_download_frame")
        return kps[:n.value].copy(), desc[:n.value].copy()

    def set_camera(self, cam):
        """Distorted camera of the batched-sequence mode (orbg_set_camera): the batch
        matching then reads mvKeysUn (Frame::UndistortKeyPoints on the device) with
        ComputeImageBounds' bounds.  cam: frame.camera(...) record, or None for the default
        (mvKeysUn = mvKeys, bounds = image)."""
        c = None if cam is None else np.ascontiguousarray(cam, L.CAMERA_DTYPE)
        L.check(L.lib().orbg_set_camera(self.ctx.handle, L.ptr(c)), "orbg_set_camera")

    def batch_keys_un(self):
        """device pointer of the last match batch's mvKeysUn ([frames][frame_cap]) and
        frame_cap (the keypoints themselves without a distorted camera)."""
        k, fc = C.c_void_p(), C.c_int32()
        L.check(L.lib().orbg_batch_keys_un(self.ctx.handle, C.byref(k), C.byref(fc)),
                "orbg_batch_keys_un")
        return k.value, fc.value

    def match_batch_device(self, f1, f2, window=100, nnratio=0.9, check_ori=True):
        a = np.ascontiguousarray(f1, np.int32)
        b = np.ascontiguousarray(f2, np.int32)
        L.check(L.lib().orbg_match_batch_device(self.ctx.handle, L.ptr(a), L.ptr(b), len(a),
                                                int(window), float(nnratio),
                                                1 if check_ori else 0),
                "orbg_match_batch_device")

    def match_pose_batch_device(self, cam, depth, d_q, d_t, d_ninliers):
        """PoseOptimization of frame f2[p] over the last match batch's matches (F1 keypoints
        back-projected at `depth`; orbg_match_pose_batch_device), on the match stream.
        cam = (fx, fy, cx, cy, bf); d_q [P][4] / d_t [P][3] float64, d_ninliers [P] int32
        device pointers."""
        c = L.PoseCamera(*[float(v) for v in cam], 0.0)
        L.check(L.lib().orbg_match_pose_batch_device(self.ctx.handle, C.byref(c), float(depth),
                                                     C.c_void_p(d_q), C.c_void_p(d_t),
                                                     C.c_void_p(d_ninliers)),
                "orbg_match_pose_batch_device")

    def match_outputs(self):
        k, m, n, fc = C.c_void_p(), C.c_void_p(), C.c_void_p(), C.c_int32()
        L.check(L.lib().orbg_match_outputs(self.ctx.handle, C.byref(k), C.byref(m), C.byref(n),
                                           C.byref(fc)), "orbg_match_outputs")
        return k.value, m.value, n.value, fc.value

    def download_matches(self, pair, n):
        knn = np.zeros((max(n, 1), 3), np.int32)
        m12 = np.zeros(max(n, 1), np.int32)
        nm = np.zeros(1, np.int32)
        L.check(L.lib().orbg_download_matches(self.ctx.handle, pair, L.ptr(knn), L.ptr(m12), n,
                                              L.ptr(nm)), "orbg_download_matches")
        return knn[:n], m12[:n], int(nm[0])

    # --- Frame::ComputeStereoMatches on frame pairs of the last batch (Frame.cc:619-834) ---
    def stereo_batch_device(self, left, right, bf, min_z):
        """Enqueue ComputeStereoMatches for (left[i], right[i]) frames of the last batch.
        min_z is Frame::mb (the reference reads it uninitialised; pass bf / fx)."""
        a = np.ascontiguousarray(left, np.int32)
        b = np.ascontiguousarray(right, np.int32)
        L.check(L.lib().orbg_stereo_batch_device(self.ctx.handle, L.ptr(a), L.ptr(b), len(a),
                                                 float(bf), float(min_z)),
                "orbg_stereo_batch_device")

    def download_stereo(self, pair, n):
        """(mvuRight[n], mvDepth[n], number of depths) of stereo pair `pair`."""
        ur = np.zeros(max(n, 1), np.float32)
        dp = np.zeros(max(n, 1), np.float32)
        nv = np.zeros(1, np.int32)
        L.check(L.lib().orbg_download_stereo(self.ctx.handle, pair, L.ptr(ur), L.ptr(dp), n,
                                             L.ptr(nv)), "orbg_download_stereo")
        return ur[:n], dp[:n], int(nv[0])

    def close(self):
        self.ctx.close()
