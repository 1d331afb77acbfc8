#!/usr/bin/env python3
"""Throughput of the Frame / MapPoint geometry kernels (csrc/frame_kernels.hip), one JSON line
per kernel, each with its HIP-event time per launch, algorithmic bytes against HBM, and the
CPU oracle (oracle/frame_oracle.c) on one host core over a bounded sample:

  undistort    Frame::UndistortKeyPoints (Frame.cc:542-572) with TUM1's distortion over
               B = 1024 frames x 2000 keypoints resident in HBM: keypoints/s.
               Algorithmic bytes: the 28-byte keypoint in and out (56 B per keypoint).
  rgbd         Frame::ComputeStereoFromRGBD (Frame.cc:837-858) over B = 256 TUM frames x 1000
               keypoints with raw uint16 depth images in HBM: keypoints/s (66 B per keypoint:
               two keypoint records, the depth pixel, mvuRight / mvDepth out).
  frustum      Frame::isInFrustum (Frame.cc:342-409) for Tracking::SearchLocalPoints over
               B = 256 frames x 8192 local map points: map points/s.  36-byte MapPoint
               record in, 24-byte projection out (60 B per point).
  distinctive  MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:342-420) over 262144 map
               points with 2..30 observations (mean 16) gathered from a pool of KeyFrame
               descriptors: map points/s.  Per point: its observations' descriptor rows and
               row indices (36 B each), the offsets, BestIdx and the 32-byte descriptor out.

    python tools/frame_geom_bench.py [--steps 20] [--warmup 3] [--no-cpu] [--only NAME]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

HBM_PEAK_GBS = 8000.0
TUM1 = (517.306408, 516.469215, 318.643040, 255.313989, 0.262383, -0.953104, -0.005358,
        0.002628, 1.163314)


def timed(ctx, name, run, steps, warmup):
    for _ in range(warmup):
        run()
    ctx.sync()
    ctx.profile(True)
    ctx.profile_reset()
    t0 = time.perf_counter()
    for _ in range(steps):
        run()
    ctx.sync()
    dt = time.perf_counter() - t0
    kern = ctx.profile_read()
    ctx.profile(False)
    tot, n = kern.get(name, (0.0, 1))
    return dt / steps, tot / max(n, 1)


def line(metric, unit, units, ms_step, avg_ms, algo, workload, extra=None):
    ach = algo / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else None
    r = {"metric": metric, "value": round(units / (ms_step), 1), "unit": unit,
         "higher_is_better": True, "data": "synthetic", "config": {"workload": workload},
         "ms_per_step": round(ms_step * 1e3, 4),
         "roofline": {"bound": "hbm", "achieved": round(ach, 1) if ach else None,
                      "peak": HBM_PEAK_GBS, "unit": "GB/s",
                      "frac": round(ach / HBM_PEAK_GBS, 4) if ach else None,
                      "algo_bytes_per_launch": int(algo), "avg_launch_ms": round(avg_ms, 5)}}
    if extra:
        r.update(extra)
    return r


def cpu_rate(fn, units_per_call, budget=2.0):
    t0 = time.perf_counter()
    calls = 0
    while time.perf_counter() - t0 < budget:
        fn()
        calls += 1
    dt = time.perf_counter() - t0
    return units_per_call * calls / dt, calls, dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--only", default="")
    args = ap.parse_args()

    import torch
    from orb_slam2_test_amd import _lib as L
    from orb_slam2_test_amd import frame as FR
    from orb_slam2_test_amd import mappoint as MP
    import test_oracle_frame as T

    ctx = FR._default_ctx()
    h = ctx.handle
    O = None
    if not args.no_cpu:
        from oracle import pyoracle as O
    rng = np.random.default_rng(20261017)

    if args.only in ("", "undistort"):
        B, cap, n = 1024, 2048, 2000
        kps = np.zeros((B, cap), L.KP_DTYPE)
        kps["x"] = rng.uniform(0, 640, (B, cap))
        kps["y"] = rng.uniform(0, 480, (B, cap))
        kps["octave"] = rng.integers(0, 8, (B, cap))
        counts = np.full(B, n, np.int32)
        dk = torch.from_numpy(kps.view(np.uint8).reshape(B, -1).copy()).cuda()
        dc = torch.from_numpy(counts).cuda()
        dout = torch.empty_like(dk)
        cam = FR.camera(*TUM1)

        def run():
            L.check(L.lib().orbg_undistort_batch_device(h, L.ptr(cam), dk.data_ptr(), dc.data_ptr(),
                                                        cap, B, dout.data_ptr()), "undistort")
        ms, avg = timed(ctx, "undistort", run, args.steps, args.warmup)
        r = line("Frame::UndistortKeyPoints keypoints/s (TUM1 distortion)", "keypoints/s", B * n,
                 ms, avg, B * n * 56, "B=%d frames x %d keypoints, TUM1 k1..k3, 5 iterations "
                 "(double)" % (B, n), {"dtype": "f64"})
        if O is not None:
            ocam = O.camera(*TUM1)
            sample = kps[0, :n].view(O.KP_DTYPE)
            v, calls, dt = cpu_rate(lambda: O.undistort_keypoints(ocam, sample), n)
            r["cpu_baseline"] = {"value": round(v, 1), "unit": "keypoints/s", "cores": 1,
                                 "kind": "port", "sample": "%d x %d keypoints, oracle -O3, one "
                                 "thread, %.2f s" % (calls, n, dt)}
        print(json.dumps(r), flush=True)

    if args.only in ("", "rgbd"):
        B, cap, n, w, hh = 256, 1024, 1000, 640, 480
        imgs = np.zeros((B, hh, w), np.uint16)
        kps = np.zeros((B, cap), L.KP_DTYPE)
        kun = np.zeros((B, cap), L.KP_DTYPE)
        cases = [T.rgbd_case(L, 70 + q, "u16", n=n) for q in range(16)]
        for b in range(B):
            d, k, ku = cases[b % 16]
            imgs[b], kps[b, :n], kun[b, :n] = d, k, ku
        counts = np.full(B, n, np.int32)
        t = {k: torch.from_numpy(np.ascontiguousarray(v).view(np.uint8).reshape(-1).copy()).cuda()
             for k, v in dict(imgs=imgs, kps=kps, kun=kun, cnt=counts).items()}
        ur = torch.empty(B * cap, dtype=torch.float32, device="cuda")
        dd = torch.empty(B * cap, dtype=torch.float32, device="cuda")
        fac = float(T.TUM_DEPTH_FACTOR)

        def run():
            L.check(L.lib().orbg_rgbd_stereo_batch_device(
                h, t["imgs"].data_ptr(), L.DEPTH_U16, fac, w, hh, w * 2, w * 2 * hh,
                t["kps"].data_ptr(), t["kun"].data_ptr(), t["cnt"].data_ptr(), cap, B,
                T.TUM_MBF, ur.data_ptr(), dd.data_ptr()), "rgbd")
        ms, avg = timed(ctx, "rgbd", run, args.steps, args.warmup)
        # per keypoint: mvKeys / mvKeysUn records (56 B), the depth pixel (2 B), two floats out
        r = line("Frame::ComputeStereoFromRGBD keypoints/s (TUM1 RGB-D, raw uint16 depth)",
                 "keypoints/s", B * n, ms, avg, B * n * 66,
                 "B=%d frames 640x480 x %d keypoints, DepthMapFactor 5000" % (B, n),
                 {"dtype": "f32"})
        if O is not None:
            d0, k0, ku0 = cases[0]
            v, calls, dt = cpu_rate(lambda: O.rgbd_stereo(d0, fac, k0, ku0, T.TUM_MBF), n)
            r["cpu_baseline"] = {"value": round(v, 1), "unit": "keypoints/s", "cores": 1,
                                 "kind": "port", "sample": "%d x %d keypoints, oracle -O3, one "
                                 "thread, %.2f s" % (calls, n, dt)}
        print(json.dumps(r), flush=True)

    if args.only in ("", "frustum"):
        B, cap = 256, 8192
        cams = np.zeros(B, L.FRUSTUM_DTYPE)
        mps = np.zeros((B, cap), L.MAPPOINT_DTYPE)
        for f in range(B):
            _, _, cams[f], mps[f] = T.frustum_case(L, cap, 1000 + f)
        counts = np.full(B, cap, np.int32)
        d_c = torch.from_numpy(cams.view(np.uint8).copy()).cuda()
        d_m = torch.from_numpy(mps.view(np.uint8).reshape(-1).copy()).cuda()
        d_n = torch.from_numpy(counts).cuda()
        d_p = torch.zeros(B * cap * L.MP_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
        d_v = torch.zeros(B, dtype=torch.int32, device="cuda")

        def run():
            L.check(L.lib().orbg_is_in_frustum_batch_device(h, d_c.data_ptr(), d_m.data_ptr(),
                                                            d_n.data_ptr(), cap, B, 0.5,
                                                            d_p.data_ptr(), d_v.data_ptr()),
                    "frustum")
        ms, avg = timed(ctx, "frustum", run, args.steps, args.warmup)
        nv = float(d_v.cpu().numpy().mean())
        r = line("Frame::isInFrustum map points/s (SearchLocalPoints)", "points/s", B * cap, ms,
                 avg, B * cap * 60, "B=%d frames x %d local map points, viewingCosLimit 0.5"
                 % (B, cap), {"dtype": "f32/f64", "visible_per_frame": round(nv, 1)})
        if O is not None:
            fc0 = cams[0:1].view(O.FRUSTUM_DTYPE)[0]
            m0 = mps[0].view(O.MAPPOINT_DTYPE)
            v, calls, dt = cpu_rate(lambda: O.is_in_frustum(fc0, m0, 0.5), cap)
            r["cpu_baseline"] = {"value": round(v, 1), "unit": "points/s", "cores": 1,
                                 "kind": "port", "sample": "%d x %d points, oracle -O3, one "
                                 "thread, %.2f s" % (calls, cap, dt)}
        print(json.dumps(r), flush=True)

    if args.only in ("", "distinctive"):
        npool, npts = 1 << 20, 1 << 18
        pool = rng.integers(0, 256, (npool, 32), dtype=np.uint8)
        counts = rng.integers(2, 31, npts)
        off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)
        base = rng.integers(0, npool, npts)
        rows = ((np.repeat(base, counts) + rng.integers(0, 4096, off[-1])) % npool).astype(np.int32)
        d_pool = torch.from_numpy(pool).cuda()
        d_rows = torch.from_numpy(rows).cuda()
        d_off = torch.from_numpy(off).cuda()
        d_best = torch.empty(npts, dtype=torch.int32, device="cuda")
        d_desc = torch.empty((npts, 32), dtype=torch.uint8, device="cuda")

        def run():
            MP.distinctive_descriptors_device(ctx, d_pool.data_ptr(), d_rows.data_ptr(),
                                              d_off.data_ptr(), npts, d_best.data_ptr(),
                                              d_desc.data_ptr())
        ms, avg = timed(ctx, "distinctive", run, args.steps, args.warmup)
        nobs = int(off[-1])
        algo = nobs * 36 + (npts + 1) * 4 + npts * 36
        r = line("MapPoint::ComputeDistinctiveDescriptors map points/s", "points/s", npts, ms,
                 avg, algo, "%d map points, 2..30 observations (mean %.1f) from a pool of %d "
                 "KeyFrame descriptors" % (npts, nobs / npts, npool), {"dtype": "u8"})
        if O is not None:
            ns = 4096
            so = off[:ns + 1]
            v, calls, dt = cpu_rate(lambda: O.distinctive_descriptors(pool, rows[:so[-1]], so), ns)
            r["cpu_baseline"] = {"value": round(v, 1), "unit": "points/s", "cores": 1,
                                 "kind": "port", "sample": "%d x %d map points, oracle -O3, one "
                                 "thread, %.2f s" % (calls, ns, dt)}
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
