#!/usr/bin/env python3
"""Tracking-matcher throughput: ORBmatcher::SearchByProjection over a batch of frames.

Workload: a synthetic 1241x376 pan sequence of B+1 frames extracted on the GPU (2000
features, 8 levels).  Frame t (t = 1..B) is CurrentFrame; frame t-1's keypoints become
    - last-frame mode: LastFrame map points back-projected at depth 10 m, camera moved by the
      sequence's pan (Tracking::TrackWithMotionModel, mono, th = 15, checkOri);
    - local mode: local-map projections (Frame::isInFrustum outputs) moved by the pan plus
      +-0.7 px (Tracking::SearchLocalPoints, th = 1, nnratio 0.8).
Everything HBM-resident; one step = orbg_search_by_projection_batch_device over B frames.
Prints one JSON line per mode with frames/s, kernel times (HIP events) and the oracle's
single-thread frames/s on a bounded sample.

    python tools/track_bench.py [--batch 256] [--steps 20] [--warmup 3] [--no-cpu]
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

W, H = 1241, 376


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-frames", type=int, default=256)
    args = ap.parse_args()

    import torch
    from orb_slam2_test_amd import ORBextractor, synthetic as S
    from orb_slam2_test_amd import _lib as L

    B = args.batch
    seed = S.DEFAULT_SEED + 5
    seq = S.sequence(B + 1, H, W, seed=seed)
    pos = S.sequence_positions(B + 1, seed=seed)
    ext = ORBextractor(2000, 1.2, 8, 20, 7, max_batch=B + 1)
    d_img = torch.from_numpy(seq).cuda()
    ext.extract_batch_device(d_img.data_ptr(), B + 1, W, H)
    d_kps, d_desc, d_cnt, fc = ext.batch_outputs()
    ext.ctx.sync()
    frames = [ext.download_frame(t) for t in range(B + 1)]

    fx, fy, cx, cy, bf = S.KITTI_FX, S.KITTI_FY, S.KITTI_CX, S.KITTI_CY, S.KITTI_BF
    lf = np.zeros((B, fc), L.LF_DTYPE)
    mp = np.zeros((B, fc), L.MP_DTYPE)
    cams = (L.TrackCamera * B)()
    shifts = []
    for t in range(1, B + 1):
        sh = (float(-(pos[t, 1] - pos[t - 1, 1])), float(-(pos[t, 0] - pos[t - 1, 0])))
        shifts.append(sh)
        kl = frames[t - 1][0]
        pts, Tcw, Tlw = S.tracking_scene(kl, sh, seed=seed + t)
        lf[t - 1, :len(pts)] = pts
        mp[t - 1, :len(kl)] = S.map_projections(kl, sh, seed=seed + t)
        cams[t - 1] = L.track_camera(Tcw, Tlw, fx, fy, cx, cy, bf, bf / fx, True)
    dev = "cuda"
    d_lf = torch.from_numpy(lf.view(np.uint8).reshape(-1)).to(dev)
    d_mp = torch.from_numpy(mp.view(np.uint8).reshape(-1)).to(dev)
    d_cams = torch.from_numpy(np.frombuffer(bytes(cams), np.uint8).copy()).to(dev)
    d_bounds = torch.from_numpy(np.tile(np.array([0, W, 0, H], np.float32), B)).to(dev)
    d_match = torch.empty(B * fc, dtype=torch.int32, device=dev)
    d_nm = torch.empty(B, dtype=torch.int32, device=dev)
    kp_bytes = L.KP_DTYPE.itemsize

    def batch(mode):
        tb = L.TrackBatch()
        tb.kps = d_kps + fc * kp_bytes          # CurrentFrame = frames 1..B
        tb.desc = d_desc + fc * 32
        tb.uright = None
        tb.taken0 = None
        tb.counts = d_cnt + 4
        tb.bounds = d_bounds.data_ptr()
        tb.frame_cap = fc
        tb.queries = (d_lf if mode == L.TRACK_LASTFRAME else d_mp).data_ptr()
        tb.qdesc = d_desc                       # frame t-1's descriptors
        tb.qcounts = d_cnt
        tb.query_cap = fc
        tb.cams = d_cams.data_ptr()
        tb.th = 15.0 if mode == L.TRACK_LASTFRAME else 1.0
        tb.nnratio = 0.8
        tb.check_ori = 1
        tb.match = d_match.data_ptr()
        tb.nmatches = d_nm.data_ptr()
        return tb

    lines = []
    for mode, name in ((L.TRACK_LASTFRAME, "lastframe"), (L.TRACK_LOCAL, "local")):
        tb = batch(mode)
        run = lambda: L.check(L.lib().orbg_search_by_projection_batch_device(  # noqa: E731
            ext.ctx.handle, mode, C.byref(tb), B), "track batch")
        for _ in range(args.warmup):
            run()
        ext.ctx.sync()
        ext.ctx.profile(True)
        ext.ctx.profile_reset()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            run()
        ext.ctx.sync()
        dt = time.perf_counter() - t0
        kern = ext.ctx.profile_read()
        ext.ctx.profile(False)
        nm = d_nm.cpu().numpy()
        out = {
            "metric": "tracking frames/s, SearchByProjection (%s), 1241x376 2000 feat" % name,
            "value": round(B * args.steps / dt, 1), "unit": "frames/s", "higher_is_better": True,
            "dtype": "u8/f32", "data": "synthetic",
            "config": {"workload": "B=%d frames, %s" % (B, "mono motion model th 15 checkOri"
                                                         if mode == L.TRACK_LASTFRAME else
                                                         "local map th 1 nnratio 0.8"),
                       "queries_per_frame": round(float(np.mean([len(f[0]) for f in frames])), 1),
                       "mean_nmatches": round(float(nm.mean()), 1)},
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "kernels": {k: {"ms_per_step": round(v[0] / args.steps, 4),
                            "avg_launch_ms": round(v[0] / max(v[1], 1), 5)}
                        for k, v in kern.items() if k.startswith("track")},
        }
        if not args.no_cpu:
            from oracle import pyoracle as O
            p = O.params(nfeatures=2000)
            sfo = np.array([p.scale[l] for l in range(8)], np.float32)
            n = min(args.cpu_frames, B)
            t0 = time.perf_counter()
            for t in range(1, n + 1):
                kc, dc = frames[t]
                kl, dl = frames[t - 1]
                if mode == L.TRACK_LASTFRAME:
                    cam = O.track_cam(np.frombuffer(bytes(cams[t - 1].Tcw), np.float32),
                                      np.frombuffer(bytes(cams[t - 1].Tlw), np.float32),
                                      fx, fy, cx, cy, bf, bf / fx, True)
                    O.search_by_projection_lastframe(kc, dc, None, None, (0, W, 0, H), sfo,
                                                     lf[t - 1, :len(kl)], dl, cam, 15.0, True)
                else:
                    O.search_by_projection_local(kc, dc, None, None, (0, W, 0, H), sfo,
                                                 mp[t - 1, :len(kl)], dl, 1.0, 0.8)
            cdt = time.perf_counter() - t0
            out["cpu_baseline"] = {"value": round(n / cdt, 1), "unit": "frames/s", "cores": 1,
                                   "kind": "port", "sample": "%d frames, oracle/ C restatement "
                                   "-O3, one thread, %.2f s" % (n, cdt)}
        lines.append(out)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
