#!/usr/bin/env python3
"""PoseOptimization throughput: Optimizer::PoseOptimization over a batch of frames.

Workload: B synthetic KITTI-like tracking frames (synthetic.pose_frame: 2000 map-point
observations, 50% stereo, 10% gross outliers, perturbed motion-model pose), HBM-resident;
one step = orbg_pose_optimization_batch_device over the B frames (one workgroup per frame:
4 rounds x <= 10 LM iterations, fp64).  Prints one JSON line with frames/s, the kernel time
(HIP events) and the oracle's single-thread frames/s on a bounded sample.

    python tools/pose_bench.py [--batch 1024] [--edges 2000] [--steps 10] [--no-cpu]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--edges", type=int, default=2000)
    ap.add_argument("--distinct", type=int, default=16)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-frames", type=int, default=64)
    args = ap.parse_args()

    import torch
    from orb_slam2_test_amd import synthetic as S
    from orb_slam2_test_amd import _lib as L
    from orb_slam2_test_amd.orbmatcher import _ctx

    B, cap = args.batch, args.edges
    cam = (S.KITTI_FX, S.KITTI_FY, S.KITTI_CX, S.KITTI_CY, S.KITTI_BF)
    base = [S.pose_frame(n=cap, seed=100 + i) for i in range(args.distinct)]
    e = np.zeros((B, cap), L.PEDGE_DTYPE)
    tin = np.zeros((B, 12), np.float32)
    cams = (L.PoseCamera * B)()
    for i in range(B):
        ed, Tt, T0 = base[i % args.distinct]
        e[i] = ed
        tin[i] = T0.reshape(12)
        cams[i] = L.PoseCamera(*[float(np.float32(v)) for v in cam], 0.0)
    dev = "cuda"
    d_e = torch.from_numpy(e.view(np.uint8).reshape(-1)).to(dev)
    d_cnt = torch.full((B,), cap, dtype=torch.int32, device=dev)
    d_cam = torch.from_numpy(np.frombuffer(bytes(cams), np.uint8).copy()).to(dev)
    d_tin = torch.from_numpy(tin).to(dev)
    d_q = torch.zeros(B * 4, dtype=torch.float64, device=dev)
    d_t = torch.zeros(B * 3, dtype=torch.float64, device=dev)
    d_to = torch.zeros(B * 12, dtype=torch.float32, device=dev)
    d_out = torch.zeros(B * cap, dtype=torch.uint8, device=dev)
    d_ni = torch.zeros(B, dtype=torch.int32, device=dev)
    ctx = _ctx(0)

    def run():
        L.check(L.lib().orbg_pose_optimization_batch_device(
            ctx.handle, d_e.data_ptr(), d_cnt.data_ptr(), cap, d_cam.data_ptr(),
            d_tin.data_ptr(), d_q.data_ptr(), d_t.data_ptr(), d_to.data_ptr(),
            d_out.data_ptr(), d_ni.data_ptr(), B), "pose batch")

    torch.cuda.synchronize()
    for _ in range(args.warmup):
        run()
    ctx.sync()
    ctx.profile(True)
    ctx.profile_reset()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run()
    ctx.sync()
    dt = time.perf_counter() - t0
    kern = ctx.profile_read()
    ctx.profile(False)
    ni = d_ni.cpu().numpy()
    out = {
        "metric": "PoseOptimization frames/s (4 x optimize(10), %d edges/frame)" % cap,
        "value": round(B * args.steps / dt, 1), "unit": "frames/s", "higher_is_better": True,
        "dtype": "f64", "data": "synthetic",
        "config": {"workload": "B=%d KITTI-like tracking frames, %d edges, 50%% stereo, 10%% "
                               "outliers" % (B, cap), "mean_inliers": round(float(ni.mean()), 1)},
        "ms_per_step": round(dt / args.steps * 1e3, 4),
        "kernels": {k: {"ms_per_step": round(v[0] / args.steps, 4),
                        "avg_launch_ms": round(v[0] / max(v[1], 1), 5)} for k, v in kern.items()},
    }
    if not args.no_cpu:
        from oracle import pyoracle as O
        n = min(args.cpu_frames, B)
        t0 = time.perf_counter()
        for i in range(n):
            ed, Tt, T0 = base[i % args.distinct]
            O.pose_optimization(ed, cam, T0)
        cdt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(n / cdt, 1), "unit": "frames/s", "cores": 1,
                               "kind": "port", "sample": "%d frames, oracle/ C restatement -O3, "
                               "one thread, %.2f s" % (n, cdt)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
