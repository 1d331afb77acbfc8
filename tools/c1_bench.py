#!/usr/bin/env python3
"""configs[0] (C1): TUM1 mono_tum shape, 640x480, 1000 features, 8 levels.  BASELINE.json
names it "reference CPU path, no GPU": the reference times one TrackMonocular call per frame
(Examples/Monocular/mono_tum.cc:85, 119-120).  This prints, for the per-frame hot path
(ORBextractor::operator() + ORBmatcher::SearchForInitialization(window 100, 0.9, checkOri)
against the previous frame, plus the all-pairs knn2):

  - the CPU restatement (oracle/, the C port; the reference itself needs OpenCV / Eigen and
    is not buildable here) on one host thread (the reference's model) and on N threads;
  - liborbg on one MI355X, batched (B frames resident in HBM per step, as bench.py) and
    for the record the host-in / host-out single-frame path is tools/single_frame_bench.py.

usage: c1_bench.py [cpu_threads] [gpu_steps]  -> one JSON line
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
W, H, NF, NL = 640, 480, 1000, 8


def main():
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    from orb_slam2_test_amd import synthetic as S
    from oracle import pyoracle as O
    sys.path.insert(0, os.path.join(ROOT))
    import bench  # host_cpu()

    B = 256
    frames = S.sequence_block(B, 0, B, H, W)  # B + 1 frames: the halo frame first
    p = O.params(nfeatures=NF, nlevels=NL)

    def cpu(n, th):
        idx = np.arange(n) % len(frames)
        sample = np.ascontiguousarray(frames[idx])
        t0 = time.perf_counter()
        O.frames_batch(p, sample, nthreads=th, window=100, nnratio=0.9)
        return n / (time.perf_counter() - t0)

    cpu1 = cpu(48, 1)
    cpun = cpu(64 * threads, threads)
    ncpu, model = bench.host_cpu()
    out = {"metric": "frames/sec ORB extract+match, configs[0] TUM1 640x480 1000feat 8lvl",
           "config": {"workload": "C1 TUM1-shaped mono 640x480, 1000 feat, 8 lvl: ORBextractor "
                                  "+ Hamming knn2 (t vs t-1) + SearchForInitialization(w=100, "
                                  "0.9, checkOri)", "data": "synthetic"},
           "cpu_port_1thread_frames_per_s": round(cpu1, 2),
           "cpu_port_threads": threads, "cpu_port_nthreads_frames_per_s": round(cpun, 2),
           "host_logical_cpus": ncpu, "host_cpu_model": model}
    try:
        import torch
        gpu = torch.cuda.is_available()
    except ImportError:
        gpu = False
    if gpu:
        from orb_slam2_test_amd import ORBextractor
        d = torch.from_numpy(frames).cuda()
        ext = ORBextractor(NF, 1.2, NL, 20, 7, max_batch=len(frames))
        st = torch.cuda.Stream()
        torch.cuda.set_stream(st)
        ext.ctx.set_stream(st.cuda_stream)
        ext.ctx.set_pipeline(True)
        f1 = np.arange(B, dtype=np.int32)
        f2 = np.arange(1, B + 1, dtype=np.int32)

        def step():
            ext.extract_batch_device(d.data_ptr(), len(frames), W, H)
            ext.match_batch_device(f1, f2, 100, 0.9, True)
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        ext.ctx.check_errors()
        out["gpu_frames_per_s"] = round(B * steps / dt, 1)
        out["gpu_ms_per_256_frames"] = round(dt / steps * 1e3, 4)
        # the same with TUM1.yaml's distortion (k1..k3, p1, p2): the matching reads mvKeysUn
        # (Frame::UndistortKeyPoints on the device, Frame.cc:259) inside ComputeImageBounds'
        # bounds, as the reference's TUM1 run does
        from orb_slam2_test_amd import frame as FR
        ext.set_camera(FR.camera(517.306408, 516.469215, 318.643040, 255.313989, 0.262383,
                                 -0.953104, -0.005358, 0.002628, 1.163314))
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        ext.ctx.check_errors()
        out["gpu_tum1_distorted_frames_per_s"] = round(B * steps / dt, 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
