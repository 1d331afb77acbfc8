#!/usr/bin/env python3
"""ORBmatcher::SearchByBoW(KeyFrame*, Frame&) throughput (Tracking::TrackReferenceKeyFrame,
Tracking.cc:1069): frame/KeyFrame pairs per second over a batch.

Workload: B + 1 synthetic 1241x376 frames extracted on the GPU (2000 features, 8 levels),
DBoW2 transform over an ORBvoc.txt-shaped synthetic vocabulary (k = 10, L = 6, levelsup 4,
ComputeBoW's), resident in HBM.  One step = orbg_search_by_bow_batch_device over the B pairs
(KeyFrame = frame t - 1 with 90% of its features carrying a good MapPoint, Frame = frame t),
nnratio 0.7 and checkOri (TrackReferenceKeyFrame's ORBmatcher(0.7, true)).  Prints one JSON
line: pairs/s, the kernel's HIP-event time and algorithmic bytes (both frames' descriptors,
keypoints and FeatureVectors + the match row) against HBM, and the oracle on one host core.

    python tools/bow_match_bench.py [--batch 1024] [--steps 20] [--warmup 3] [--no-cpu]
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
HBM_PEAK_GBS = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-pairs", type=int, default=64)
    args = ap.parse_args()

    import torch
    from orb_slam2_test_amd import ORBextractor, ORBVocabulary, synthetic as S
    from orb_slam2_test_amd import _lib as L

    B = args.batch
    nf = B + 1
    seq = S.sequence(nf, H, W, seed=S.DEFAULT_SEED + 43)
    ext = ORBextractor(2000, 1.2, 8, 20, 7, max_batch=nf)
    d_img = torch.from_numpy(seq).cuda()
    ext.extract_batch_device(d_img.data_ptr(), nf, W, H)
    d_kps, d_desc, d_cnt, fc = ext.batch_outputs()
    ext.ctx.sync()
    voc = S.vocabulary(10, 6, seed=S.DEFAULT_SEED + 2)
    gv = ORBVocabulary.from_tree(voc["k"], voc["L"], voc["scoring"], voc["weighting"],
                                 voc["parent"], voc["is_leaf"], voc["desc"], voc["weight"])
    dev = "cuda"
    out = {k: torch.empty(nf * fc, dtype=torch.int32, device=dev)
           for k in ("bow_words", "fv_nodes", "fv_feats")}
    out["bow_weights"] = torch.empty(nf * fc, dtype=torch.float64, device=dev)
    out["fv_off"] = torch.empty(nf * (fc + 1), dtype=torch.int32, device=dev)
    out["nbow"] = torch.empty(nf, dtype=torch.int32, device=dev)
    out["nfv"] = torch.empty(nf, dtype=torch.int32, device=dev)
    gv.transform_batch_device(d_desc, d_cnt, fc, nf, 4, {k: v.data_ptr() for k, v in out.items()},
                              ext.ctx)
    rng = np.random.default_rng(7)
    valid = torch.from_numpy((rng.random(nf * fc) < 0.9).astype(np.uint8)).to(dev)
    kf_i = torch.arange(0, B, dtype=torch.int32, device=dev)
    f_i = torch.arange(1, B + 1, dtype=torch.int32, device=dev)
    match = torch.empty(B * fc, dtype=torch.int32, device=dev)
    nmatch = torch.empty(B, dtype=torch.int32, device=dev)
    ext.ctx.sync()
    torch.cuda.synchronize()
    side = dict(desc=d_desc, kps=d_kps, counts=d_cnt, fv_nodes=out["fv_nodes"].data_ptr(),
                fv_off=out["fv_off"].data_ptr(), fv_feats=out["fv_feats"].data_ptr(),
                nfv=out["nfv"].data_ptr())
    K = L.BowFrames(valid=valid.data_ptr(), **side)
    F = L.BowFrames(valid=None, **side)
    h = ext.ctx.handle

    def run():
        L.check(L.lib().orbg_search_by_bow_batch_device(
            h, C.byref(K), C.byref(F), fc, C.c_void_p(kf_i.data_ptr()),
            C.c_void_p(f_i.data_ptr()), B, 0.7, 1, C.c_void_p(match.data_ptr()),
            C.c_void_p(nmatch.data_ptr())), "orbg_search_by_bow_batch_device")

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
    cnt = np.array([ext.download_frame(t)[0].shape[0] for t in range(nf)])
    nm = nmatch.cpu().numpy()
    # per pair: both frames' descriptors (32 B), keypoint angle (28-B records), FeatureVector
    # (node + offset + feature index, 12 B per feature), the KF valid flags and the match row
    kpf = float(cnt.mean())
    algo = B * (2 * kpf * (32 + 28 + 12) + kpf + kpf * 4)
    km = kern.get("bow_match", (0.0, 1))
    avg_ms = km[0] / max(km[1], 1)
    ach = algo / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else None
    res = {
        "metric": "SearchByBoW(KF, F) pairs/s (TrackReferenceKeyFrame), 1241x376 2000 feat, "
                  "k10 L6 vocab, levelsup 4",
        "value": round(B * args.steps / dt, 1), "unit": "pairs/s", "higher_is_better": True,
        "dtype": "u8", "data": "synthetic",
        "config": {"workload": "B=%d pairs (KF = frame t-1, F = frame t), nnratio 0.7, checkOri, "
                               "90%% of KF features with a good MapPoint" % B,
                   "features_per_frame": round(kpf, 1),
                   "nodes_per_frame": round(float(out["nfv"].cpu().numpy().mean()), 1),
                   "matches_per_pair": round(float(nm.mean()), 1)},
        "ms_per_step": round(dt / args.steps * 1e3, 4),
        "kernels": {k: {"ms_per_step": round(v[0] / args.steps, 4),
                        "avg_launch_ms": round(v[0] / max(v[1], 1), 5)}
                    for k, v in kern.items() if k == "bow_match"},
        "roofline": {"kernel": "bow_match", "bound": "hbm", "achieved": round(ach, 1) if ach else None,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(ach / HBM_PEAK_GBS, 4) if ach else None,
                     "algo_bytes_per_launch": int(algo), "avg_launch_ms": round(avg_ms, 5)},
    }
    if not args.no_cpu:
        from oracle import pyoracle as O
        n = min(args.cpu_pairs, B)
        hv = valid.cpu().numpy().reshape(nf, fc)
        hfv = {k: out[k].cpu().numpy() for k in ("fv_nodes", "fv_off", "fv_feats", "nfv")}
        frames = [ext.download_frame(t) for t in range(n + 1)]

        def fv(f):
            k = hfv["nfv"][f]
            vo = hfv["fv_off"][f * (fc + 1):f * (fc + 1) + k + 1]
            return hfv["fv_nodes"][f * fc:f * fc + k], vo, hfv["fv_feats"][f * fc:f * fc + vo[-1]]

        args_l = [(frames[t][1], frames[t][0]["angle"], hv[t, :len(frames[t][0])], fv(t),
                   frames[t + 1][1], frames[t + 1][0]["angle"], fv(t + 1)) for t in range(n)]
        # the n pairs repeated for about 3 s of CPU work (one pair takes ~0.25 ms)
        t0 = time.perf_counter()
        reps = 0
        while time.perf_counter() - t0 < 3.0:
            for a in args_l:
                O.search_by_bow(*a, nnratio=0.7, check_ori=True)
            reps += 1
        cdt = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": round(n * reps / cdt, 1), "unit": "pairs/s", "cores": 1,
                               "kind": "port", "sample": "%d pairs x %d passes, oracle/ C "
                               "restatement -O3, one thread, %.2f s" % (n, reps, cdt)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
