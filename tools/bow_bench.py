#!/usr/bin/env python3
"""DBoW2 transform throughput (Frame::ComputeBoW): frames/s over a batch of frames.

Workload: B synthetic 1241x376 frames extracted on the GPU (2000 features, 8 levels); an
ORBvoc.txt-shaped vocabulary (k = 10, L = 6, 1,111,111 nodes, TF_IDF + L1; synthetic since
ORBvoc.txt is not in the reference checkout) resident in HBM.  One step =
orbg_bow_transform_batch_device over the B frames, levelsup 4.  Prints one JSON line with
frames/s, per-kernel times (HIP events), the descent kernel's algorithmic bytes / time and
the oracle's single-thread frames/s on a bounded sample.

    python tools/bow_bench.py [--batch 256] [--steps 20] [--warmup 3] [--no-cpu]
"""
import argparse
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
    ap.add_argument("--cpu-frames", type=int, default=32)
    args = ap.parse_args()

    import torch
    from orb_slam2_test_amd import ORBextractor, ORBVocabulary, synthetic as S

    B = args.batch
    seq = S.sequence(B, H, W, seed=S.DEFAULT_SEED + 41)
    ext = ORBextractor(2000, 1.2, 8, 20, 7, max_batch=B)
    d_img = torch.from_numpy(seq).cuda()
    ext.extract_batch_device(d_img.data_ptr(), B, W, H)
    d_kps, d_desc, d_cnt, fc = ext.batch_outputs()
    ext.ctx.sync()
    voc = S.vocabulary(10, 6, seed=S.DEFAULT_SEED + 2)
    t0 = time.perf_counter()
    gv = ORBVocabulary.from_tree(voc["k"], voc["L"], voc["scoring"], voc["weighting"],
                                 voc["parent"], voc["is_leaf"], voc["desc"], voc["weight"])
    upload_s = time.perf_counter() - t0
    dev = "cuda"
    out = {k: torch.empty(B * fc, dtype=torch.int32, device=dev)
           for k in ("bow_words", "fv_nodes", "fv_feats")}
    out["bow_weights"] = torch.empty(B * fc, dtype=torch.float64, device=dev)
    out["fv_off"] = torch.empty(B * (fc + 1), dtype=torch.int32, device=dev)
    out["nbow"] = torch.empty(B, dtype=torch.int32, device=dev)
    out["nfv"] = torch.empty(B, dtype=torch.int32, device=dev)
    ptrs = {k: v.data_ptr() for k, v in out.items()}

    def run():
        gv.transform_batch_device(d_desc, d_cnt, fc, B, 4, ptrs, ext.ctx)

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
    nfeat = int(np.sum([ext.download_frame(t)[0].shape[0] for t in range(B)]))
    nb = out["nbow"].cpu().numpy()
    # descent: per feature the 32-byte descriptor + L levels x k 64-byte slot records +
    # 16 bytes of outputs (word, node, weight)
    desc_bytes = nfeat * (32 + voc["L"] * voc["k"] * 64 + 16)
    kw = kern.get("bow_words", (0.0, 1))
    avg_ms = kw[0] / max(kw[1], 1)
    res = {
        "metric": "BoW transform frames/s (Frame::ComputeBoW), 1241x376 2000 feat, k10 L6 vocab",
        "value": round(B * args.steps / dt, 1), "unit": "frames/s", "higher_is_better": True,
        "dtype": "u8/f64", "data": "synthetic",
        "config": {"workload": "B=%d frames, levelsup 4, TF_IDF + L1" % B,
                   "features_per_frame": round(nfeat / B, 1),
                   "words_per_frame": round(float(nb.mean()), 1),
                   "vocab_nodes": len(voc["parent"]), "vocab_upload_s": round(upload_s, 3)},
        "ms_per_step": round(dt / args.steps * 1e3, 4),
        "kernels": {k: {"ms_per_step": round(v[0] / args.steps, 4),
                        "avg_launch_ms": round(v[0] / max(v[1], 1), 5)}
                    for k, v in kern.items() if k.startswith("bow")},
        "descent_gbs": round(desc_bytes / (avg_ms * 1e-3) / 1e9, 1) if avg_ms > 0 else None,
    }
    if not args.no_cpu:
        from oracle import pyoracle as O
        ov = O.Vocab(voc["k"], voc["L"], voc["scoring"], voc["weighting"], voc["parent"],
                     voc["is_leaf"], voc["desc"], voc["weight"])
        n = min(args.cpu_frames, B)
        frames = [ext.download_frame(t)[1] for t in range(n)]
        t0 = time.perf_counter()
        for d in frames:
            O.bow_transform(ov, d, 4)
        cdt = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": round(n / cdt, 1), "unit": "frames/s", "cores": 1,
                               "kind": "port", "sample": "%d frames, oracle/ C restatement -O3, "
                               "one thread, %.2f s" % (n, cdt)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
