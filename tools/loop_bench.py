#!/usr/bin/env python3
"""Throughput of the relocalization and loop-closing projection matchers on the device
(csrc/track_kernels.hip, TRK_RELOC / TRK_LOOP), one JSON line each, with HIP-event kernel
times, algorithmic bytes against HBM and the CPU oracle (oracle/loop_oracle.c) on one host
core over a bounded sample:

  reloc  ORBmatcher::SearchByProjection(CurrentFrame, pKF, sAlreadyFound, 10, 100)
         (Tracking::Relocalization): 256 (CurrentFrame of 2000 keypoints, candidate KeyFrame
         of 1500 map points) pairs per launch, checkOri: frames/s.
  loop   ORBmatcher::SearchByProjection(pKF, Scw, vpPoints, vpMatched, 10)
         (LoopClosing::ComputeSim3): 256 (KeyFrame of 2000 keypoints, 1500 loop map points)
         pairs per launch: keyframes/s.
  sim3   ORBmatcher::SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, 7.5)
         (LoopClosing::ComputeSim3): 256 pairs of 2000-keypoint KeyFrames: pairs/s.

Algorithmic bytes per pair: per keypoint its KP record, descriptor, written flag and output
slot (28 + 32 + 1 + 4 B); per query its record and descriptor (reloc 28 + 32 B, loop 36 + 32 B).
The synthetic cases are tests/test_oracle_loop.py's (32 distinct, each used 8 times).

    python tools/loop_bench.py [--steps 20] [--warmup 3] [--no-cpu] [--only reloc|loop|sim3]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    import torch
    from orb_slam2_test_amd import _lib as L
    from orb_slam2_test_amd.orbmatcher import _ctx
    import test_oracle_loop as T
    ctx = _ctx()
    NQ, REP, N, NP = 32, 8, 2000, 1500
    B = NQ * REP
    for mode in ("reloc", "loop"):
        if args.only not in ("", mode):
            continue
        projection_line(args, L, T, ctx, mode, NQ, REP, N, NP, B)
    if args.only in ("", "sim3"):
        sim3_line(args, L, T, ctx, NQ, REP, N)


def sim3_line(args, L, T, ctx, NQ, REP, N):
    import torch
    M = 1300
    P = NQ * REP
    cases = [T.sim3_case(L, 980 + q, n=N, m=M, s12=0.95 + 0.005 * q) for q in range(NQ)]
    nk = 2 * NQ
    kps = np.zeros((nk, N), L.KP_DTYPE)
    desc = np.zeros((nk, N, 32), np.uint8)
    mps = np.zeros((nk, N), L.MAPPOINT_DTYPE)
    md = np.zeros((nk, N, 32), np.uint8)
    am1 = np.zeros((P, N), np.uint8)
    am2 = np.zeros((P, N), np.uint8)
    pairs = np.zeros(P, L.SIM3_PAIR_DTYPE)
    for q, (kf1, mp1, md1, a1, kf2, mp2, md2, a2, g, perm) in enumerate(cases):
        kps[2 * q], desc[2 * q], mps[2 * q], md[2 * q] = kf1["kps"], kf1["desc"], mp1, md1
        kps[2 * q + 1], desc[2 * q + 1], mps[2 * q + 1], md[2 * q + 1] = kf2["kps"], kf2["desc"], mp2, md2
    qi = np.arange(P) % NQ
    for p in range(P):
        c = cases[qi[p]]
        am1[p], am2[p], pairs[p] = c[3], c[7], c[8]
    cnt = np.full(nk, N, np.int32)
    t = {k: torch.from_numpy(np.ascontiguousarray(v).view(np.uint8).reshape(-1).copy()).cuda()
         for k, v in dict(kps=kps, desc=desc, cnt=cnt, mps=mps, md=md, am1=am1, am2=am2,
                          pairs=pairs).items()}
    K = L.KeyFrames(t["desc"].data_ptr(), t["kps"].data_ptr(), None, None, t["cnt"].data_ptr(),
                    None, None, None, None)
    i1 = torch.from_numpy((2 * qi).astype(np.int32)).cuda()
    i2 = torch.from_numpy((2 * qi + 1).astype(np.int32)).cuda()
    out = torch.empty(P * N, dtype=torch.int32, device="cuda")
    nf = torch.empty(P, dtype=torch.int32, device="cuda")

    def run():
        L.check(L.lib().orbg_search_by_sim3_batch_device(
            ctx.handle, C.byref(K), N, i1.data_ptr(), i2.data_ptr(), t["pairs"].data_ptr(),
            t["mps"].data_ptr(), t["md"].data_ptr(), t["am1"].data_ptr(), t["am2"].data_ptr(), P,
            7.5, out.data_ptr(), nf.data_ptr()), "sim3")
    for _ in range(args.warmup):
        run()
    ctx.sync()
    ctx.profile(True)
    ctx.profile_reset()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run()
    ctx.sync()
    dt = (time.perf_counter() - t0) / args.steps
    kern = ctx.profile_read()
    ctx.profile(False)
    tot, cnt_ = kern.get("sim3_match", (0.0, 1))
    avg = tot / max(cnt_, 1)
    # per pair: both KeyFrames' keypoints, descriptors, map point records and descriptors,
    # already-matched flags (129 B per slot), vnMatch1 / vnMatch2 and matches12 (12 B)
    algo = P * N * (2 * 129 + 12)
    ach = algo / (avg * 1e-3) / 1e9
    r = {"metric": "ORBmatcher::SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th) "
                   "KeyFrame pairs/s (LoopClosing::ComputeSim3)",
         "value": round(P / dt, 1), "unit": "pairs/s", "higher_is_better": True,
         "data": "synthetic", "dtype": "u8/f32",
         "config": {"workload": "%d pairs of %d-keypoint KeyFrames with a map point per slot "
                                "(88%% valid), %d common points, s12 0.95-1.1, th 7.5" % (P, N, M),
                    "mean_found": round(float(nf.cpu().numpy().mean()), 1)},
         "ms_per_step": round(dt * 1e3, 4),
         "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                      "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                      "algo_bytes_per_launch": int(algo), "avg_launch_ms": round(avg, 5),
                      "kernel": "k_sim3_match + k_sim3_resolve"}}
    if not args.no_cpu:
        from oracle import pyoracle as O
        sf = T._sf(O)
        t0 = time.perf_counter()
        calls = 0
        while time.perf_counter() - t0 < 3.0:
            kf1, mp1, md1, a1, kf2, mp2, md2, a2, g, perm = cases[calls % NQ]
            O.search_by_sim3(kf1, mp1.view(O.MAPPOINT_DTYPE), md1, a1, kf2,
                             mp2.view(O.MAPPOINT_DTYPE), md2, a2, g.view(O.SIM3_PAIR_DTYPE), 7.5, sf)
            calls += 1
        cdt = time.perf_counter() - t0
        r["cpu_baseline"] = {"value": round(calls / cdt, 1), "unit": "pairs/s", "cores": 1,
                             "kind": "port", "sample": "%d pairs, oracle -O3, one thread, "
                             "%.2f s" % (calls, cdt)}
    print(json.dumps(r), flush=True)


def projection_line(args, L, T, ctx, mode, NQ, REP, N, NP, B):
    import torch
    if mode == "reloc":
        cases = [T.reloc_case(L, 900 + q, n=N, npts=NP) for q in range(NQ)]
        qdt = L.RELOC_DTYPE
    else:
        cases = [T.sim3proj_case(L, 950 + q, n=N, nm=NP, scale=0.6 + 0.05 * q)
                 for q in range(NQ)]
        qdt = L.MAPPOINT_DTYPE
    kps = np.zeros((B, N), L.KP_DTYPE)
    desc = np.zeros((B, N, 32), np.uint8)
    tk = np.zeros((B, N), np.uint8)
    q = np.zeros((B, NP), qdt)
    qd = np.zeros((B, NP, 32), np.uint8)
    bounds = np.zeros((B, 4), np.float32)
    fcams = np.zeros(B, L.FRUSTUM_DTYPE)
    for b in range(B):
        f, fcam, pts, pd = cases[b % NQ]
        kps[b], desc[b], tk[b], q[b], qd[b] = f["kps"], f["desc"], f["taken0"], pts, pd
        bounds[b] = [fcam["min_x"], fcam["max_x"], fcam["min_y"], fcam["max_y"]]
        fcams[b] = fcam
    cnt = np.full(B, N, np.int32)
    qcnt = np.full(B, NP, np.int32)
    t = {k: torch.from_numpy(np.ascontiguousarray(v).view(np.uint8).reshape(-1).copy()).cuda()
         for k, v in dict(kps=kps, desc=desc, tk=tk, q=q, qd=qd, cnt=cnt, qcnt=qcnt,
                          bounds=bounds, fcams=fcams).items()}
    match = torch.empty(B * N, dtype=torch.int32, device="cuda")
    nm = torch.empty(B, dtype=torch.int32, device="cuda")
    tb = L.TrackBatch()
    tb.kps, tb.desc, tb.uright, tb.taken0 = t["kps"].data_ptr(), t["desc"].data_ptr(), None, t["tk"].data_ptr()
    tb.counts, tb.bounds, tb.frame_cap = t["cnt"].data_ptr(), t["bounds"].data_ptr(), N
    tb.queries, tb.qdesc = t["q"].data_ptr(), t["qd"].data_ptr()
    tb.qcounts, tb.query_cap = t["qcnt"].data_ptr(), NP
    tb.cams, tb.th, tb.nnratio, tb.check_ori = None, 10.0, 0.0, 1
    tb.match, tb.nmatches = match.data_ptr(), nm.data_ptr()
    tb.fcams, tb.orb_dist = t["fcams"].data_ptr(), 100
    md = L.TRACK_RELOC if mode == "reloc" else L.TRACK_LOOP

    def run():
        L.check(L.lib().orbg_search_by_projection_batch_device(ctx.handle, md, C.byref(tb),
                                                               B), mode)
    for _ in range(args.warmup):
        run()
    ctx.sync()
    ctx.profile(True)
    ctx.profile_reset()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run()
    ctx.sync()
    dt = (time.perf_counter() - t0) / args.steps
    kern = ctx.profile_read()
    ctx.profile(False)
    kt = {k: v[0] / max(v[1], 1) for k, v in kern.items() if k.startswith("track")}
    both = sum(kt.values())
    algo = B * (N * (28 + 32 + 1 + 4) + NP * (qdt.itemsize + 32))
    ach = algo / (both * 1e-3) / 1e9
    if mode == "reloc":
        title = ("ORBmatcher::SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist) "
                 "frames/s (Tracking::Relocalization)")
        wl = "%d (CurrentFrame of %d keypoints, candidate KeyFrame of %d map points), th 10, ORBdist 100, checkOri" % (B, N, NP)
    else:
        title = ("ORBmatcher::SearchByProjection(pKF, Scw, vpPoints, vpMatched, th) keyframes/s "
                 "(LoopClosing::ComputeSim3)")
        wl = "%d (KeyFrame of %d keypoints, %d loop map points, Sim3 scale 0.6-2.15), th 10" % (B, N, NP)
    r = {"metric": title, "value": round(B / dt, 1), "unit": "frames/s" if mode == "reloc" else "keyframes/s",
         "higher_is_better": True, "data": "synthetic", "dtype": "u8/f32",
         "config": {"workload": wl, "mean_nmatches": round(float(nm.cpu().numpy().mean()), 1)},
         "ms_per_step": round(dt * 1e3, 4),
         "kernels": {k: round(v, 5) for k, v in kt.items()},
         "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                      "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                      "algo_bytes_per_launch": int(algo),
                      "avg_launch_ms": round(both, 5), "kernel": "track_cands + track_resolve"}}
    if not args.no_cpu:
        from oracle import pyoracle as O
        sf = T._sf(O)
        t0 = time.perf_counter()
        calls = 0
        while time.perf_counter() - t0 < 3.0:
            f, fcam, pts, pd = cases[calls % NQ]
            if mode == "reloc":
                O.search_by_projection_reloc(f["kps"], f["desc"], f["taken0"],
                                             fcam.view(O.FRUSTUM_DTYPE), sf,
                                             pts.view(O.RELOC_DTYPE), pd, 10, 100, True)
            else:
                O.search_by_projection_sim3(f["kps"], f["desc"], f["taken0"],
                                            fcam.view(O.FRUSTUM_DTYPE), sf,
                                            pts.view(O.MAPPOINT_DTYPE), pd, 10)
            calls += 1
        cdt = time.perf_counter() - t0
        r["cpu_baseline"] = {"value": round(calls / cdt, 1), "unit": r["unit"], "cores": 1,
                             "kind": "port", "sample": "%d pairs, oracle -O3, one thread, "
                             "%.2f s" % (calls, cdt)}
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
