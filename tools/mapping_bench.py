#!/usr/bin/env python3
"""Throughput of LocalMapping's matchers on the device (csrc/mapping_kernels.hip), one JSON
line per kernel with its HIP-event time per launch, algorithmic bytes against HBM and the CPU
oracle (oracle/mapping_oracle.c) on one host core over a bounded sample:

  tri_match  ORBmatcher::SearchForTriangulation (LocalMapping::CreateNewMapPoints): 1024
             KeyFrame pairs (64 generated pairs of 2000-feature KITTI KeyFrames, 120-node
             FeatureVectors, 60% stereo, 25% with a MapPoint, each pair 16 times) per launch:
             pairs/s.  Algorithmic bytes per pair: both KeyFrames' descriptors, keypoints,
             mvuRight, MapPoint flags and FeatureVector entries (69 B per feature) plus the
             vMatches12 row (4 B per KF1 feature).
  fuse       ORBmatcher::Fuse(pKF, vpMapPoints, th = 3)'s search (SearchInNeighbors): 256
             (KeyFrame, 2000 MapPoints) pairs per launch: map points/s.  Bytes: per KeyFrame
             the keypoints, descriptors and mvuRight (64 B per keypoint); per MapPoint its
             record and descriptor (68 B) and bestIdx / bestDist (8 B).
  fuse_sim3  ORBmatcher::Fuse(pKF, Scw, vpPoints, th = 4, vpReplacePoint)'s search
             (LoopClosing::SearchAndFuse): the same shape with one Sim3 per KeyFrame (no
             mvuRight: 60 B per keypoint).
  triangulate  LocalMapping::CreateNewMapPoints' triangulation (csrc/triangulate_kernels.hip):
             1024 KeyFrame pairs (64 generated pairs of 2000-feature KeyFrames, 60% stereo,
             8% wrong matches, 10% unmatched; each 16 times) per launch: matched pairs/s.
             Bytes per pKF1 feature: its mvKeysUn + mvKeys + mvuRight + mvDepth (64 B), the
             vMatches12 entry (4 B), the partner's same 64 B, status + x3D (13 B) = 145 B.
             Per-thread ALU (a 4x4 Jacobi in double, glibc atan2f / cosf), so latency- and
             ALU-bound: the HBM fraction is low by construction.

    python tools/mapping_bench.py [--steps 20] [--warmup 3] [--no-cpu] [--only NAME]
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


def line(metric, unit, units, s_step, avg_ms, algo, workload, extra):
    ach = algo / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else None
    r = {"metric": metric, "value": round(units / s_step, 1), "unit": unit,
         "higher_is_better": True, "data": "synthetic", "config": {"workload": workload},
         "ms_per_step": round(s_step * 1e3, 4),
         "roofline": {"bound": "hbm", "achieved": round(ach, 1) if ach else None,
                      "peak": HBM_PEAK_GBS, "unit": "GB/s",
                      "frac": round(ach / HBM_PEAK_GBS, 4) if ach else None,
                      "algo_bytes_per_launch": int(algo), "avg_launch_ms": round(avg_ms, 5)}}
    r.update(extra)
    return r


def dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy()).cuda()


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
    import test_oracle_mapping as T
    O = None
    if not args.no_cpu:
        from oracle import pyoracle as O
    ctx = _ctx()
    h = ctx.handle

    if args.only in ("", "tri_match"):
        NQ, REP, cap = 64, 16, 2048
        cases = [T.tri_case(L.KP_DTYPE, L.TRI_GEOM_DTYPE, 500 + q, n=2000) for q in range(NQ)]
        nk = 2 * NQ
        desc = np.zeros((nk, cap, 32), np.uint8)
        kps = np.zeros((nk, cap), L.KP_DTYPE)
        ur = np.zeros((nk, cap), np.float32)
        mp = np.zeros((nk, cap), np.uint8)
        cnt = np.zeros(nk, np.int32)
        nodes = np.zeros((nk, cap), np.int32)
        off = np.zeros((nk, cap + 1), np.int32)
        feats = np.zeros((nk, cap), np.int32)
        nfv = np.zeros(nk, np.int32)
        for q, (k1, k2, g, _, _) in enumerate(cases):
            for s, kf in ((2 * q, k1), (2 * q + 1, k2)):
                n = len(kf["kps"])
                desc[s, :n], kps[s, :n], ur[s, :n], mp[s, :n], cnt[s] = (
                    kf["desc"], kf["kps"], kf["uright"], kf["has_mp"], n)
                fn, fo, ff = kf["fv"]
                nodes[s, :len(fn)], off[s, :len(fo)], feats[s, :len(ff)], nfv[s] = fn, fo, ff, len(fn)
        t = {k: dev(v) for k, v in dict(desc=desc, kps=kps, ur=ur, mp=mp, cnt=cnt, nodes=nodes,
                                        off=off, feats=feats, nfv=nfv).items()}
        K = L.KeyFrames(*(t[k].data_ptr() for k in ("desc", "kps", "ur", "mp", "cnt", "nodes",
                                                      "off", "feats", "nfv")))
        P = NQ * REP
        q = np.arange(P) % NQ
        i1 = torch.from_numpy((2 * q).astype(np.int32)).cuda()
        i2 = torch.from_numpy((2 * q + 1).astype(np.int32)).cuda()
        G = np.array([cases[j][2] for j in q], L.TRI_GEOM_DTYPE)
        dg = dev(G)
        dm = torch.empty(P * cap, dtype=torch.int32, device="cuda")
        dn = torch.empty(P, dtype=torch.int32, device="cuda")

        def run():
            L.check(L.lib().orbg_search_for_triangulation_batch_device(
                h, C.byref(K), cap, i1.data_ptr(), i2.data_ptr(), dg.data_ptr(), P, 0, 0,
                dm.data_ptr(), dn.data_ptr()), "tri")
        s_step, avg = timed(ctx, "tri_match", run, args.steps, args.warmup)
        algo = P * (2 * 2000 * 69 + 2000 * 4)
        r = line("ORBmatcher::SearchForTriangulation KeyFrame pairs/s (CreateNewMapPoints)",
                 "pairs/s", P, s_step, avg, algo,
                 "%d pairs of 2000-feature KeyFrames (120 FeatureVector nodes, 60%% stereo, 25%% "
                 "with a MapPoint), bOnlyStereo false, checkOri false" % P,
                 {"dtype": "u8/f32", "matches_per_pair": round(float(dn.cpu().numpy().mean()), 1)})
        if O is not None:
            p = O.params(nfeatures=2000)
            sf, s2 = np.array(p.scale[:8], np.float32), np.array(p.sigma2[:8], np.float32)
            t0 = time.perf_counter()
            calls = 0
            while time.perf_counter() - t0 < 3.0:
                k1, k2, g, _, _ = cases[calls % NQ]
                O.search_for_triangulation(k1, k2, g, sf, s2)
                calls += 1
            cdt = time.perf_counter() - t0
            r["cpu_baseline"] = {"value": round(calls / cdt, 1), "unit": "pairs/s", "cores": 1,
                                 "kind": "port", "sample": "%d pairs, oracle -O3, one thread, "
                                 "%.2f s" % (calls, cdt)}
        print(json.dumps(r), flush=True)

    for sim3 in (False, True):
        if args.only not in ("", "fuse_sim3" if sim3 else "fuse"):
            continue
        fuse_line(args, L, T, O, ctx, h, sim3)
    if args.only in ("", "triangulate"):
        triangulate_line(args, L, O, ctx, h)


def triangulate_line(args, L, O, ctx, h):
    import torch
    import test_oracle_triangulate as TT
    NQ, REP, cap, N = 64, 16, 2048, 2000
    cases = [TT.tri_pair_case(L, 900 + q, n=N, baseline=0.3 + 0.05 * q) for q in range(NQ)]
    nk = 2 * NQ
    kps = np.zeros((nk, cap), L.KP_DTYPE)
    raw = np.zeros((nk, cap), L.KP_DTYPE)
    ur = np.full((nk, cap), -1, np.float32)
    dp = np.zeros((nk, cap), np.float32)
    cnt = np.full(nk, N, np.int32)
    cam = np.zeros(nk, L.KF_CAMERA_DTYPE)
    for q, c in enumerate(cases):
        for s, kf, cm in ((2 * q, c[0], c[2]), (2 * q + 1, c[1], c[3])):
            kps[s, :N], raw[s, :N], ur[s, :N], dp[s, :N] = kf["kps"], kf["kps_raw"], kf["uright"], kf["depth"]
            cam[s] = np.asarray(cm).view(L.KF_CAMERA_DTYPE)
    P = NQ * REP
    qq = np.arange(P) % NQ
    m12 = np.full((P, cap), -1, np.int32)
    for p in range(P):
        m12[p, :N] = cases[qq[p]][4]
    t = {k: dev(v) for k, v in dict(kps=kps, raw=raw, ur=ur, dp=dp, cnt=cnt, cam=cam,
                                    m12=m12).items()}
    K = L.KeyFrames(None, t["kps"].data_ptr(), t["ur"].data_ptr(), None, t["cnt"].data_ptr(),
                    None, None, None, None)
    i1 = torch.from_numpy((2 * qq).astype(np.int32)).cuda()
    i2 = torch.from_numpy((2 * qq + 1).astype(np.int32)).cuda()
    dx = torch.empty(P * cap * 3, dtype=torch.float32, device="cuda")
    dst = torch.empty(P * cap, dtype=torch.int8, device="cuda")
    dn = torch.empty(P, dtype=torch.int32, device="cuda")

    def run():
        L.check(L.lib().orbg_triangulate_batch_device(
            h, C.byref(K), t["raw"].data_ptr(), t["dp"].data_ptr(), cap, t["cam"].data_ptr(),
            i1.data_ptr(), i2.data_ptr(), t["m12"].data_ptr(), P, dx.data_ptr(),
            dst.data_ptr(), dn.data_ptr()), "triangulate")
    s_step, avg = timed(ctx, "triangulate", run, args.steps, args.warmup)
    matched = int((m12 >= 0).sum())
    algo = P * N * 145
    r = line("LocalMapping::CreateNewMapPoints triangulation: matched pairs/s", "matches/s",
             matched, s_step, avg, algo,
             "%d KeyFrame pairs of 2000 features (60%% stereo, 8%% wrong / 10%% no match), "
             "%d matched pairs per launch" % (P, matched),
             {"dtype": "f32/f64", "new_points_per_pair": round(float(dn.cpu().numpy().mean()), 1),
              "keyframe_pairs_per_s": round(P / s_step, 1)})
    if O is not None:
        p = O.params(nfeatures=2000)
        sf, s2 = np.array(p.scale[:8], np.float32), np.array(p.sigma2[:8], np.float32)
        t0 = time.perf_counter()
        calls = done = 0
        while time.perf_counter() - t0 < 3.0:
            c = cases[calls % NQ]
            O.triangulate(c[0], c[1], c[2], c[3], c[4], sf, s2, 1.2)
            done += int((c[4] >= 0).sum())
            calls += 1
        cdt = time.perf_counter() - t0
        r["cpu_baseline"] = {"value": round(done / cdt, 1), "unit": "matches/s", "cores": 1,
                             "kind": "port", "sample": "%d KeyFrame pairs (%d matches), oracle "
                             "-O3, one thread, %.2f s" % (calls, done, cdt)}
    print(json.dumps(r), flush=True)


def fuse_line(args, L, T, O, ctx, h, sim3):
    import torch
    NQ, REP, cap, mcap = 32, 8, 2048, 2000
    cases = [T.fuse_case(L, 700 + q, n=2000, nmp=mcap, scale=(0.6 + 0.05 * q) if sim3 else None)
             for q in range(NQ)]
    desc = np.zeros((NQ, cap, 32), np.uint8)
    kps = np.zeros((NQ, cap), L.KP_DTYPE)
    ur = np.zeros((NQ, cap), np.float32)
    cnt = np.zeros(NQ, np.int32)
    P = NQ * REP
    cams = np.zeros(P, L.FRUSTUM_DTYPE)
    mps = np.zeros((P, mcap), L.MAPPOINT_DTYPE)
    md = np.zeros((P, mcap, 32), np.uint8)
    mc = np.full(P, mcap, np.int32)
    for j, (kf, fc, m, mdsc) in enumerate(cases):
        desc[j, :2000], kps[j, :2000], ur[j, :2000], cnt[j] = kf["desc"], kf["kps"], kf["uright"], 2000
    for p in range(P):
        kf, fc, m, mdsc = cases[p % NQ]
        cams[p], mps[p], md[p] = fc, m, mdsc
    t = {k: dev(v) for k, v in dict(desc=desc, kps=kps, ur=ur, cnt=cnt, cams=cams, mps=mps,
                                    md=md, mc=mc).items()}
    K = L.KeyFrames(t["desc"].data_ptr(), t["kps"].data_ptr(), t["ur"].data_ptr(), None,
                    t["cnt"].data_ptr(), None, None, None, None)
    kfi = torch.from_numpy((np.arange(P) % NQ).astype(np.int32)).cuda()
    bi = torch.empty(P * mcap, dtype=torch.int32, device="cuda")
    bd = torch.empty(P * mcap, dtype=torch.int32, device="cuda")
    nf = torch.empty(P, dtype=torch.int32, device="cuda")

    fn = L.lib().orbg_fuse_sim3_batch_device if sim3 else L.lib().orbg_fuse_batch_device
    th = 4.0 if sim3 else 3.0

    def run():
        L.check(fn(h, C.byref(K), cap, kfi.data_ptr(), t["cams"].data_ptr(),
                   t["mps"].data_ptr(), t["md"].data_ptr(), t["mc"].data_ptr(), mcap, P, th,
                   bi.data_ptr(), bd.data_ptr(), nf.data_ptr()), "fuse")
    s_step, avg = timed(ctx, "fuse_sim3" if sim3 else "fuse", run, args.steps, args.warmup)
    # per KeyFrame its keypoints and descriptors (+ mvuRight unless Sim3); per MapPoint
    # its record, descriptor and bestIdx / bestDist
    algo = P * (2000 * (60 if sim3 else 64) + mcap * 76)
    if sim3:
        title = ("ORBmatcher::Fuse(pKF, Scw, vpPoints, th, vpReplacePoint) search: map "
                 "points/s (LoopClosing::SearchAndFuse)")
        wl = "%d (KeyFrame of 2000 keypoints, 2000 loop MapPoints, Sim3 scale 0.6-2.15) pairs, th 4" % P
    else:
        title = "ORBmatcher::Fuse(pKF, vpMapPoints) search: map points/s (SearchInNeighbors)"
        wl = "%d (KeyFrame of 2000 keypoints, 2000 MapPoints) pairs, th 3" % P
    r = line(title, "points/s", P * mcap, s_step, avg, algo, wl,
             {"dtype": "f32/f64", "fused_per_pair": round(float(nf.cpu().numpy().mean()), 1)})
    if O is not None:
        p = O.params(nfeatures=2000)
        sf, isg = np.array(p.scale[:8], np.float32), np.array(p.inv_sigma2[:8], np.float32)
        t0 = time.perf_counter()
        calls = 0
        while time.perf_counter() - t0 < 3.0:
            kf, fc, m, mdsc = cases[calls % NQ]
            if sim3:
                O.fuse_sim3_search(kf, fc.view(O.FRUSTUM_DTYPE), m.view(O.MAPPOINT_DTYPE),
                                   mdsc, th, sf)
            else:
                O.fuse_search(kf, fc.view(O.FRUSTUM_DTYPE), m.view(O.MAPPOINT_DTYPE), mdsc,
                              th, sf, isg)
            calls += 1
        cdt = time.perf_counter() - t0
        r["cpu_baseline"] = {"value": round(calls * mcap / cdt, 1), "unit": "points/s",
                             "cores": 1, "kind": "port", "sample": "%d x %d map points, "
                             "oracle -O3, one thread, %.2f s" % (calls, mcap, cdt)}
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
