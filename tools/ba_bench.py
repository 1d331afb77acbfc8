#!/usr/bin/env python3
"""LocalBundleAdjustment linearisation throughput (configs[4]: KITTI00-like windows).

One "iteration" = g2o's computeActiveErrors + buildSystem arithmetic for every edge of W
independent LBA windows (10 local + 10 fixed KFs, 6000 points, ~27k edges, 60% stereo,
KITTI intrinsics), HBM-resident: orbg_ba_linearize_device -- k_ba_edges (thread per point
over its edges, fp64: H_pl per edge, the point blocks) + k_ba_pose_mfma (MFMA f64 pose
blocks, rows recomputed) -- and the error pass orbg_ba_errors_device (k_ba_errors: chi2 and
the robust term per edge).  Prints one JSON line with edges/s, per-kernel HIP-event times,
the HBM roofline of k_ba_edges (108 algorithmic bytes per edge; beside it the
bytes the ABI makes unavoidable: the 112-byte edge record in, H_pl's 144 bytes out, the
point's 24 + 96 bytes per edge share) and the oracle (fp64 C restatement) on one window on
one host core.

    python tools/ba_bench.py [--windows 64] [--iters 20] [--warmup 3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0
EDGE_ALGO_BYTES = 108  # per-edge algorithmic bytes
F64_MFMA_PEAK_TFLOPS = 78.6  # MI355X FP64 matrix, AMD spec (the guide lists no FP64 row)
PMC_BA = "r06_ba_pmc_kernels.json"  # tools/profile.sh r06_ba tools/ba_bench.py (round 6 build)


def schur_roofline(poses, edges, sk, iters, pk):
    """The Schur solve's kernels against their bounds (csrc/schur_kernels.hip):
    - k_schur_blocks: one v_mfma_f64_4x4x4f64 per (e1, e2) pair of free-pose edges of one
      landmark (a <= b in the landmark's edge list): pairs = sum over points of f (f + 1) / 2,
      f = the point's active edges to free poses.  Issued 512 FLOP per MFMA (4 blocks x 4x4x4
      x 2); useful 216 (the 6x3 x 3x6 product, 2 FLOP per multiply-add).  Algorithmic bytes
      per pair: the pair's B D^-1 (6x3 f64, 144 B) and H_pl (3x6 f64, 144 B), each read once
      per pair as the kernel does (no reuse across pairs is assumed); the dense system's
      writes (36 f64 per upper block, mirrored) are added per launch.
    - k_schur_points: per active edge slot to a free pose, H_pl (144 B) + the point's H_ll | b_l
      (96 B) in and the 24-f64 record (192 B) out.
    mfma_frac / traffic from the committed PMC pass when it holds the kernel (pmc_source)."""
    fixed = poses["fixed"] != 0
    act = edges["active"] != 0
    free_e = act & ~fixed[edges["pose"]]
    f = np.bincount(edges["point"][free_e], minlength=1).astype(np.int64)
    pairs = int((f * (f + 1) // 2).sum())
    nfree = int((~fixed).sum())
    nslot_free = int(free_e.sum())
    out = {"pairs_per_launch": pairs, "free_poses": nfree, "free_slots": nslot_free}

    def avg(k):
        v = sk.get(k)
        return v[0] / max(v[1], 1) if v else None

    ms = avg("schur_blocks")
    if ms:
        # upper blocks: the diagonal ones + the distinct free-pose pairs sharing a landmark
        # (an upper bound on the block count is enough for the write term: 36 f64 x 2 each)
        flop_issued = pairs * 512
        flop_useful = pairs * 216
        byts = pairs * 288
        out["schur_blocks"] = {
            "avg_launch_ms": round(ms, 5),
            "mfma_per_launch": pairs,
            "issued_tflops": round(flop_issued / (ms * 1e-3) / 1e12, 3),
            "useful_tflops": round(flop_useful / (ms * 1e-3) / 1e12, 3),
            "peak_tflops": F64_MFMA_PEAK_TFLOPS,
            "useful_frac_of_peak": round(flop_useful / (ms * 1e-3) / 1e12 / F64_MFMA_PEAK_TFLOPS, 4),
            "useful_work_per_mfma": round(216 / 512, 4),
            "algo_bytes_per_launch": byts,
            "achieved_gbs": round(byts / (ms * 1e-3) / 1e9, 1),
            "hbm_frac": round(byts / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "pairs_per_s": round(pairs / (ms * 1e-3), 1),
            "mfma_frac": pk.get("schur_blocks", {}).get("mfma_frac"),
            "traffic": pk.get("schur_blocks", {}).get("hbm_bytes_per_launch"),
        }
    ms = avg("schur_points")
    if ms:
        byts = nslot_free * (144 + 96 + 192)
        out["schur_points"] = {
            "avg_launch_ms": round(ms, 5), "algo_bytes_per_launch": byts,
            "achieved_gbs": round(byts / (ms * 1e-3) / 1e9, 1),
            "hbm_frac": round(byts / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "traffic": pk.get("schur_points", {}).get("hbm_bytes_per_launch")}
    for k in ("schur_rhs", "schur_ldlt", "schur_backsub"):
        ms = avg(k)
        if ms:
            out[k] = {"avg_launch_ms": round(ms, 5),
                      "traffic": pk.get(k, {}).get("hbm_bytes_per_launch"),
                      "wait_inst_any_frac": pk.get(k, {}).get("wait_inst_any_frac")}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--windows", type=int, default=64)
    ap.add_argument("--distinct", type=int, default=4, help="distinct synthetic windows, tiled")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--jacobians", action="store_true",
                    help="also store g2o's per-edge Jacobians eout.jp / jt (orbg_ba_set_jacobians)")
    ap.add_argument("--no-graph", action="store_true",
                    help="orbg_ba_build_system_device / orbg_ba_errors_device on the 104-byte edge "
                         "records instead of an orbg_ba_graph (packed 24-byte edges)")
    ap.add_argument("--records", action="store_true",
                    help="buildSystem through orbg_ba_linearize_device (H_pl inside the 400-byte "
                         "orbg_edge_out records) instead of orbg_ba_build_system_device (compact "
                         "H_pl)")
    ap.add_argument("--edge-errors", action="store_true",
                    help="also store eout.err / chi2 / rho1 in the linearisation pass "
                         "(orbg_ba_set_edge_errors; the iteration's error pass provides them)")
    ap.add_argument("--no-solve", action="store_true",
                    help="skip the full LM iteration line (build + errors + the device-resident "
                         "Schur solve, orbg_ba_graph_schur_solve)")
    args = ap.parse_args()

    import torch
    from orb_slam2_test_amd import synthetic as S
    from orb_slam2_test_amd.optimizer import DeviceLBA
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_gpu_ba import concat_windows

    base = [S.ba_window(seed=500 + i) for i in range(args.distinct)]
    poses, pts, edges = concat_windows([base[i % args.distinct] for i in range(args.windows)])
    use_records = args.records or args.jacobians or args.edge_errors
    use_graph = not (use_records or args.no_graph)
    lba = DeviceLBA(poses, pts, edges, jacobians=args.jacobians, edge_errors=args.edge_errors,
                    graph=use_graph)

    def iteration():
        if use_records:
            lba.linearize()
        else:
            lba.build_system()
        lba.errors()

    for _ in range(args.warmup):
        iteration()
    lba.ctx.sync()
    torch.cuda.synchronize()
    # the timed pass carries no profiling events (a HIP event between launches costs ~10 us of
    # queue time each); a second pass of the same iterations times each kernel with events
    t0 = time.perf_counter()
    for _ in range(args.iters):
        iteration()
    lba.ctx.sync()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    lba.ctx.profile(True)
    lba.ctx.profile_reset()
    for _ in range(args.iters):
        iteration()
    lba.ctx.sync()
    kern = lba.ctx.profile_read()
    lba.ctx.profile(False)
    ne = len(edges)
    out = {
        "metric": "LBA linearisation edges/s (computeActiveErrors + buildSystem arithmetic)",
        "value": round(ne * args.iters / dt, 1), "unit": "edges/s", "higher_is_better": True,
        "dtype": "f64", "data": "synthetic",
        "config": {"workload": "configs[4]: %d KITTI00-like LBA windows (20 KFs, 6000 points)"
                               % args.windows, "edges": ne, "poses": len(poses),
                   "points": len(pts), "stereo_frac": round(float(np.mean(edges["stereo"])), 3),
                   "edge_jacobians_stored": bool(args.jacobians),
                   "edge_errors_stored": bool(args.edge_errors),
                   "iteration": ("orbg_ba_linearize_device + orbg_ba_errors_device" if use_records
                                 else "orbg_ba_graph_build_system + orbg_ba_graph_errors (packed "
                                      "24-byte edges)" if use_graph
                                 else "orbg_ba_build_system_device + orbg_ba_errors_device") +
                                " (buildSystem + computeActiveErrors)"},
        "ms_per_iter": round(dt / args.iters * 1e3, 4),
        "kernels": {k: {"ms_per_iter": round(v[0] / args.iters, 4),
                        "avg_launch_ms": round(v[0] / max(v[1], 1), 5)} for k, v in kern.items()},
    }
    if "ba_edges" in kern:
        ms = kern["ba_edges"][0] / max(kern["ba_edges"][1], 1)
        ach = ne * EDGE_ALGO_BYTES / (ms * 1e-3) / 1e9
        # the bytes the ABI makes unavoidable: the edge record and its CSR slot in, H_pl out
        # (g2o's _Hpl, read by the Schur step: not in SURVEY 8d's 108 B), the point in and its
        # H_ll | b_l out
        from orb_slam2_test_amd import _lib as LB
        # the edge as the iteration reads it (24-byte packed edge of a graph, or the record)
        ebytes = 24 if use_graph else LB.EDGE_DTYPE.itemsize
        abi = ne * (ebytes + 4 + 144) + len(pts) * (24 + 4 + 96)
        out["roofline"] = {"kernel": "ba_edges", "bound": "hbm", "achieved": round(ach, 1),
                           "peak": HBM_PEAK_GBS, "unit": "GB/s",
                           "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
                           "algo_bytes_per_launch": ne * EDGE_ALGO_BYTES,
                           "abi_min_bytes_per_launch": abi,
                           "abi_min_achieved": round(abi / (ms * 1e-3) / 1e9, 1),
                           "avg_launch_ms": round(ms, 5)}
    pk = {}
    pmc = os.path.join(ROOT, "profiles", PMC_BA)
    if os.path.exists(pmc):
        with open(pmc) as f:
            pk = json.load(f)
    if "roofline" in out:
        tr = pk.get("ba_edges", {}).get("hbm_bytes_per_launch")
        out["roofline"]["traffic"] = tr
        if tr:
            out["roofline"]["traffic_over_algo"] = round(tr / out["roofline"]["algo_bytes_per_launch"], 3)
            out["roofline"]["traffic_over_abi_min"] = round(tr / out["roofline"]["abi_min_bytes_per_launch"], 3)
        out["roofline"]["pmc_source"] = os.path.relpath(pmc, ROOT) if pk else None
    if "ba_pose_mfma" in kern:
        # MFMAs issued by the pose-slice pass (csrc/ba_kernels.hip ba_pose_slice): per slice of
        # <= 64 edges of a free pose, the active edges' nonzero rows (2 mono, 3 stereo)
        # compacted and padded to a multiple of 16, one v_mfma_f64_4x4x4f64 per 4 rows
        # (4 blocks x 4x4 x K 4 = 512 FLOP).  Useful work: the 6 x 7 entries of [H_pp | b_p]
        # of the 8 x 8 tile (42 / 64) over the rows that are not padding.
        nmfma, rows_used = 0, 0
        fixed = poses["fixed"] != 0
        order = np.argsort(edges["pose"], kind="stable")
        D = np.where(edges["active"] != 0, np.where(edges["stereo"] != 0, 3, 2), 0)[order]
        pe = edges["pose"][order]
        starts = np.searchsorted(pe, np.arange(len(poses) + 1))
        for pidx in np.nonzero(~fixed)[0]:
            a, b = starts[pidx], starts[pidx + 1]
            for s0 in range(a, b, 64):
                nr = int(D[s0:min(b, s0 + 64)].sum())
                nmfma += ((nr + 15) // 16) * 4
                rows_used += nr
        ms = kern["ba_pose_mfma"][0] / max(kern["ba_pose_mfma"][1], 1)
        tf = nmfma * 512 / (ms * 1e-3) / 1e12
        useful = (42.0 / 64.0) * rows_used / max(4 * nmfma, 1)
        out["mfma"] = {"kernel": "ba_pose_mfma (k_ba_slices_special)",
                       "instr": "v_mfma_f64_4x4x4f64", "mfma_per_launch": nmfma,
                       "issued_tflops": round(tf, 2), "peak_tflops": F64_MFMA_PEAK_TFLOPS,
                       "issued_frac": round(tf / F64_MFMA_PEAK_TFLOPS, 4),
                       "useful_work_frac": round(useful, 4),
                       "useful_tflops": round(tf * useful, 2),
                       "mfma_frac": pk.get("ba_pose_mfma", {}).get("mfma_frac"),
                       "note": "issued = every MFMA the pass issues; useful = the [H_pp | b_p] "
                               "entries (42 of the 8x8 tile's 64) x the rows that are not "
                               "padding; mfma_frac = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x "
                               "GPU cycles) from the committed PMC pass (pmc_source)"}
    if use_graph and not args.no_solve:
        # g2o's whole LM iteration on the device: buildSystem + computeActiveErrors + the
        # Schur solve (setLambda, BlockSolver<6,3>::solve), one stream, no host copy
        lba.schur_plan(poses["fixed"])
        lam = 1e-4 * float(np.abs(lba.d_hpose.cpu().numpy().reshape(len(poses), 36)[:, ::7]).max())

        def lm_iteration():
            lba.build_system()
            lba.errors()
            lba.schur_solve(lam)

        for _ in range(args.warmup):
            lm_iteration()
        lba.ctx.sync()
        t0 = time.perf_counter()
        for _ in range(args.iters):
            lm_iteration()
        lba.ctx.sync()
        ldt = time.perf_counter() - t0
        lba.ctx.profile(True)
        lba.ctx.profile_reset()
        for _ in range(args.iters):
            lba.schur_solve(lam)
        lba.ctx.sync()
        sk = lba.ctx.profile_read()
        lba.ctx.profile(False)
        out["lm_iteration"] = {
            "what": "orbg_ba_graph_build_system + orbg_ba_graph_errors + orbg_ba_graph_schur_solve "
                    "(Schur products on v_mfma_f64_4x4x4f64, one dense LDLT per window)",
            "ms_per_iter": round(ldt / args.iters * 1e3, 4),
            "edges_per_s": round(ne * args.iters / ldt, 1),
            "schur_ms": round(sum(v[0] for k, v in sk.items() if k.startswith("schur")) / args.iters, 4),
            "schur_kernels_ms": {k: round(v[0] / args.iters, 4) for k, v in sk.items()},
            "ok": int(lba.d_ok.cpu().numpy()[0]), "lambda": lam}
        out["schur_roofline"] = schur_roofline(poses, edges, sk, args.iters, pk)
        # optimizer.optimize(5) end to end (orbg_ba_graph_optimize): per trial the build, the
        # Schur solve, the update, the error pass and the three scalars read back, from the
        # same starting estimates each run
        p0, q0 = lba.d_poses.clone(), lba.d_points.clone()
        runs, rep = 3, None
        lba.ctx.sync()
        t0 = time.perf_counter()
        for _ in range(runs):
            lba.d_poses.copy_(p0)
            lba.d_points.copy_(q0)
            torch.cuda.synchronize()  # torch's copies before liborbg's stream reads them
            rep = lba.optimize(5)
        lba.ctx.sync()
        odt = time.perf_counter() - t0
        out["lm_optimize"] = {
            "what": "orbg_ba_graph_optimize(5): g2o's Levenberg-Marquardt with every trial's build, "
                    "Schur solve, update and error pass on the device, three scalars read back "
                    "per trial",
            "ms_per_optimize5": round(odt / runs * 1e3, 3),
            "ms_per_trial": round(odt / runs / max(rep["trials"], 1) * 1e3, 4),
            "report": {k: (round(v, 6) if isinstance(v, float) else v) for k, v in rep.items()}}
    if not args.no_cpu:
        from oracle import pyoracle as O
        p, q, e = base[0]
        t0 = time.perf_counter()
        reps = 0
        while time.perf_counter() - t0 < 5.0:
            O.ba_linearize(p, q, e)
            reps += 1
        cdt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(len(e) * reps / cdt, 1), "unit": "edges/s",
                               "cores": 1, "kind": "port",
                               "sample": "%d x one window (%d edges), oracle/ba_oracle.c -O3, "
                                         "1 thread, %.1f s" % (reps, len(e), cdt)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
