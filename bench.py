#!/usr/bin/env python3
"""bench.py -- frames/s of ORB extract + match at 1241x376, 2000 features, 8 levels.

A step = one pass of the hot path over one batch of B synthetic frames per GPU, resident
in HBM before the timed region (sequence.BenchStep, which the -m gpu parity tests run
unchanged):
  ORBextractor::operator() on every frame (pyramid, FAST cells, quadtree, blur,
  IC_Angle + rBRIEF) and, for every frame t, the matcher between t-1 and t
  (all-pairs Hamming knn2 + SearchForInitialization(window 100, nnratio 0.9, checkOri)).
The steps cycle through --blocks distinct resident blocks of the sequence, so a step never
re-reads the frames the step before it read.
Multi-GPU (torch.distributed.run, one process per GPU): frames are sharded (each rank
owns its own blocks of the sequence, weak scaling); the only collectives are RCCL
all_gathers of the per-frame outputs (keypoint and match counts, vnMatches12 rows) per step.

Prints ONE JSON line on rank 0 (contract in the task statement):
  value = all ranks' frames / max-over-ranks wall time of K steps,
  roofline = dominant kernel, algorithmic bytes / HIP-event duration (on the stream the
             kernels run on) vs 8 TB/s HBM,
  cpu_baseline = the oracle (C restatement, "port") on a bounded sample on host cores.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "frames/sec ORB extract+match, 1241×376 2000feat 8lvl, 1/2/4/8 GPU"
METRIC_STEREO = ("stereo frames/sec ORB extract L+R + ComputeStereoMatches, 1241×376 "
                 "2000feat/eye 8lvl")
W, H, NFEAT, NLEV = 1241, 376, 2000, 8
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
# SURVEY.md 8d algorithmic bytes per unit
PYR_BYTES = 1444097          # all 8 levels at 1241x376
FRAME_ALGO_BYTES = 2701578   # extract 2,533,578 + match 168,000
STEREO_FRAME_ALGO_BYTES = 5235156  # 2 x extract + match
EXTRACT_FRAME_ALGO_BYTES = 2533578  # configs[1] / C2: ORBextractor only
METRIC_EXTRACT = "frames/sec ORBextractor only, 1241×376 2000feat 8lvl (configs[1], C2)"


# serial-pass PMC profiles of the bench lines (tools/round_prof.sh), copied from the run dirs
PMC_MONO = "r06e_pmc_kernels.json"
PMC_STEREO = "r06e_stereo_pmc_kernels.json"


def kernel_algo_bytes(name, B, npairs, ncand, nkp, launches_per_step, ndepth=0, blur_plan=None):
    """Algorithmic bytes of one launch of `name` (see DESIGN.md 'Kernels').  B images, npairs
    frame pairs, ncand FAST candidates and nkp keypoints over the batch, ndepth stereo
    matches (keypoints with a depth) over the batch.  blur_plan = orbg_get_blur_plan's (fused,
    interior px, border px) per frame: with the GaussianBlur fused into the FAST cells,
    fast_cells also writes the interior's blurred bytes and "blur" (k_blur_border) reads and
    writes only the border's."""
    lv = level_sizes()
    fused, inner, border = blur_plan if blur_plan else (False, 0, PYR_BYTES)
    if name == "resize":
        tot = B * sum(lv[l - 1][0] * lv[l - 1][1] + lv[l][0] * lv[l][1] for l in range(1, NLEV))
    elif name == "fast_cells":
        tot = B * PYR_BYTES + 8 * ncand + (B * inner if fused else 0)
    elif name == "blur":
        tot = 2 * B * (border if fused else PYR_BYTES)
    elif name == "octree":
        tot = 8 * ncand + 4 * nkp
    elif name == "orient_desc":
        tot = nkp * (749 + 512 + 4 + 28 + 32)
    elif name == "knn2":
        kp = nkp / max(B, 1)
        tot = npairs * (2 * kp * 32 + kp * 12)
    elif name == "init_cands":
        kp = nkp / max(B, 1)
        tot = npairs * (kp * 28 + kp * 32 + kp * 64)
    elif name == "init_resolve":
        kp = nkp / max(B, 1)
        tot = npairs * (kp * 64 + kp * 4)
    elif name == "stereo_match":
        kp = nkp / max(B, 1)
        tot = npairs * (2 * kp * (32 + 28) + kp * 8)  # both frames' kps + desc, uR + depth
    elif name == "stereo_rows":
        # right keypoints' (y, octave) in; row offsets (H + 1) and the row lists (u16 per
        # listed row: a keypoint of octave l spans ~4 scale_l + 2 rows) out
        kp = nkp / max(B, 1)
        fpl = features_per_level()
        sc = [1.2 ** l for l in range(NLEV)]
        rows = sum(f * (4 * s + 2) for f, s in zip(fpl, sc)) / sum(fpl)
        tot = npairs * (kp * 8 + (H + 1) * 4 + kp * rows * 2)
    elif name == "stereo_sad":
        # per match: the 11x11 left patch and the 11 x 21 right strip at the keypoint's level,
        # (uR, depth, SAD) out
        tot = ndepth * (11 * 11 + 11 * 21 + 12)
    elif name == "stereo_median":
        tot = ndepth * (4 + 8)  # SADs in, cleared (uR, depth) out
    else:
        return None
    return tot / max(launches_per_step, 1)


def features_per_level():
    """mnFeaturesPerLevel at 2000 features, 8 levels, 1.2 (ORBextractor.cc:466-476)."""
    f = np.float32(1.0) / np.float32(1.2)
    d = np.float32(NFEAT) * (np.float32(1) - f) / (np.float32(1) - np.float32(f ** NLEV))
    out, s = [], 0
    for _ in range(NLEV - 1):
        out.append(int(np.rint(d)))
        s += out[-1]
        d = np.float32(d * f)
    return out + [max(NFEAT - s, 0)]


def level_sizes():
    sizes, s = [], np.float32(1.0)
    for l in range(NLEV):
        inv = np.float32(1.0) / s
        sizes.append((int(np.rint(np.float32(W) * inv)), int(np.rint(np.float32(H) * inv))))
        s = np.float32(np.float64(s) * np.float64(np.float32(1.2)))
    return sizes


def cpu_baseline_stereo(lefts, rights, threads, nframes, nframes_1core=8):
    """oracle/ (C restatement) on host threads, as the mono baseline: extract L + R +
    ComputeStereoMatches per stereo frame, `nframes` frames over `threads` threads (ctypes
    calls release the GIL), and `nframes_1core` frames on one thread."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import pyoracle as O
    from orb_slam2_test_amd import synthetic as S
    p = O.params(nfeatures=NFEAT, nlevels=NLEV)

    def one(i):
        i %= len(lefts)
        lft = O.extract(p, lefts[i], with_pyramid=True)
        rgt = O.extract(p, rights[i], with_pyramid=True)
        O.stereo_matches(p, lft, rgt, W, H, S.KITTI_BF, S.KITTI_BF / S.KITTI_FX)

    def run(n, th):
        t0 = time.perf_counter()
        with ThreadPoolExecutor(th) as pool:
            list(pool.map(one, range(n)))
        return time.perf_counter() - t0

    dt = run(nframes, threads)
    dt1 = run(nframes_1core, 1)
    ncpu, model = host_cpu()
    return {"value": round(nframes / dt, 3), "unit": "stereo frames/s", "cores": threads,
            "kind": "port", "value_1core": round(nframes_1core / dt1, 3),
            "host_logical_cpus": ncpu, "host_affinity_cpus": len(os.sched_getaffinity(0)),
            "host_cpu_model": model,
            "sample": ("%d synthetic 1241x376 stereo frames (extract L+R 2000 feat/8 lvl + "
                       "ComputeStereoMatches), oracle/ C restatement -O3, %d threads, %.1f s "
                       "wall; 1 thread: %d frames, %.1f s" % (nframes, threads, dt,
                                                             nframes_1core, dt1))}


def cpu_baseline_extract(frames, threads, nframes, nframes_1core=48):
    """oracle/ ORBextractor only (C2) on host threads (ctypes calls release the GIL)."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import pyoracle as O
    p = O.params(nfeatures=NFEAT, nlevels=NLEV)

    def run(n, th):
        t0 = time.perf_counter()
        with ThreadPoolExecutor(th) as pool:
            list(pool.map(lambda i: O.extract(p, frames[i % len(frames)]), range(n)))
        return time.perf_counter() - t0

    dt = run(nframes, threads)
    dt1 = run(nframes_1core, 1)
    ncpu, model = host_cpu()
    return {"value": round(nframes / dt, 3), "unit": "frames/s", "cores": threads,
            "kind": "port", "value_1core": round(nframes_1core / dt1, 3),
            "host_logical_cpus": ncpu, "host_affinity_cpus": len(os.sched_getaffinity(0)),
            "host_cpu_model": model,
            "sample": ("%d synthetic 1241x376 frames (ORBextractor 2000 feat/8 lvl), oracle/ C "
                       "restatement -O3, %d threads, %.1f s wall; 1 thread: %d frames, %.1f s"
                       % (nframes, threads, dt, nframes_1core, dt1))}


def cpu_share():
    """Host threads for the CPU baseline: the CPUs this process may run on
    (os.sched_getaffinity), capped at the lease's CPU share when the environment states one
    (OMP_NUM_THREADS: 16 on a 1-GPU box of this pool, whose sched_getaffinity shows the
    whole machine)."""
    n = len(os.sched_getaffinity(0))
    share = os.environ.get("OMP_NUM_THREADS")
    if share and share.isdigit() and int(share) > 0:
        n = min(n, int(share))
    return max(1, n)


def host_cpu():
    """The GPU box's host: logical CPUs (std::thread::hardware_concurrency) and the model
    name lscpu prints (/proc/cpuinfo)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return os.cpu_count(), model


def cpu_baseline(frames, threads, nframes, nframes_1core=32):
    """oracle/ (C restatement) on host pthreads: `threads` threads over `nframes` frames,
    and one thread over `nframes_1core` frames (the reference's own single-threaded
    Tracking loop, mono_kitti.cc:78-90, extracts one frame per call)."""
    from oracle import pyoracle as O
    p = O.params(nfeatures=NFEAT, nlevels=NLEV)

    def run(n, th):
        idx = np.arange(n) % len(frames)
        sample = np.ascontiguousarray(frames[idx])
        t0 = time.perf_counter()
        O.frames_batch(p, sample, nthreads=th, window=100, nnratio=0.9)
        return time.perf_counter() - t0

    dt = run(nframes, threads)
    dt1 = run(nframes_1core, 1)
    ncpu, model = host_cpu()
    return {"value": round(nframes / dt, 3), "unit": "frames/s", "cores": threads,
            "kind": "port", "value_1core": round(nframes_1core / dt1, 3),
            "host_logical_cpus": ncpu, "host_affinity_cpus": len(os.sched_getaffinity(0)),
            "host_cpu_model": model,
            "sample": ("%d synthetic 1241x376 frames (extract 2000 feat/8 lvl + knn2 + "
                       "SearchForInitialization vs t-1), oracle/ C restatement -O3, %d pthreads, "
                       "%.1f s wall; 1 thread: %d frames, %.1f s.  The restatement is scalar C; "
                       "the reference runs OpenCV's SIMD FAST / resize / GaussianBlur, and its "
                       "README (README.md:117) reports a 27.4 ms median whole-tracking time per "
                       "KITTI03 frame on its authors' machine (extraction + matching + pose + "
                       "local map), so this CPU column understates the reference's CPU speed"
                       % (nframes, threads, dt, nframes_1core, dt1))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=None,
                    help="frames (stereo: L/R pairs) per GPU per step; default "
                         "sequence.BENCH_BATCH: 1024 (stereo 512 pairs = 1024 images), the fixed "
                         "cost of a step's dependent launches spread over more frames (512: "
                         "-2.5%%, 2048: -1%% frames/s)")
    ap.add_argument("--blocks", type=int, default=4,
                    help="distinct resident input blocks the steps cycle through (4 x 478 MB "
                         "> the 256 MB Infinity Cache: every step reads new frames); 1 = the "
                         "same block every step (round 2's bench)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0: the host CPUs this process may run on (os.sched_getaffinity), "
                         "capped at the lease's CPU share (OMP_NUM_THREADS, 16 on a 1-GPU box)")
    ap.add_argument("--cpu-frames", type=int, default=0, help="0: 256 x threads (~10-20 s)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--pipeline", type=int, default=int(os.environ.get("ORBG_PIPELINE", "1")),
                    help="1: pipelined batches (image half of step k+1 beside the keypoint half "
                         "of step k, orbg_set_pipeline); 0: one batch after the other")
    ap.add_argument("--serial", action="store_true",
                    help="run the timed steps serially (orbg_set_serial), as the roofline's "
                         "kernel-timing pass does: for PMC collection, not a bench line")
    ap.add_argument("--stereo", action="store_true",
                    help="configs[3]: stereo frames (extract L+R + ComputeStereoMatches)")
    ap.add_argument("--extract-only", action="store_true",
                    help="configs[1] (C2): ORBextractor only, no matching")
    ap.add_argument("--with-pose", action="store_true",
                    help="mono: the full batched-sequence step, with the pose/trajectory stub "
                         "of every pair (orbg_match_pose_batch_device) gathered beside the "
                         "summary and vnMatches12 rows (SURVEY.md 8e); not the headline metric")
    ap.add_argument("--host-input", action="store_true",
                    help="host-fed frames: the blocks sit in pinned host memory and every step's "
                         "block is copied H2D on a copy stream (3 device staging slots) "
                         "overlapped with the previous steps' extraction; PCIe-inclusive "
                         "frames/s, a second line beside the device-resident headline")
    ap.add_argument("--force-collective", action="store_true",
                    help="run the per-step RCCL all_gathers even at world size 1 (a one-rank "
                         "nccl process group): exercises the multi-GPU gather path on one GPU")
    args = ap.parse_args()

    # stdout carries exactly the one JSON line: everything else written to fd 1 (RCCL's
    # version banner at communicator init, library prints) goes to stderr
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)

    import torch
    import torch.distributed as dist
    from orb_slam2_test_amd import ORBextractor, sequence, synthetic

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist_info = {"world_size": 1, "backend": None}
    collective = world > 1 or args.force_collective
    if collective:
        if world == 1:  # a one-rank group outside torch.distributed.run
            import socket
            with socket.socket() as s:
                s.bind(("127.0.0.1", 0))
                port = s.getsockname()[1]
            for k, v in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", str(port)),
                         ("RANK", "0"), ("WORLD_SIZE", "1")):
                os.environ.setdefault(k, v)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        # what the collectives really run on (RCCL reports itself as "nccl" on ROCm)
        dist_info = {"world_size": dist.get_world_size(), "backend": dist.get_backend(),
                     "rccl": torch.cuda.nccl.version() if hasattr(torch.cuda, "nccl") else None}
    if not args.cpu_threads:
        args.cpu_threads = cpu_share()

    B = args.batch or sequence.BENCH_BATCH["stereo" if args.stereo else
                                           "extract" if args.extract_only else "mono"]
    # Streamed input: the step cycles through `nblocks` distinct resident blocks of the
    # sequence (nblocks x 478 MB > the 256 MB Infinity Cache at the defaults), so every step
    # reads frames the previous steps did not (no cross-step cache reuse of the input).
    nblocks = max(1, args.blocks)
    if args.stereo:
        lefts, rights, _ = synthetic.stereo_sequence(nblocks * B, H, W,
                                                     seed=synthetic.DEFAULT_SEED + 1000 * rank)
        blocks = []
        for k in range(nblocks):
            fr = np.empty((2 * B, H, W), np.uint8)
            fr[0::2], fr[1::2] = lefts[k * B:(k + 1) * B], rights[k * B:(k + 1) * B]
            blocks.append(fr)
    else:
        # batched-sequence partition (sequence.run_sharded): rank r's block k
        # holds frames [(k world + r) B, (k world + r + 1) B) of one cyclic sequence plus the
        # frame before it (1-frame halo), so its B pairs (t-1, t) match with no exchange
        n_total, ranges = synthetic.bench_block_ranges(B, world, rank, nblocks)
        blocks = synthetic.sequence_blocks(n_total, ranges, H, W)
        if args.extract_only:  # no pairs: the halo frame is not needed
            blocks = [np.ascontiguousarray(b[1:]) for b in blocks]
    frames = blocks[0]
    nimg = len(frames)
    d_blocks = [torch.from_numpy(b).to("cuda") for b in blocks]
    torch.cuda.synchronize()
    ext = ORBextractor(NFEAT, 1.2, NLEV, 20, 7, device=local, max_batch=nimg)
    # one non-null torch stream for everything: liborbg's kernels, the summary and RCCL
    # (the null stream's handle is 0, which orbg_set_stream reads as "own stream")
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    ext.ctx.set_stream(stream.cuda_stream)
    ext.ctx.set_pipeline(bool(args.pipeline))
    if args.serial:  # PMC runs (tools/round_prof.sh): one dispatch per kernel and step
        ext.ctx.set_serial(True)
    mode = "stereo" if args.stereo else "extract" if args.extract_only else "mono"
    bstep = sequence.BenchStep(ext, B, mode, world=world, with_pose=args.with_pose,
                               collective=collective)
    torch.cuda.synchronize()
    it = [0]

    def step():
        d = d_blocks[it[0] % nblocks]
        it[0] += 1
        bstep(d.data_ptr(), W, H)

    h2d = None
    if args.host_input:
        # Frame.cc:310-316 / mono_kitti.cc:78-90 read frames from host memory: here every
        # step's block goes H2D on its own stream into one of 3 device slots while the
        # extraction of the steps before runs.  The copy into a slot is issued once the step
        # that read it last is done (orbg_batch_acquire: the last reads of its input, IC_Angle's
        # level-0 patches, are done when its outputs are written), gated on the host: an event
        # on a compute stream that the host waits for after enqueuing the next step, so the
        # copy stream never waits on a device event (a copy queued behind one ran serialised
        # with the extraction: profiles/r05_host_input_trace.txt)
        h_blocks = [torch.from_numpy(b).pin_memory() for b in blocks]
        stage = [torch.empty_like(d_blocks[0]) for _ in range(3)]
        cstream = torch.cuda.Stream()
        gstream = torch.cuda.Stream()
        ev_copy = [torch.cuda.Event() for _ in range(3)]
        ev_done = [torch.cuda.Event() for _ in range(3)]

        def issue_copy(j):
            with torch.cuda.stream(cstream):
                stage[j % 3].copy_(h_blocks[j % nblocks], non_blocking=True)
                ev_copy[j % 3].record(cstream)

        # the H2D rate alone (the bound of a host-fed pipeline): the step's own copies (the
        # copy stream, the 3 staging slots), after an untimed round, the best of 5 rounds of 12
        # (round 5 timed 4 cold copies, and one round of 12 in round 6 came out 2% under the
        # host-fed line itself: the link's rate drifts from round to round)
        for j in range(3):
            issue_copy(j)
        torch.cuda.synchronize()
        nprobe, h2d = 12, 0.0
        for _ in range(5):
            t0 = time.perf_counter()
            for j in range(nprobe):
                issue_copy(j)
            torch.cuda.synchronize()
            h2d = max(h2d, nprobe * h_blocks[0].numel() / (time.perf_counter() - t0) / 1e9)
        for j in range(3):
            issue_copy(j)

        def step():  # noqa: F811 -- the host-fed step replaces the resident one
            k = it[0]
            it[0] += 1
            stream.wait_event(ev_copy[k % 3])
            bstep(stage[k % 3].data_ptr(), W, H)
            ext.ctx.batch_acquire(gstream.cuda_stream)
            ext.ctx.batch_release(gstream.cuda_stream)
            ev_done[k % 3].record(gstream)
            if k >= 1:
                ev_done[(k - 1) % 3].synchronize()  # step k - 1 no longer reads its slot
                issue_copy(k + 2)                   # into that slot: (k + 2) % 3 == (k - 1) % 3

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ncand, nkp = ext.ctx.batch_stats()
    ndepth = int(bstep.ssum[B:].sum().item()) if args.stereo else 0
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    # sticky device error flags (quadtree capacity overflows) of every timed batch: a step
    # that lost keypoints would make `value` invalid, so fail instead of reporting it
    ext.ctx.check_errors()
    if world > 1:
        e = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    # per-kernel HIP event times (roofline): a second pass of the same K steps, so that the
    # events recorded around every launch (~5% of a step) stay out of `value`.  It runs
    # serially (orbg_set_serial, the matching after the extraction): in the timed pass the
    # kernels of two batches and three streams overlap, and an event pair around a kernel
    # would time its neighbours too.
    kern = {}
    if not args.no_kernel_timing and not args.host_input:
        ext.ctx.set_serial(True)

        def step_serial():
            d = d_blocks[it[0] % nblocks]
            it[0] += 1
            ext.extract_batch_device(d.data_ptr(), nimg, W, H)
            if args.stereo:
                ext.ctx.sync()
                ext.stereo_batch_device(bstep.sl, bstep.sr, synthetic.KITTI_BF,
                                        synthetic.KITTI_BF / synthetic.KITTI_FX)
            elif not args.extract_only:
                ext.ctx.sync()
                ext.match_batch_device(bstep.f1, bstep.f2, 100, 0.9, True)
            ext.ctx.sync()

        step_serial()
        ext.ctx.profile(True)
        ext.ctx.profile_reset()
        for _ in range(args.steps):
            step_serial()
        torch.cuda.synchronize()
        kern = ext.ctx.profile_read()
        ext.ctx.profile(False)
        ext.ctx.set_serial(False)
        if world > 1:
            dist.barrier()

    frames_total = B * args.steps * world
    value = frames_total / elapsed
    out = None
    if rank == 0:
        # PMC figures from the committed serial-pass profile of this workload
        # (tools/round_prof.sh -> tools/pmc_kernels.py): HBM bytes per launch and the
        # fractions of the chip's VALU issue / LDS cycles each kernel used
        pmc = os.path.join(ROOT, "profiles", PMC_STEREO if args.stereo else PMC_MONO)
        pmc_all = {}
        if os.path.exists(pmc) and not args.extract_only:
            with open(pmc) as f:
                pmc_all = json.load(f)
        def pmc_hbm(name, lps):
            # per bench launch (one PROF_LAUNCH may be several dispatches: octree's level-0
            # pair), from the PMC run's per-step sum when it has one
            e = pmc_all.get(name, {})
            if e.get("hbm_bytes_per_step") and lps > 0:
                return int(e["hbm_bytes_per_step"] / lps)
            return e.get("hbm_bytes_per_launch")

        blur_plan = ext.ctx.blur_plan()
        kstats = {}
        for name, (ms, n) in kern.items():
            lps = n / max(args.steps, 1)
            avg = ms / max(n, 1)
            ab = kernel_algo_bytes(name, nimg, B, ncand, nkp, lps, ndepth, blur_plan)
            kstats[name] = {"ms_per_step": round(ms / args.steps, 4), "launches_per_step": lps,
                            "avg_launch_ms": round(avg, 5),
                            "algo_bytes_per_launch": None if ab is None else int(ab),
                            "achieved_GBps": None if ab is None else round(ab / (avg * 1e-3) / 1e9, 1),
                            "hbm_bytes_per_launch": pmc_hbm(name, lps)}
        roof = None
        if kstats:
            dom = max(kstats, key=lambda k: kstats[k]["ms_per_step"])
            ks = kstats[dom]
            ach = ks["achieved_GBps"]
            pk = pmc_all.get(dom, {})
            roof = {"kernel": dom, "bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4) if ach else None,
                    "traffic": ks["hbm_bytes_per_launch"],
                    "traffic_over_algo": (round(ks["hbm_bytes_per_launch"] /
                                                ks["algo_bytes_per_launch"], 3)
                                          if ks["hbm_bytes_per_launch"] and
                                          ks["algo_bytes_per_launch"] else None),
                    "valu_frac": pk.get("valu_frac"), "lds_frac": pk.get("lds_frac"),
                    "pmc_source": os.path.relpath(pmc, ROOT) if pk else None,
                    "algo_bytes_per_launch": ks["algo_bytes_per_launch"],
                    "avg_launch_ms": ks["avg_launch_ms"],
                    "timing": "serial pass (orbg_set_serial), HIP events on the launch stream"}
        fab = (STEREO_FRAME_ALGO_BYTES if args.stereo else
               EXTRACT_FRAME_ALGO_BYTES if args.extract_only else FRAME_ALGO_BYTES)
        if args.extract_only:
            workload = ("configs[1] (C2) synthetic 1241x376, 2000 feat, 8 lvl: ORBextractor "
                        "only (frames [r*B, (r+1)*B) of the sequence, no matching)")
        elif args.stereo:
            workload = ("configs[3] KITTI00-shaped stereo 1241x376 L+R, 2000 feat/eye, 8 lvl: "
                        "ORBextractor x2 + Frame::ComputeStereoMatches (bf=386.1448, "
                        "mb=bf/fx)")
        else:
            workload = ("C3 KITTI03-shaped mono 1241x376, 2000 feat, 8 lvl: ORBextractor + "
                        "Hamming knn2 (t vs t-1) + SearchForInitialization(w=100, 0.9, checkOri)")
            if args.with_pose:
                workload += (" + pose stub (PoseOptimization over the matches, 10 m "
                             "back-projection) gathered with the summary")
        metric = (METRIC_STEREO if args.stereo else METRIC_EXTRACT if args.extract_only else METRIC)
        if args.host_input:
            metric += " -- host-fed (pinned host frames, H2D copies overlapped, PCIe-inclusive)"
        out = {
            "metric": metric, "value": round(value, 2),
            "unit": "stereo frames/s" if args.stereo else "frames/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "ms_per_256_frames": round(elapsed / args.steps * 1e3 * 256 / B, 4),
            "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {
                "workload": workload,
                "frames_per_gpu_per_step": B, "global_batch": B * world, "width": W,
                "pipelined_batches": bool(args.pipeline) and not args.serial,
                "serial_pass_only": bool(args.serial),
                "input_blocks": nblocks,
                "input_reuse": ("none within %d steps: the step cycles through %d resident "
                                "blocks of %.0f MB (%.0f MB in all, > the 256 MB Infinity "
                                "Cache)" % (nblocks, nblocks, nimg * W * H / 1e6,
                                            nblocks * nimg * W * H / 1e6)
                                if nblocks > 1 else "the same resident block every step"),
                "height": H, "nfeatures": NFEAT, "nlevels": NLEV,
                "parallelism": ("frames sharded over %d GPU(s), RCCL all_gather of the "
                                "per-frame outputs per step" % world if collective else
                                "1 GPU, no collective (the gathers run only at world > 1 or "
                                "with --force-collective)")},
            "dist": dist_info,
            "roofline": roof,
            "pipeline_roofline": {"algo_bytes_per_frame": fab,
                                  "achieved_GBps": round(value * fab / 1e9, 1),
                                  "frac": round(value * fab / 1e9 / HBM_PEAK_GBS, 4)},
            "kernels": kstats,
            "host_input": ({"h2d_GBps_alone": round(h2d, 2),
                            "input_bytes_per_frame": W * H,
                            "h2d_bound_frames_per_s": round(h2d * 1e9 / (W * H), 1),
                            "staging": "3 device slots, copy stream, the copy of step k+2 issued "
                                       "once step k-1's outputs are written (host-gated "
                                       "orbg_batch_acquire)"}
                           if args.host_input else None),
            "blur_plan": {"fused_into_fast_cells": blur_plan[0],
                          "interior_px_per_image": blur_plan[1],
                          "border_px_per_image": blur_plan[2]},
            "candidates_per_image": round(ncand / nimg, 1),
            "keypoints_per_image": round(nkp / nimg, 1),
        }
        if world == 1 and not args.no_cpu and args.stereo:
            out["cpu_baseline"] = cpu_baseline_stereo(lefts, rights, args.cpu_threads,
                                                      args.cpu_frames or 32 * args.cpu_threads)
        elif world == 1 and not args.no_cpu and args.extract_only:
            out["cpu_baseline"] = cpu_baseline_extract(frames, args.cpu_threads,
                                                       args.cpu_frames or 256 * args.cpu_threads)
        elif world == 1 and not args.no_cpu:
            n = args.cpu_frames or 256 * args.cpu_threads
            out["cpu_baseline"] = cpu_baseline(frames, args.cpu_threads, n)
        else:
            out["cpu_baseline"] = None
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    if collective:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
