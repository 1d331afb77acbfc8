"""Batched-sequence mode: a frame sequence sharded over ranks.

One process per GPU (torch.distributed, RCCL over xGMI between GPUs, gloo in the CPU tests).
Rank r owns the contiguous block [lo, hi) of the sequence.  It extracts that block plus the
frame before it, a 1-frame halo, so every pair (t-1, t) with t in [lo, hi) is matched
locally with no exchange on the data path.  The only collectives are all_gathers of the
per-frame outputs: the trajectory summary (keypoint count, and
SearchForInitialization matches of (t-1, t)) and, with `with_matches`, the match indices
themselves: row t = vnMatches12 of (t-1, t) (ORBmatcher.cc:487-631), frame_cap int32, -1
where keypoint i of frame t-1 has no match.

The sequence is cyclic, as in bench.py: frame 0 pairs with frame N-1, so every frame costs
exactly one extraction and one match.

A backend maps a local batch `imgs` [n, h, w] (halo first) to (nkp[n], nmatch[n]) with
nmatch[i] = matches of (i-1, i) for i >= 1, with `with_matches` also m12[n, cap] with
row i = vnMatches12 of (i-1, i) (row 0 unused), and with `with_pose` also pose[n, 8]: row i
= the pose stub of frame i (PoseOptimization over the matches of (i-1, i), frame i-1's
keypoints back-projected at POSE_DEPTH: SE3Quat q (x, y, z, w), t, inlier count; row 0
unused) -- the "pose/trajectory stub" SURVEY.md 8e gathers beside the counts and indices.
`GpuBackend` runs liborbg's batched device entry points (ORBextractor.extract_batch_device /
match_batch_device / match_pose_batch_device).
"""
import numpy as np

# the pose stub's scene depth (m) and camera (KITTI00-02.yaml intrinsics, mbf)
POSE_DEPTH = 10.0
POSE_CAM = (718.856, 718.856, 607.1928, 185.2157, 386.1448)


def shard(nframes, world, rank):
    """Contiguous block [lo, hi) of rank `rank` (sizes differ by at most one)."""
    if not 0 <= rank < world:
        raise ValueError("rank %d of %d" % (rank, world))
    return nframes * rank // world, nframes * (rank + 1) // world


def local_indices(nframes, lo, hi):
    """Global frame indices a rank extracts: the halo (lo-1, cyclic) then [lo, hi)."""
    if hi <= lo:
        return np.zeros(0, np.int64)
    return np.concatenate([[(lo - 1) % nframes], np.arange(lo, hi)]).astype(np.int64)


class PendingGather:
    """An all_gather in flight (async_op=True) on the process group's own stream: the stream
    that issued it does not wait for it, so the next step's kernels on that stream are not
    held behind the collective.  result() orders the current stream after the collective and
    returns the rows in rank order (cast back to `dtype` when they travelled narrowed)."""

    def __init__(self, work, out, sizes, dtype=None, wire_view=None):
        self.work, self.out, self.sizes, self.dtype = work, out, sizes, dtype
        self.wire_view = wire_view
        self._res = None

    def result(self):
        import torch
        if self._res is None:
            if self.work is not None:
                self.work.wait()
                self.work = None
            r = torch.cat([o[:n] for o, n in zip(self.out, self.sizes)], dim=0)
            if self.wire_view is not None:  # bytes on the wire -> the narrowed dtype
                r = r.view(self.wire_view)
            self._res = r if self.dtype is None else r.to(self.dtype)
            self.out = None
        return self._res


def gather_rows(local, world, group=None, sizes=None, force=False, async_op=False,
                wire_dtype=None):
    """all_gather a per-rank tensor whose dim 0 holds m_r frames into the global tensor, in
    rank (= frame) order.  Ranks may hold different m_r, so blocks are padded to the largest
    before the collective.  Pass `sizes` (every rank's m_r) when known to skip the size
    exchange and its host sync (bench.py's fixed per-rank batch).  At world 1 the local
    tensor is returned with no collective unless `force` (bench.py --force-collective and
    tests/test_gpu_rccl.py run the RCCL path on a one-rank group)."""
    import torch
    import torch.distributed as dist
    if world == 1 and not force:
        return PendingGather(None, [local], [local.shape[0]]) if async_op else local
    if sizes is None:
        m = torch.tensor([local.shape[0]], dtype=torch.int64, device=local.device)
        st = [torch.zeros_like(m) for _ in range(world)]
        dist.all_gather(st, m, group=group)
        sizes = [int(t.item()) for t in st]
    mx = max(sizes)
    wd = local.dtype if wire_dtype is None else wire_dtype
    if mx == local.shape[0]:  # the common case (bench.py's fixed batch): one copy / cast
        pad = local.to(wd, copy=True)
    else:
        pad = torch.zeros((mx,) + tuple(local.shape[1:]), dtype=wd, device=local.device)
        pad[:local.shape[0]] = local
    # RCCL has no 16-bit integer collectives: a narrowed tensor travels as its bytes
    view = wd if wd in (torch.int16, torch.uint16) else None
    if view is not None:
        pad = pad.view(torch.uint8)
    out = [torch.empty_like(pad) for _ in range(world)]
    work = dist.all_gather(out, pad, group=group, async_op=async_op)
    res = PendingGather(work if async_op else None, out, sizes,
                        None if wd == local.dtype else local.dtype, view)
    return res if async_op else res.result()


def gather_summary(local, world, group=None, sizes=None, force=False):
    """all_gather a per-rank int32 tensor of shape [2, m_r] (row 0 keypoints, row 1
    matches) into the global [2, N] summary (gather_rows along the frame axis)."""
    if world == 1 and not force:
        return local
    return gather_rows(local.t().contiguous(), world, group, sizes, force).t().contiguous()


class _PendingT:
    """A PendingGather of a transposed [2, m] summary, transposed back on result()."""

    def __init__(self, p):
        self.p = p

    def result(self):
        return self.p.result().t().contiguous()


def run_sharded(frames, world, rank, backend, group=None, device="cpu", with_matches=False,
                with_pose=False):
    """Process this rank's block of the cyclic sequence `frames` [N, h, w] with `backend`
    and return the gathered global outputs as numpy: (nkp[N], nmatch[N]), then m12[N, cap]
    (row t = vnMatches12 of (t-1, t)) with `with_matches`, then pose[N, 8] (row t = frame t's
    pose stub) with `with_pose`."""
    import torch
    n = len(frames)
    lo, hi = shard(n, world, rank)
    idx = local_indices(n, lo, hi)
    m12 = pose = None
    if len(idx):
        r = backend(np.ascontiguousarray(frames[idx]))
        nkp, nm = r[0], r[1]
        local = np.stack([np.asarray(nkp, np.int32)[1:], np.asarray(nm, np.int32)[1:]])
        k = 2
        if with_matches:
            m12 = np.ascontiguousarray(np.asarray(r[k], np.int32)[1:])
            k += 1
        if with_pose:
            pose = np.ascontiguousarray(np.asarray(r[k], np.float64)[1:])
    else:
        local = np.zeros((2, 0), np.int32)
        pose = np.zeros((0, 8))
    g = gather_summary(torch.from_numpy(local).to(device), world, group).cpu().numpy()
    out = [g[0], g[1]]
    if with_matches:
        if m12 is None:  # an empty block still takes part in the collectives
            cap = torch.zeros(1, dtype=torch.int64, device=device)
            if world > 1:
                import torch.distributed as dist
                dist.all_reduce(cap, op=dist.ReduceOp.MAX, group=group)
            m12 = np.zeros((0, int(cap.item())), np.int32)
        elif world > 1:
            import torch.distributed as dist
            cap = torch.tensor([m12.shape[1]], dtype=torch.int64, device=device)
            dist.all_reduce(cap, op=dist.ReduceOp.MAX, group=group)
            if int(cap.item()) > m12.shape[1]:  # rows padded with -1 to the widest rank's cap
                m12 = np.pad(m12, ((0, 0), (0, int(cap.item()) - m12.shape[1])), constant_values=-1)
        out.append(gather_rows(torch.from_numpy(m12).to(device), world, group).cpu().numpy())
    if with_pose:
        out.append(gather_rows(torch.from_numpy(pose).to(device), world, group).cpu().numpy())
    return tuple(out)


def run_sharded_stereo(lefts, rights, world, rank, backend, group=None, device="cpu"):
    """Stereo frames shard with L and R of a frame on the same rank (the stereo Frame
    constructor extracts both, Frame.cc:110-113, then ComputeStereoMatches :619-834): rank r
    owns stereo frames [lo, hi), no halo (stereo frames are independent).  `backend` maps
    (lefts[n], rights[n]) to (nkp_left[n], ndepth[n]); returns the gathered global
    (nkp_left[N], ndepth[N]) as numpy."""
    import torch
    n = len(lefts)
    lo, hi = shard(n, world, rank)
    if hi > lo:
        nkp, nd = backend(np.ascontiguousarray(lefts[lo:hi]), np.ascontiguousarray(rights[lo:hi]))
        local = np.stack([np.asarray(nkp, np.int32), np.asarray(nd, np.int32)])
    else:
        local = np.zeros((2, 0), np.int32)
    g = gather_summary(torch.from_numpy(local).to(device), world, group).cpu().numpy()
    return g[0], g[1]


class GpuBackend:
    """liborbg batch path: extract all local frames in one launch sequence, then match the
    consecutive pairs (i-1, i) on the device (and with `with_pose` run the pose stub on
    them); only the per-frame outputs leave HBM."""

    def __init__(self, extractor, window=100, nnratio=0.9, check_ori=True, with_matches=False,
                 with_pose=False):
        self.ext = extractor
        self.window, self.nnratio, self.check_ori = window, nnratio, check_ori
        self.with_matches, self.with_pose = with_matches, with_pose

    def __call__(self, imgs):
        import torch
        n, h, w = imgs.shape
        # upload, kernels and the summary read-back all on one (non-null) torch stream
        if not hasattr(self, "_stream"):
            self._stream = torch.cuda.Stream()
            self.ext.ctx.set_stream(self._stream.cuda_stream)
        with torch.cuda.stream(self._stream):
            return self._run(imgs)

    def _run(self, imgs):
        import torch
        n, h, w = imgs.shape
        d = torch.from_numpy(np.ascontiguousarray(imgs)).to("cuda")
        self.ext.extract_batch_device(d.data_ptr(), n, w, h)
        nm = np.zeros(n, np.int32)
        summary = torch.zeros(2 * n, dtype=torch.int32, device="cuda")
        if n > 1:
            self.ext.match_batch_device(np.arange(n - 1), np.arange(1, n), self.window,
                                        self.nnratio, self.check_ori)
        if self.with_pose and n > 1:
            dq = torch.zeros((n - 1, 4), dtype=torch.float64, device="cuda")
            dt = torch.zeros((n - 1, 3), dtype=torch.float64, device="cuda")
            dn = torch.zeros(n - 1, dtype=torch.int32, device="cuda")
            self.ext.match_pose_batch_device(POSE_CAM, POSE_DEPTH, dq.data_ptr(), dt.data_ptr(),
                                             dn.data_ptr())
        self.ext.ctx.batch_summary(summary.data_ptr())
        if self.with_matches:
            cap = self.ext.ctx.batch_matches(None) if n > 1 else 0
            dm = torch.full((n, max(cap, 1)), -1, dtype=torch.int32, device="cuda")
            if n > 1:
                self.ext.ctx.batch_matches(dm[1:].data_ptr())
        self.ext.ctx.sync()  # the summary / matches / poses are written on the match stream
        s = summary.cpu().numpy()
        nkp = s[:n].copy()
        if n > 1:
            nm[1:] = s[n:2 * n - 1]
        out = [nkp, nm]
        if self.with_matches:
            out.append(dm.cpu().numpy())
        if self.with_pose:
            pose = np.zeros((n, 8))
            if n > 1:
                pose[1:, :4] = dq.cpu().numpy()
                pose[1:, 4:7] = dt.cpu().numpy()
                pose[1:, 7] = dn.cpu().numpy()
            out.append(pose)
        return tuple(out)


# bench.py's per-GPU batch per step (frames; stereo: L/R pairs), measured best on MI355X:
# mono 1024 frames (+2.5% frames/s over 512, -1% at 2048), stereo 512 pairs (+3% over 256)
BENCH_BATCH = {"mono": 1024, "extract": 1024, "stereo": 512}


class BenchStep:
    """One step of the batched-sequence mode on one rank, exactly as bench.py times it.

    mode "mono" (C3): ORBextractor on the B + 1 resident frames of a block (halo first),
    then knn2 + SearchForInitialization(window, nnratio, checkOri) of the B pairs (i, i + 1)
    (ORBmatcher.cc:487-631), the per-frame summary (keypoints of frames 1..B, matches of the
    pairs) and the vnMatches12 rows, all on liborbg's match stream, and with world > 1
    their RCCL all_gathers there.
    mode "extract" (C2): ORBextractor on the B frames of a block only.
    mode "stereo" (C4): ORBextractor on B left/right pairs (2B images, L and R
    interleaved), Frame::ComputeStereoMatches of every pair (Frame.cc:619-834), the stereo
    summary on the match stream and its all_gather.

    `with_pose` (mono): also the pose/trajectory stub of every pair (orbg_match_pose_batch_device,
    PoseOptimization over the pair's matches, Optimizer.cc:356-631) into `pose` [B, 8] = (q
    x y z w, t, inliers), gathered beside the summary and the rows with world > 1 (SURVEY.md
    8e's third per-frame payload, as run_sharded(with_pose=True)).  BASELINE.json's headline
    metric is extract + match, so bench.py times it without the stub by default
    (`bench.py --with-pose` times the full sequence step).

    `group` is the process group of the gathers (None: the default group; the 2-process
    one-GPU tests run them over gloo).  The gathers run when world > 1, or with
    `collective=True` at any world size (a one-rank RCCL group: bench.py
    --force-collective, tests/test_gpu_rccl.py).

    `capture(step)`, when set (tests), runs on the match stream after the step's outputs
    are written (orbg_batch_acquire) and before liborbg may reuse them
    (orbg_batch_release); the bench leaves it unset."""

    def __init__(self, ext, B, mode="mono", world=1, window=100, nnratio=0.9, check_ori=True,
                 bf=None, min_z=None, with_pose=False, group=None, collective=None):
        import torch
        from . import synthetic
        if mode not in ("mono", "extract", "stereo"):
            raise ValueError(mode)
        self.ext, self.B, self.mode, self.world = ext, B, mode, world
        self.window, self.nnratio, self.check_ori = window, nnratio, check_ori
        self.bf = synthetic.KITTI_BF if bf is None else bf
        self.min_z = synthetic.KITTI_BF / synthetic.KITTI_FX if min_z is None else min_z
        self.nimg = {"mono": B + 1, "extract": B, "stereo": 2 * B}[mode]
        self.f1 = np.arange(B, dtype=np.int32)        # local frame i (0 = the halo) ...
        self.f2 = np.arange(1, B + 1, dtype=np.int32)  # ... matched to frame i + 1
        self.sl, self.sr = np.arange(B, dtype=np.int32) * 2, np.arange(B, dtype=np.int32) * 2 + 1
        self.summary = torch.zeros(2 * B + 1, dtype=torch.int32, device="cuda")
        self.ssum = torch.zeros(2 * B, dtype=torch.int32, device="cuda")
        self.m12 = None
        self.with_pose = with_pose and mode == "mono"
        self.group = group
        self.collective = world > 1 if collective is None else bool(collective)
        # the gathers run async on the process group's stream (the match stream does not wait
        # for them) and the vnMatches12 rows travel as int16 (indices < frame_cap <= 32767):
        # ORBG_GATHER=sync32 restores round 4's blocking int32 gathers (A/B)
        import os
        self.gather_async = os.environ.get("ORBG_GATHER", "async16") != "sync32"
        self._pending = None
        if self.with_pose:
            self.dq = torch.zeros((B, 4), dtype=torch.float64, device="cuda")
            self.dt = torch.zeros((B, 3), dtype=torch.float64, device="cuda")
            self.dn = torch.zeros(B, dtype=torch.int32, device="cuda")
        self.pose = None
        self.mstream = torch.cuda.ExternalStream(ext.ctx.match_stream())
        self.capture = None
        self._gathered = None

    @property
    def gathered(self):
        """The last step's gathered outputs (stereo: the [2, N] summary; mono: (summary,
        vnMatches12 rows[, pose rows])), waiting for the collectives if they are in flight."""
        import torch
        if self._pending is not None:
            with torch.cuda.stream(self.mstream):
                g = tuple(x.result() for x in self._pending)
            self._gathered = g[0] if self.mode == "stereo" else g
            self._pending = None
        return self._gathered

    def _gather_rows(self, t, wire_dtype=None):
        sizes = [self.B] * self.world
        if not self.gather_async:
            g = gather_rows(t, self.world, self.group, sizes=sizes, force=True)
            return PendingGather(None, [g], [g.shape[0]])
        return gather_rows(t, self.world, self.group, sizes=sizes, force=True, async_op=True,
                           wire_dtype=wire_dtype)

    def _gather_summary(self, t):
        return _PendingT(self._gather_rows(t.t().contiguous()))

    def __call__(self, d_frames_ptr, w, h):
        import torch
        ext, B = self.ext, self.B
        ext.extract_batch_device(d_frames_ptr, self.nimg, w, h)
        if self.mode == "stereo":
            ext.stereo_batch_device(self.sl, self.sr, self.bf, self.min_z)
            ext.ctx.stereo_summary(self.ssum.data_ptr())
            if self.collective:  # per-frame (keypoints, depths) of every rank
                with torch.cuda.stream(self.mstream):
                    self._pending = (self._gather_summary(self.ssum.view(2, B)),)
        elif self.mode == "mono":
            ext.match_batch_device(self.f1, self.f2, self.window, self.nnratio, self.check_ori)
            ext.ctx.batch_summary(self.summary.data_ptr())
            if self.m12 is None:
                self.m12 = torch.empty((B, ext.ctx.batch_matches(None)), dtype=torch.int32,
                                       device="cuda")
            ext.ctx.batch_matches(self.m12.data_ptr())  # vnMatches12 rows of the B pairs
            if self.with_pose:  # pose stub of frame i + 1 from the matches of (i, i + 1)
                ext.match_pose_batch_device(POSE_CAM, POSE_DEPTH, self.dq.data_ptr(),
                                            self.dt.data_ptr(), self.dn.data_ptr())
                with torch.cuda.stream(self.mstream):  # written there (orbg.h)
                    self.pose = torch.cat([self.dq, self.dt, self.dn.double()[:, None]], 1)
            if self.collective:
                with torch.cuda.stream(self.mstream):
                    local = torch.stack([self.summary[1:B + 1], self.summary[B + 1:]])
                    g = [self._gather_summary(local),
                         self._gather_rows(self.m12, wire_dtype=torch.int16)]
                    if self.with_pose:
                        g.append(self._gather_rows(self.pose))
                    self._pending = tuple(g)
        if self.capture is not None:
            ext.ctx.batch_acquire(self.mstream.cuda_stream)
            with torch.cuda.stream(self.mstream):
                self.capture(self)
            ext.ctx.batch_release(self.mstream.cuda_stream)
