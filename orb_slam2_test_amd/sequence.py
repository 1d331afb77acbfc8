"""Batched-sequence mode: a frame sequence sharded over ranks.

One process per GPU (torch.distributed, RCCL over xGMI between GPUs, gloo in the CPU tests).
Rank r owns the contiguous block [lo, hi) of the sequence.  It extracts that block plus the
frame before it, a 1-frame halo, so every pair (t-1, t) with t in [lo, hi) is matched
locally with no exchange on the data path.  The only collective is one all_gather of the
per-frame trajectory summary: keypoint count, and SearchForInitialization matches of
(t-1, t).

The sequence is cyclic, as in bench.py: frame 0 pairs with frame N-1, so every frame costs
exactly one extraction and one match.

A backend maps a local batch `imgs` [n, h, w] (halo first) to (nkp[n], nmatch[n]) with
nmatch[i] = matches of (i-1, i) for i >= 1.  `GpuBackend` runs liborbg's batched
device entry points (ORBextractor.extract_batch_device / match_batch_device).
"""
import numpy as np


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


def gather_summary(local, world, group=None, sizes=None):
    """all_gather a per-rank int32 tensor of shape [2, m_r] (row 0 keypoints, row 1
    matches) into the global [2, N] summary, in rank (= frame) order.  Ranks may hold
    different m_r, so blocks are padded to the largest before the collective.  Pass
    `sizes` (every rank's m_r) when known to skip the size exchange and its host sync
    (bench.py's fixed per-rank batch)."""
    import torch
    import torch.distributed as dist
    if world == 1:
        return local
    if sizes is None:
        m = torch.tensor([local.shape[1]], dtype=torch.int64, device=local.device)
        st = [torch.zeros_like(m) for _ in range(world)]
        dist.all_gather(st, m, group=group)
        sizes = [int(t.item()) for t in st]
    mx = max(sizes)
    pad = torch.zeros((2, mx), dtype=local.dtype, device=local.device)
    pad[:, :local.shape[1]] = local
    out = [torch.zeros_like(pad) for _ in range(world)]
    dist.all_gather(out, pad, group=group)
    return torch.cat([o[:, :n] for o, n in zip(out, sizes)], dim=1)


def run_sharded(frames, world, rank, backend, group=None, device="cpu"):
    """Process this rank's block of the cyclic sequence `frames` [N, h, w] with `backend`
    and return the gathered global summary as numpy (nkp[N], nmatch[N])."""
    import torch
    n = len(frames)
    lo, hi = shard(n, world, rank)
    idx = local_indices(n, lo, hi)
    if len(idx):
        nkp, nm = backend(np.ascontiguousarray(frames[idx]))
        local = np.stack([np.asarray(nkp, np.int32)[1:], np.asarray(nm, np.int32)[1:]])
    else:
        local = np.zeros((2, 0), np.int32)
    t = torch.from_numpy(local).to(device)
    g = gather_summary(t, world, group)
    g = g.cpu().numpy()
    return g[0], g[1]


class GpuBackend:
    """liborbg batch path: extract all local frames in one launch sequence, then match the
    consecutive pairs (i-1, i) on the device; only the per-frame summary leaves HBM."""

    def __init__(self, extractor, window=100, nnratio=0.9, check_ori=True):
        self.ext = extractor
        self.window, self.nnratio, self.check_ori = window, nnratio, check_ori

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
        self.ext.ctx.batch_summary(summary.data_ptr())
        self.ext.ctx.sync()  # the summary is written on liborbg's match stream
        s = summary.cpu().numpy()
        nkp = s[:n].copy()
        if n > 1:
            nm[1:] = s[n:2 * n - 1]
        return nkp, nm
