"""CPU, multi-process: the batched-sequence sharding (orb_slam2_test_amd/sequence.py) over a
gloo process group, world_size 2 and 3, against one process doing the whole sequence.

Each rank runs the oracle on its block plus its 1-frame halo; the gathered trajectory
summary (keypoints per frame, SearchForInitialization matches of (t-1, t)) must equal the
single-process result frame for frame.  The same shard/gather functions drive the GPU path
(GpuBackend; tests/test_gpu_match.py::test_sharded_sequence_gpu) and bench.py's gather.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from orb_slam2_test_amd import sequence, synthetic

H, W, NF = 240, 320, 7


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, frames, q):
    import torch.distributed as dist
    from oracle import pyoracle as O
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        p = O.params(nfeatures=500)

        def backend(imgs):
            return O.frames_batch(p, imgs, nthreads=1, window=100, nnratio=0.9)

        nkp, nm = sequence.run_sharded(frames, world, rank, backend)
        q.put((rank, nkp.tolist(), nm.tolist()))
    finally:
        dist.destroy_process_group()


def test_shard_partition():
    for n in (1, 7, 256):
        for world in (1, 2, 3, 8):
            blocks = [sequence.shard(n, world, r) for r in range(world)]
            assert blocks[0][0] == 0 and blocks[-1][1] == n
            for (a, b), (c, d) in zip(blocks, blocks[1:]):
                assert b == c
            sizes = [b - a for a, b in blocks]
            assert max(sizes) - min(sizes) <= 1
    assert list(sequence.local_indices(10, 0, 3)) == [9, 0, 1, 2]
    assert list(sequence.local_indices(10, 4, 7)) == [3, 4, 5, 6]
    assert len(sequence.local_indices(10, 5, 5)) == 0


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_sequence_matches_single_process(oracle, world):
    frames = synthetic.sequence(NF, H, W, seed=synthetic.DEFAULT_SEED + 5)
    p = oracle.params(nfeatures=500)
    ref_nkp, ref_nm = oracle.frames_batch(p, frames, nthreads=1, window=100, nnratio=0.9)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, frames, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    for rank, nkp, nm in res:
        assert np.array_equal(nkp, ref_nkp), rank
        assert np.array_equal(nm, ref_nm), rank
