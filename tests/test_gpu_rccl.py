"""GPU: the RCCL collective of bench.py's batched-sequence mode, executed on the box's one GPU.

bench.py's gathers (sequence.gather_summary / gather_rows on liborbg's match stream, SURVEY.md
8e) run over RCCL only at world > 1, i.e. only in the driver's multi-GPU runs.  Here a child
process (tests/rccl_worker.py) creates a one-rank "nccl" process group on cuda:0 and runs
BenchStep(collective=True): the same all_gathers, on the same ExternalStream, with the
world == 1 shortcut bypassed.  The gathered tensors must equal the local outputs of every
step, and those must equal the oracle (mono: per-frame keypoints and SearchForInitialization
matches, every vnMatches12 row; stereo: keypoints and depths per stereo frame).
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from orb_slam2_test_amd import synthetic as S

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W, H = 1241, 376


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(mode, B, steps, tmp_path):
    out = str(tmp_path / ("rccl_%s.npz" % mode))
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_free_port()))
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "rccl_worker.py"), mode,
                        str(B), str(steps), out], env=env, stdout=subprocess.PIPE,
                       stderr=subprocess.STDOUT, timeout=240)
    log = p.stdout.decode(errors="replace")
    assert p.returncode == 0, log[-3000:]
    return dict(np.load(out))


def test_rccl_one_rank_mono_gather(oracle, tmp_path):
    B, steps = 8, 2
    r = _run("mono", B, steps, tmp_path)
    assert str(r["backend"]) == "nccl"
    for k in range(steps):
        assert np.array_equal(r["gathered_summary_%d" % k], r["local_summary_%d" % k]), k
        assert np.array_equal(r["gathered_m12_%d" % k], r["local_m12_%d" % k]), k
    p = oracle.params()
    n_total, ranges = S.bench_block_ranges(B, 1, 0, 1)
    block = S.sequence_blocks(n_total, ranges, H, W)[0]
    bk, bm, _, _, _, rm12 = oracle.frames_full(p, block, nthreads=8, window=100, nnratio=0.9)
    g = r["gathered_summary_%d" % (steps - 1)]
    assert np.array_equal(g[0], bk[1:]) and np.array_equal(g[1], bm[1:])
    m12 = r["gathered_m12_%d" % (steps - 1)]
    for t in range(B):
        ref = rm12[t + 1]
        assert np.array_equal(m12[t, :len(ref)], ref) and (m12[t, len(ref):] == -1).all(), t
    assert np.median(bm[1:]) > 150


def test_rccl_one_rank_stereo_gather(oracle, tmp_path):
    B, steps = 4, 2
    r = _run("stereo", B, steps, tmp_path)
    for k in range(steps):
        assert np.array_equal(r["gathered_summary_%d" % k], r["local_summary_%d" % k]), k
    p = oracle.params()
    lefts, rights, _ = S.stereo_sequence(B, H, W, seed=S.DEFAULT_SEED)
    g = r["gathered_summary_%d" % (steps - 1)]
    for i in range(B):
        rl = oracle.extract(p, lefts[i], with_pyramid=True)
        rr = oracle.extract(p, rights[i], with_pyramid=True)
        _, dp = oracle.stereo_matches(p, rl, rr, W, H, S.KITTI_BF, S.KITTI_BF / S.KITTI_FX)
        assert g[0][i] == len(rl["kps"]) and g[1][i] == int((dp > 0).sum()), i
