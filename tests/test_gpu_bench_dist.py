"""GPU: bench.py's multi-GPU step (sequence.BenchStep with world = 2) executed for real.

The box has one GPU, so two ranks share cuda:0: the test starts two child processes
(tests/dist_bench_worker.py, RANK 0 / 1) that each build their blocks as bench.py does, run
pipelined BenchSteps with world = 2 and gather over gloo on the device tensors -- the same
gather_summary / gather_rows calls bench.py runs over RCCL on the match stream.  The gathered
outputs must equal the single-process oracle result on the whole sequence:

  mono (C3): per-frame keypoints and SearchForInitialization matches, every vnMatches12 row
     (ORBmatcher.cc:487-631) and the pose/trajectory stub of every frame (PoseOptimization
     over the pair's matches, Optimizer.cc:356-631);
  stereo (C4): per stereo frame the left keypoints and the keypoints with a depth
     (Frame.cc:619-834), ranks seeded as bench.py seeds them.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from orb_slam2_test_amd import sequence, synthetic as S

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W, H = 1241, 376
WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_ranks(mode, B, steps, tmp_path):
    port = _free_port()
    procs, outs = [], []
    for r in range(WORLD):
        out = str(tmp_path / ("%s_rank%d.npz" % (mode, r)))
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(WORLD), LOCAL_RANK="0",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(
            [sys.executable, os.path.join(ROOT, "tests", "dist_bench_worker.py"), mode, str(B),
             str(steps), out], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
        outs.append(out)
    logs = []
    try:
        for p in procs:
            logs.append(p.communicate(timeout=240)[0].decode(errors="replace"))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    for r, p in enumerate(procs):
        assert p.returncode == 0, "rank %d failed:\n%s" % (r, logs[r][-3000:])
    return [dict(np.load(o)) for o in outs]


def test_bench_step_world2_mono_gathers_equal_oracle(oracle, tmp_path):
    B = 12
    got = _run_ranks("mono", B, 3, tmp_path)
    p = oracle.params()
    nkp, nm, rows, poses = [], [], [], []
    for r in range(WORLD):
        n_total, ranges = S.bench_block_ranges(B, WORLD, r, 1)
        block = S.sequence_blocks(n_total, ranges, H, W)[0]
        bk, bm, rk, _, _, rm12 = oracle.frames_full(p, block, nthreads=8, window=100, nnratio=0.9)
        nkp.append(bk[1:])
        nm.append(bm[1:])
        for i in range(B):
            rows.append(rm12[i + 1])
            poses.append(oracle.match_pose(p, rk[i], rk[i + 1], rm12[i + 1], sequence.POSE_CAM,
                                           sequence.POSE_DEPTH))
    nkp, nm = np.concatenate(nkp), np.concatenate(nm)
    for r in range(WORLD):  # every rank holds the same gathered result
        g = got[r]
        assert np.array_equal(g["summary"][0], nkp), r
        assert np.array_equal(g["summary"][1], nm), r
        assert g["m12"].shape[0] == WORLD * B and g["pose"].shape == (WORLD * B, 8)
        for t in range(WORLD * B):
            ref = rows[t]
            assert np.array_equal(g["m12"][t, :len(ref)], ref), (r, t)
            assert (g["m12"][t, len(ref):] == -1).all(), (r, t)
            rn, rq, rt = poses[t]
            assert g["pose"][t, 7] == rn, (r, t)
            assert np.array_equal(g["pose"][t, :4], rq), (r, t)
            assert np.array_equal(g["pose"][t, 4:7], rt), (r, t)
    # (rank 0's halo is the cyclic sequence's last frame: its first pair finds little)
    assert np.median(nm) > 150 and np.median([q[0] for q in poses]) > 100


def test_bench_step_world2_stereo_gathers_equal_oracle(oracle, tmp_path):
    B = 4
    got = _run_ranks("stereo", B, 2, tmp_path)
    p = oracle.params()
    bf, min_z = S.KITTI_BF, S.KITTI_BF / S.KITTI_FX
    ref_k, ref_d = [], []
    for r in range(WORLD):
        lefts, rights, _ = S.stereo_sequence(B, H, W, seed=S.DEFAULT_SEED + 1000 * r)
        for i in range(B):
            rl = oracle.extract(p, lefts[i], with_pyramid=True)
            rr = oracle.extract(p, rights[i], with_pyramid=True)
            _, dp = oracle.stereo_matches(p, rl, rr, W, H, bf, min_z)
            ref_k.append(len(rl["kps"]))
            ref_d.append(int((dp > 0).sum()))
    for r in range(WORLD):
        assert np.array_equal(got[r]["summary"][0], ref_k), r
        assert np.array_equal(got[r]["summary"][1], ref_d), r
    assert min(ref_d) > 100
