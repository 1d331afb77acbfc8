"""One rank of bench.py's multi-GPU step (sequence.BenchStep, world > 1), run by
tests/test_gpu_bench_dist.py as a child process: RANK / WORLD_SIZE / MASTER_ADDR /
MASTER_PORT come from the environment, every rank uses cuda:0 (the test box has one GPU), and
the gathers run over gloo on the device tensors (RCCL refuses two ranks on one device).

  python tests/dist_bench_worker.py <mono|stereo> <B> <steps> <out.npz>

The rank builds its blocks exactly as bench.py does (synthetic.bench_block_ranges /
stereo_sequence seeded per rank), runs `steps` BenchSteps pipelined on a caller torch stream,
and writes the last step's gathered outputs.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

W, H = 1241, 376


def main():
    mode, B, steps, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    import torch
    import torch.distributed as dist
    from orb_slam2_test_amd import ORBextractor, sequence, synthetic

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    if mode == "stereo":
        lefts, rights, _ = synthetic.stereo_sequence(B, H, W,
                                                     seed=synthetic.DEFAULT_SEED + 1000 * rank)
        frames = np.empty((2 * B, H, W), np.uint8)
        frames[0::2], frames[1::2] = lefts, rights
    else:
        n_total, ranges = synthetic.bench_block_ranges(B, world, rank, 1)
        frames = synthetic.sequence_blocks(n_total, ranges, H, W)[0]
    d = torch.from_numpy(frames).cuda()
    ext = ORBextractor(2000, 1.2, 8, 20, 7, max_batch=len(frames))
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    ext.ctx.set_stream(stream.cuda_stream)
    ext.ctx.set_pipeline(True)
    bstep = sequence.BenchStep(ext, B, mode, world=world, with_pose=(mode == "mono"))
    for _ in range(steps):
        bstep(d.data_ptr(), W, H)
    ext.ctx.check_errors()
    torch.cuda.synchronize()
    g = bstep.gathered
    res = {}
    if mode == "stereo":
        res["summary"] = g.cpu().numpy()
    else:
        res["summary"] = g[0].cpu().numpy()
        res["m12"] = g[1].cpu().numpy()
        res["pose"] = g[2].cpu().numpy()
    np.savez(out, **res)
    dist.barrier()
    dist.destroy_process_group()
    ext.close()


if __name__ == "__main__":
    main()
