"""A one-rank RCCL run of bench.py's gather path, for tests/test_gpu_rccl.py (child process:
a fresh HIP context and a fresh process group per run).

  python tests/rccl_worker.py <mono|stereo> <B> <steps> <out.npz>

WORLD_SIZE = 1 with MASTER_ADDR / MASTER_PORT from the environment.  The process group is
"nccl" (RCCL on ROCm) bound to cuda:0; sequence.BenchStep(collective=True) runs the same
gather_summary / gather_rows all_gathers as a world > 1 bench step, on liborbg's match stream
(an ExternalStream), and the worker writes both the gathered tensors and the local outputs
they were gathered from.
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

    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    backend = dist.get_backend()
    if mode == "stereo":
        lefts, rights, _ = synthetic.stereo_sequence(B, H, W, seed=synthetic.DEFAULT_SEED)
        frames = np.empty((2 * B, H, W), np.uint8)
        frames[0::2], frames[1::2] = lefts, rights
    else:
        n_total, ranges = synthetic.bench_block_ranges(B, 1, 0, 1)
        frames = synthetic.sequence_blocks(n_total, ranges, H, W)[0]
    d = torch.from_numpy(frames).cuda()
    ext = ORBextractor(2000, 1.2, 8, 20, 7, max_batch=len(frames))
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    ext.ctx.set_stream(stream.cuda_stream)
    ext.ctx.set_pipeline(True)
    bstep = sequence.BenchStep(ext, B, mode, world=1, collective=True)
    res = {}
    for k in range(steps):
        bstep(d.data_ptr(), W, H)
        torch.cuda.synchronize()
        g = bstep.gathered
        if mode == "stereo":
            res["gathered_summary_%d" % k] = g.cpu().numpy()
            res["local_summary_%d" % k] = bstep.ssum.view(2, B).cpu().numpy()
        else:
            res["gathered_summary_%d" % k] = g[0].cpu().numpy()
            res["gathered_m12_%d" % k] = g[1].cpu().numpy()
            res["local_summary_%d" % k] = torch.stack(
                [bstep.summary[1:B + 1], bstep.summary[B + 1:]]).cpu().numpy()
            res["local_m12_%d" % k] = bstep.m12.cpu().numpy()
    ext.ctx.check_errors()
    res["backend"] = np.array(backend)
    np.savez(out, **res)
    dist.barrier()
    dist.destroy_process_group()
    ext.close()


if __name__ == "__main__":
    main()
