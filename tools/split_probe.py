#!/usr/bin/env python3
"""Developer probe: one 256-frame step (extract + knn2 + SearchForInitialization) split over
K contexts, each on its own stream with B/K frames, launched back to back -- do independent
sub-batches fill the idle CUs of each other's latency-bound phases (resize chain, quadtree)?
Prints ms per 256 frames for each K."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orb_slam2_test_amd import ORBextractor, synthetic as S  # noqa: E402

B, W, H, STEPS = 256, 1241, 376, 20
fr = S.sequence(B, H, W)
d = torch.from_numpy(fr).cuda()


def run(K, match=True):
    n = B // K
    exts, streams = [], []
    for k in range(K):
        e = ORBextractor(2000, 1.2, 8, 20, 7, max_batch=n)
        s = torch.cuda.Stream()
        e.ctx.set_stream(s.cuda_stream)
        exts.append(e)
        streams.append(s)
    f1 = ((np.arange(n) - 1) % n).astype(np.int32)
    f2 = np.arange(n, dtype=np.int32)

    def step():
        for k, e in enumerate(exts):
            e.extract_batch_device(d.data_ptr() + k * n * W * H, n, W, H)
            if match:
                e.match_batch_device(f1, f2, 100, 0.9, True)

    for _ in range(3):
        step()
    for e in exts:
        e.ctx.sync()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(STEPS):
        step()
    for e in exts:
        e.ctx.sync()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / STEPS * 1e3
    print("K=%d match=%d  %.3f ms per 256 frames  (%.0f frames/s)" % (K, match, ms, B / ms * 1e3),
          flush=True)
    for e in exts:
        e.close()


for K in (1, 2, 4):
    run(K, match=False)
    run(K, match=True)
