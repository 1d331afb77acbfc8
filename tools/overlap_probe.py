#!/usr/bin/env python3
"""Developer probe: wall time per 256-frame step of extraction alone, matching alone (on the
last extracted batch) and both as bench.py runs them, to see how much of the matching hides
behind the next batch's extraction."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orb_slam2_test_amd import ORBextractor, synthetic as S  # noqa: E402

B, W, H, K = 256, 1241, 376, 20
fr = S.sequence(B, H, W)
d = torch.from_numpy(fr).cuda()
e = ORBextractor(2000, 1.2, 8, 20, 7, max_batch=B)
st = torch.cuda.Stream()
torch.cuda.set_stream(st)
e.ctx.set_stream(st.cuda_stream)
f1 = ((np.arange(B) - 1) % B).astype(np.int32)
f2 = np.arange(B, dtype=np.int32)
summ = torch.zeros(2 * B, dtype=torch.int32, device="cuda")


def run(name, fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e.ctx.sync()
    t0 = time.perf_counter()
    for _ in range(K):
        fn()
    torch.cuda.synchronize()
    e.ctx.sync()
    print("%-22s %.3f ms/step" % (name, (time.perf_counter() - t0) / K * 1e3), flush=True)


def ext():
    e.extract_batch_device(d.data_ptr(), B, W, H)


def mat():
    e.match_batch_device(f1, f2, 100, 0.9, True)


def both():
    ext()
    mat()
    e.ctx.batch_summary(summ.data_ptr())


run("extract", ext)
run("match (same batch)", mat)
run("extract + match", both)
