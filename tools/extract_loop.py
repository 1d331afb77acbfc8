#!/usr/bin/env python3
"""Developer driver for profilers: N extractions of a 256-frame batch (no matching), in
this process (rocprofv3 --pmc does not follow the subprocesses of oct_timing.py)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orb_slam2_test_amd import ORBextractor, synthetic as S  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
N = int(sys.argv[2]) if len(sys.argv) > 2 else 4
d = torch.from_numpy(S.sequence(B, 376, 1241, seed=11)).cuda()
e = ORBextractor(2000, 1.2, 8, 20, 7, max_batch=B)
for _ in range(N):
    e.extract_batch_device(d.data_ptr(), B, 1241, 376)
e.ctx.sync()
print("ok")
