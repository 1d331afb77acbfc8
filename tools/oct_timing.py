#!/usr/bin/env python3
"""Developer timing of the batch pipeline under ORBG_DBG variants (subprocess per variant)."""
import os
import subprocess
import sys

CODE = r'''
import sys, time, numpy as np, torch
sys.path.insert(0, ".")
import os
import orb_slam2_test_amd._lib as _L
if os.environ.get("ORBG_VARIANT"):  # developer A/B: a liborbg.so built into lib/<variant>/
    _L.LIB_PATH = os.path.join(os.path.dirname(_L.LIB_PATH), os.environ["ORBG_VARIANT"], "liborbg.so")
from orb_slam2_test_amd import ORBextractor, synthetic as S
B = int(sys.argv[1])
fr = S.sequence(B, 376, 1241, seed=11)
d = torch.from_numpy(fr).cuda()
e = ORBextractor(2000, 1.2, 8, 20, 7, max_batch=B)
f1 = (np.arange(B) - 1) % B; f2 = np.arange(B)
M = not os.environ.get("ORBG_NOMATCH")  # extraction alone: kernel times without overlap
for _ in range(3):
    e.extract_batch_device(d.data_ptr(), B, 1241, 376)
    if M: e.match_batch_device(f1, f2)
e.ctx.sync(); e.ctx.profile(True); e.ctx.profile_reset()
for _ in range(5):
    e.extract_batch_device(d.data_ptr(), B, 1241, 376)
    if M: e.match_batch_device(f1, f2)
e.ctx.sync()
print(" ".join("%s=%.3f" % (k, v[0] / 5) for k, v in e.ctx.profile_read().items()))
'''
B = sys.argv[1] if len(sys.argv) > 1 else "256"
for dbg in sys.argv[2:] or ["0"]:
    # "<dbg>" or "<dbg>@<variant>" (variant = subdirectory of orb_slam2_test_amd/lib)
    d, _, var = dbg.partition("@")
    env = dict(os.environ, ORBG_DBG=d, ORBG_VARIANT=var)
    out = subprocess.run([sys.executable, "-c", CODE, B], env=env, capture_output=True, text=True)
    print("ORBG_DBG=%s B=%s: %s %s" % (dbg, B, out.stdout.strip(), out.stderr.strip()[-300:] if out.returncode else ""))
