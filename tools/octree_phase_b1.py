#!/usr/bin/env python3
"""k_octree_lds at B = 1 (the single-frame drop-in): mean duration per launch shape from
rocprofv3 kernel traces of compat_selftest bench, one trace directory per ORBG_DBG phase
stop (tools/octree_phase.sh's stops: 1 count + histogram, 2 + scan / scatter, 3 + phase 1,
4 + phase 2, 0 whole).  usage: octree_phase_b1.py <dir>/<dbg>/... for dbg in 1 2 3 4 0
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def launches(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    out = defaultdict(list)
    for r in csv.DictReader(open(f[0])):
        name = r["Kernel_Name"]
        if "k_octree_lds" not in name:
            continue
        gy = int(r.get("Grid_Size_Y", r.get("Grid_Y", "1")) or 1)
        wg = int(r.get("Workgroup_Size_X", "512") or 512)
        key = "grid_y=%d" % (gy,)
        out[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return out


root = sys.argv[1]
for d in ("1", "2", "3", "4", "0"):
    p = os.path.join(root, d)
    if not os.path.isdir(p):
        continue
    L = launches(p)
    print("dbg %s  " % d + "  ".join("%s: %.1f us (n=%d)" % (k, sorted(v)[len(v) // 2], len(v))
                                     for k, v in sorted(L.items())))
