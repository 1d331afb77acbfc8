#!/usr/bin/env python3
"""Per-kernel HBM traffic from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

usage: pmc_traffic.py <FETCH_SIZE counter_collection.csv> <WRITE_SIZE counter_collection.csv> <out.json>

Both counters are reported in KiB per dispatch.  Per MI355X_MICROARCH.md ("HBM"),
FETCH_SIZE on gfx950 counts exactly half of the bytes of wide coalesced streaming reads,
so hbm_bytes_per_launch = 2 * FETCH + WRITE.  The correction is calibrated for
16-B-per-lane loads only, and our kernels also issue byte/dword loads, so the raw
numbers are kept beside the corrected one.
"""
import csv
import json
import sys
from collections import defaultdict

# rocprof kernel name -> bench.py kernel key
NAMES = {
    "k_resize": "resize", "k_fast_cells": "fast_cells", "k_blur": "blur", "k_blur2": "blur", "k_blur2_edge": "blur",
    "k_octree_lds": "octree", "k_octree": "octree_big", "k_orient_desc": "orient_desc",
    "k_knn2_pairs": "knn2", "k_knn2_pairs_i8": "knn2", "k_init_cands_pairs": "init_cands",
    "k_init_resolve_pairs": "init_resolve",
}


def per_kernel(path, counter):
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"].split("(")[0].replace("orbg::", "").strip()
        if name in NAMES:
            acc[NAMES[name]].append(float(r["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in acc.items()}, {k: len(v) for k, v in acc.items()}


def main(fetch_csv, write_csv, out):
    fe, n = per_kernel(fetch_csv, "FETCH_SIZE")
    wr, _ = per_kernel(write_csv, "WRITE_SIZE")
    res = {"_note": ("bytes per launch, averaged over the dispatches of a short bench run; "
                     "hbm_bytes_per_launch = 2 * FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE "
                     "halving, MI355X_MICROARCH.md 'HBM'); Infinity-Cache hits are counted")}
    for k in sorted(fe):
        res[k] = {"dispatches": n[k], "fetch_size_raw_bytes": round(fe[k]),
                  "write_size_bytes": round(wr.get(k, 0.0)),
                  "hbm_bytes_per_launch": round(2 * fe[k] + wr.get(k, 0.0))}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
