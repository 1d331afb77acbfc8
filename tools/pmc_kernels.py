#!/usr/bin/env python3
"""Per-kernel PMC summary (profiles/*pmc_kernels.json) from rocprofv3 --pmc passes, each in
its own run directory (tools/profile.sh).  Counters are averaged per dispatch; with the
number of steps the profiled run issued (argument 3, > 0) the per-step sums are given too.
bench.py's roofline prices one launch of its serial pass (orbg_set_serial: one dispatch per
kernel and step, except octree's two by design), so the PMC run is that serial pass
(tools/round_prof.sh) and hbm_bytes_per_launch is directly comparable with
algo_bytes_per_launch.

- hbm_bytes_per_launch = 2 * FETCH_SIZE + WRITE_SIZE (KiB counters; the gfx950 FETCH_SIZE
  halving of MI355X_MICROARCH.md 'HBM'; Infinity-Cache hits count as fetched).
- SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_* are quad-cycles summed over waves; the
  wait/active fractions are of SQ_WAVE_CYCLES.
- cycles = GRBM_GUI_ACTIVE / 8 (summed over the 8 XCDs): the dispatch's GPU cycles.
- valu_frac = 2 * SQ_INSTS_VALU / (1024 SIMDs * cycles): fraction of the chip's VALU issue
  capacity (one wave64 instruction per SIMD per 2 cycles).
- lds_frac = SQ_LDS_IDX_ACTIVE / (256 CUs * cycles): fraction of the LDS array cycles.
- mfma_frac = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs * cycles).

usage: pmc_kernels.py <dir with pmc*/run_counter_collection.csv> <out.json> [steps]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kernel_keys import key  # noqa: E402


def main(d, out, steps="0"):
    steps = int(steps)
    acc = defaultdict(lambda: defaultdict(list))
    for path in glob.glob(os.path.join(d, "*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(path)):
            k = key(r["Kernel_Name"])
            if k:
                acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {"_note": __doc__.split("usage:")[0].strip()}
    for k, c in sorted(acc.items()):
        a = {n: sum(v) / len(v) for n, v in c.items()}
        e = {"dispatches": max(len(v) for v in c.values())}
        if "FETCH_SIZE" in a and "WRITE_SIZE" in a:
            e["fetch_size_raw_bytes"] = int(a["FETCH_SIZE"] * 1024)
            e["write_size_bytes"] = int(a["WRITE_SIZE"] * 1024)
            e["hbm_bytes_per_launch"] = int((2 * a["FETCH_SIZE"] + a["WRITE_SIZE"]) * 1024)
            if steps > 0:
                nd = len(c["FETCH_SIZE"])
                e["steps"] = steps
                e["dispatches_per_step"] = round(nd / steps, 3)
                e["hbm_bytes_per_step"] = int((2 * sum(c["FETCH_SIZE"]) + sum(c["WRITE_SIZE"]))
                                              * 1024 / steps)
        wc = a.get("SQ_WAVE_CYCLES")
        if wc:
            for n in ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY"):
                if n in a:
                    e[n.lower().replace("sq_", "") + "_frac"] = round(a[n] / wc, 3)
        if a.get("SQ_WAVES"):
            w = a["SQ_WAVES"]
            e["waves"] = int(w)
            for n in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD"):
                if n in a:
                    e[n.lower().replace("sq_insts_", "") + "_per_wave"] = round(a[n] / w, 1)
        if a.get("SQ_INSTS_LDS"):
            if "SQ_LDS_BANK_CONFLICT" in a:
                e["lds_bank_conflict_cycles_per_lds_instr"] = round(a["SQ_LDS_BANK_CONFLICT"] / a["SQ_INSTS_LDS"], 2)
        cyc = a.get("GRBM_GUI_ACTIVE", 0) / 8
        if cyc > 0:
            e["cycles"] = int(cyc)
            if "SQ_INSTS_VALU" in a:
                e["valu_frac"] = round(2 * a["SQ_INSTS_VALU"] / (1024 * cyc), 4)
            if "SQ_LDS_IDX_ACTIVE" in a:
                e["lds_frac"] = round(a["SQ_LDS_IDX_ACTIVE"] / (256 * cyc), 4)
            if "SQ_VALU_MFMA_BUSY_CYCLES" in a:
                e["mfma_frac"] = round(a["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * cyc), 4)
        e["counters"] = {n: round(v, 1) for n, v in sorted(a.items())}
        res[k] = e
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: {x: v for x, v in e.items() if x != "counters"} for k, e in res.items() if k[0] != "_"}, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
