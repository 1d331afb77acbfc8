#!/usr/bin/env python3
"""Per-kernel launch durations of a rocprofv3 kernel trace of bench.py, split into the timed
(pipelined) pass and the serial kernel-timing pass that follows it (bench.py runs the
serial pass last, `steps` steps, so each kernel's last steps x launches_per_step dispatches
are the serial ones).  The serial averages are the ones bench.py's roofline quotes.

usage: rocprof_phase.py <run_kernel_trace.csv> <bench.json> [out.md]
"""
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kernel_keys import key  # noqa: E402


def main(trace, bench, out=None):
    b = json.load(open(bench))
    steps = b["steps"]
    per = defaultdict(list)
    for r in sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"])):
        k = key(r["Kernel_Name"])
        if k:
            per[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    lines = ["| kernel | dispatches | all: avg us | serial pass: dispatches | serial pass: avg us "
             "| bench.py event avg us |", "|---|---|---|---|---|---|"]
    for k, d in sorted(per.items()):
        ks = b.get("kernels", {}).get(k)
        n = int(round(ks["launches_per_step"] * steps)) if ks else 0
        ser = d[-n:] if n else []
        lines.append("| %s | %d | %.2f | %d | %s | %s |" % (
            k, len(d), sum(d) / len(d), len(ser),
            "%.2f" % (sum(ser) / len(ser)) if ser else "-",
            "%.2f" % (ks["avg_launch_ms"] * 1e3) if ks else "-"))
    txt = "\n".join(lines) + "\n"
    if out:
        open(out, "w").write(txt)
    print(txt)


if __name__ == "__main__":
    main(*sys.argv[1:])
