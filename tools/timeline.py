#!/usr/bin/env python3
"""Per-step timeline of a rocprofv3 kernel trace (run_kernel_trace.csv) of bench.py: for the
last N steps (a step begins at the first k_resize of level 1 ... heuristics: step boundary =
every 7th k_resize), prints each kernel's start/end relative to the step start (us)."""
import csv
import sys

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"].split("(")[0].replace("orbg::", "").replace("void ", "")
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, r.get("Queue_Id", ""),
                 r.get("Stream_Id", "")))
rows.sort()
# step starts: every 7th k_resize (7 pyramid levels per batch; pipelined batches let the
# next batch's resizes start before this batch's orient_desc)
pyr = [r[0] for r in rows if r[2] == "k_pyramid"]  # one launch per batch (all levels)
starts = pyr if pyr else [s for i, s in enumerate([r[0] for r in rows if r[2] == "k_resize"]) if i % 7 == 0]
nshow = int(sys.argv[2]) if len(sys.argv) > 2 else 2
for k in range(max(0, len(starts) - 1 - nshow), len(starts) - 1):
    t0, t1 = starts[k], starts[k + 1]
    print("step %d: %.1f us" % (k, (t1 - t0) / 1e3))
    for s, e, n, q, st in rows:
        if t0 - 200000 <= s < t1:
            print("   %-22s q=%-3s st=%-3s %8.1f .. %8.1f  (%6.1f)" % (n[:22], q, st, (s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3))
