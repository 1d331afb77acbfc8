#!/usr/bin/env python3
"""One pipelined bench.py step from a rocprofv3 kernel trace: every dispatch between two
consecutive `resize` (k_pyramid) starts of the timed pass, by stream, relative to the step
start, and each stream's busy time (union of its dispatches) over the step -- which stream's
chain the step waits on.  The timed pass is the trace's dispatches before bench.py's serial
kernel-timing pass (its last `steps` x launches-per-step dispatches per kernel).

usage: pipeline_timeline.py <run_kernel_trace.csv> <bench.json> [step index] [out.txt]
"""
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kernel_keys import key  # noqa: E402


def union(iv):
    tot, cur = 0, None
    for a, b in sorted(iv):
        if cur is None or a > cur[1]:
            if cur:
                tot += cur[1] - cur[0]
            cur = [a, b]
        else:
            cur[1] = max(cur[1], b)
    return tot + (cur[1] - cur[0] if cur else 0)


def main():
    trace, bench = sys.argv[1], sys.argv[2]
    b = json.load(open(bench))
    steps = b["steps"]
    ev = []
    for r in csv.DictReader(open(trace)):
        k = key(r["Kernel_Name"])
        if k:
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k, r["Stream_Id"]))
    ev.sort()
    # drop the serial pass: each kernel's last steps x launches_per_step dispatches
    serial_n = {k: int(round(v["launches_per_step"] * steps)) for k, v in b.get("kernels", {}).items()}
    cnt = defaultdict(int)
    for e in ev:
        cnt[e[2]] += 1
    seen = defaultdict(int)
    timed = []
    for e in ev:
        seen[e[2]] += 1
        if seen[e[2]] <= cnt[e[2]] - serial_n.get(e[2], 0):
            timed.append(e)
    starts = [i for i, e in enumerate(timed) if e[2] == "resize"]
    k = int(sys.argv[3]) if len(sys.argv) > 3 else len(starts) // 2
    i0, i1 = starts[k], starts[k + 1]
    t0, t1 = timed[i0][0], timed[i1][0]
    # every dispatch overlapping [t0, t1)
    win = [e for e in timed if e[1] > t0 and e[0] < t1]
    lines = ["step %d of %d timed steps: %.1f us" % (k, len(starts), (t1 - t0) / 1e3),
             "%9s %9s %8s  %-14s %s" % ("start_us", "end_us", "dur_us", "kernel", "stream")]
    for e in win:
        lines.append("%9.1f %9.1f %8.1f  %-14s s%s" % ((e[0] - t0) / 1e3, (e[1] - t0) / 1e3,
                                                       (e[1] - e[0]) / 1e3, e[2], e[3]))
    per = defaultdict(list)
    for e in win:
        per[e[3]].append((max(e[0], t0), min(e[1], t1)))
    lines.append("")
    for s, iv in sorted(per.items()):
        ks = sorted({e[2] for e in win if e[3] == s})
        lines.append("stream s%s busy %.1f us of %.1f (%s)" % (s, union(iv) / 1e3, (t1 - t0) / 1e3,
                                                              ", ".join(ks)))
    allv = [iv for v in per.values() for iv in v]
    lines.append("any stream busy %.1f us" % (union(allv) / 1e3))
    txt = "\n".join(lines) + "\n"
    if len(sys.argv) > 4:
        open(sys.argv[4], "w").write(txt)
    print(txt)


if __name__ == "__main__":
    main()
