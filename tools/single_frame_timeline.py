#!/usr/bin/env python3
"""One frame of the single-frame drop-in path (tools/single_frame_bench.py under rocprofv3
--kernel-trace --memory-copy-trace) as a timeline: every kernel and copy between two
consecutive k_pyramid starts, relative to the first, plus the per-frame totals (kernel busy
time, copy time, launches, idle gaps).  usage: single_frame_timeline.py <trace dir> [frame]
"""
import csv
import os
import sys


def load(d):
    ev = []
    for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                   r["Kernel_Name"].split("(")[0].replace("void ", "").replace("orbg::", ""),
                   r["Stream_Id"], "kernel"))
    p = os.path.join(d, "run_memory_copy_trace.csv")
    if os.path.exists(p):
        for r in csv.DictReader(open(p)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                       r["Direction"].replace("MEMORY_COPY_", "dma "), r["Stream_Id"], "copy"))
    ev.sort()
    return ev


def main():
    d = sys.argv[1]
    ev = load(d)
    starts = [i for i, e in enumerate(ev) if e[2].startswith("k_pyramid")]
    k = int(sys.argv[2]) if len(sys.argv) > 2 else len(starts) // 2
    i0, i1 = starts[k], starts[k + 1]
    # the frame's window starts at the end of the previous frame's last event before k_pyramid
    j0 = i0
    while j0 > 0 and ev[j0 - 1][2].startswith("__amd_rocclr_copyBuffer"):
        j0 -= 1
    t0 = ev[i0][0]
    print("%9s %9s %7s  %-30s %s" % ("start_us", "end_us", "dur_us", "what", "stream"))
    busy = []
    for e in ev[j0:i1]:
        print("%9.1f %9.1f %7.1f  %-30s s%s" % ((e[0] - t0) / 1e3, (e[1] - t0) / 1e3,
                                                (e[1] - e[0]) / 1e3, e[2][:30], e[3]))
        busy.append((e[0], e[1]))
    # union of busy intervals over the period
    period = ev[i1][0] - ev[j0][0]
    busy.sort()
    tot, cur = 0, None
    for a, b in busy:
        if cur is None or a > cur[1]:
            if cur:
                tot += cur[1] - cur[0]
            cur = [a, b]
        else:
            cur[1] = max(cur[1], b)
    if cur:
        tot += cur[1] - cur[0]
    kern = [e for e in ev[j0:i1] if e[4] == "kernel" and not e[2].startswith("__amd")]
    copies = [e for e in ev[j0:i1] if e[4] == "copy" or e[2].startswith("__amd")]
    n = len(starts) - 1
    mean_period = (ev[starts[-1]][0] - ev[starts[0]][0]) / max(n, 1) / 1e3
    print("\nframe period %.1f us (mean over %d frames %.1f us); GPU busy %.1f us (%.0f%%), idle %.1f us"
          % (period / 1e3, n, mean_period, tot / 1e3, 100 * tot / period, (period - tot) / 1e3))
    print("compute kernels %d launches, %.1f us summed; copies / blits %d, %.1f us summed"
          % (len(kern), sum(e[1] - e[0] for e in kern) / 1e3, len(copies),
             sum(e[1] - e[0] for e in copies) / 1e3))


if __name__ == "__main__":
    main()
