#!/usr/bin/env python3
"""The host side of one single-frame drop-in iteration: every HIP API call of the host thread
(rocprofv3 --hip-trace) merged with the kernels and copies of the same window (between two
consecutive k_pyramid starts), relative to the first k_pyramid start, plus a per-function sum.
usage: single_frame_api_timeline.py <trace dir> [frame]
"""
import collections
import csv
import os
import sys


def main():
    d = sys.argv[1]
    ev = []
    for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "GPU  " +
                   r["Kernel_Name"].split("(")[0].replace("void ", "").replace("orbg::", "")[:34]))
    p = os.path.join(d, "run_memory_copy_trace.csv")
    if os.path.exists(p):
        for r in csv.DictReader(open(p)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                       "GPU  " + r["Direction"].replace("MEMORY_COPY_", "dma ")))
    api = []
    for r in csv.DictReader(open(os.path.join(d, "run_hip_api_trace.csv"))):
        api.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "host " + r["Function"]))
    starts = sorted(e[0] for e in ev if "k_pyramid" in e[2])
    k = int(sys.argv[2]) if len(sys.argv) > 2 else len(starts) // 2
    t0, t1 = starts[k], starts[k + 1]
    # the window opens at the previous frame's last kernel end, so the image upload's API calls
    # (issued before k_pyramid) are in it
    prev_end = max(e[1] for e in ev if e[1] <= t0)
    lo = min(prev_end, t0)
    win = sorted([e for e in ev + api if lo <= e[0] < t1])
    print("%9s %9s %7s  %s" % ("start_us", "end_us", "dur_us", "what"))
    tot = collections.Counter()
    cnt = collections.Counter()
    for s, e, w in win:
        print("%9.1f %9.1f %7.1f  %s" % ((s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3, w))
        if w.startswith("host"):
            tot[w] += (e - s) / 1e3
            cnt[w] += 1
    print("\nhost API time in the window (%.1f us):" % ((t1 - lo) / 1e3))
    for w, v in tot.most_common():
        print("  %-40s %3d calls %8.1f us" % (w[5:], cnt[w], v))
    print("  %-40s %13.1f us" % ("total", sum(tot.values())))


if __name__ == "__main__":
    main()
