#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats kernel_stats.csv into markdown."""
import csv
import sys


def main(path, out=None, steps=None):
    rows = list(csv.DictReader(open(path)))
    lines = ["| kernel | calls | total ms | avg us | min us | max us | % |", "|---|---|---|---|---|---|---|"]
    for r in rows:
        name = r["Name"].split("(")[0]
        lines.append("| %s | %s | %.3f | %.2f | %.2f | %.2f | %.2f |" % (
            name, r["Calls"], int(r["TotalDurationNs"]) / 1e6, float(r["AverageNs"]) / 1e3,
            int(r["MinNs"]) / 1e3, int(r["MaxNs"]) / 1e3, float(r["Percentage"])))
    txt = "\n".join(lines) + "\n"
    if out:
        open(out, "w").write(txt)
    print(txt)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
