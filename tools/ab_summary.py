"""Summarise an A/B job's bench and single-frame outputs: gpurun_out/<tag>_bench_<v>.<r>.json
and <tag>_single_<v>.<r>.json -> value, step ms and the named kernels' serial ms per variant."""
import glob
import json
import sys

tag = sys.argv[1]
kern = sys.argv[2].split(",") if len(sys.argv) > 2 else ["fast_cells", "orient_desc", "octree", "blur"]
for f in sorted(glob.glob("gpurun_out/%s_bench_*.json" % tag)):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(f, "unreadable", e)
        continue
    k = d.get("kernels", {})
    print("%-40s %10.1f %7.4f  %s" % (f.split("/")[-1], d["value"], d["ms_per_step"],
          " ".join("%s %.4f" % (n, k[n]["ms_per_step"]) for n in kern if n in k)))
for f in sorted(glob.glob("gpurun_out/%s_single_*.json" % tag)):
    d = json.load(open(f))
    print("%-40s p50 %.4f extract %.4f match %.4f" % (f.split("/")[-1], d["ms_per_frame"]["p50"],
          d["extract_ms_per_frame"]["p50"], d["match_ms_per_frame"]["p50"]))
