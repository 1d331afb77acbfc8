#!/bin/bash
# kernel trace of the single-frame drop-in path
set -e -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r02single}
mkdir -p $O
cd /tmp
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/t -o run --output-format csv -- python3 $R/tools/single_frame_bench.py 50 > $O/single.json 2> $O/err.log
python3 $R/tools/rocprof_summary.py $O/t/run_kernel_stats.csv | head -30
python3 - $O/t/run_kernel_trace.csv <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
# one frame's timeline near the end
t = rows[-40:]
t0 = int(t[0]["Start_Timestamp"])
for r in t:
    print("%-34s %8.1f .. %8.1f (%6.1f)" % (r["Kernel_Name"].split("(")[0][:34], (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
PY
