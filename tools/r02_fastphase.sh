#!/bin/bash
# serial k_fast2 time per phase (ORBG_DBG stops: 11 window, 14 pretest, 12 scores, 13 NMS,
# 0 full) with ORBG_FAST0=0 (one launch, no concurrent streams)
set -e -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r02fp}
mkdir -p $O
cd /tmp
export TMPDIR=/tmp
for DBG in 11 14 12 13 0; do
  ORBG_DBG=$DBG ORBG_FAST0=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace_d$DBG -o run --output-format csv -- python3 $R/tools/extract_loop.py 256 4 > /dev/null 2>&1
  python3 - $O/trace_d$DBG/run_kernel_stats.csv $DBG <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"].split("(")[0][:30]
    if sys.argv[2] == "0" or "fast" in n:
        print("  dbg=%s %-30s calls %4s avg_us %9.1f" % (sys.argv[2], n, r["Calls"], float(r["AverageNs"])/1e3))
PY
done
