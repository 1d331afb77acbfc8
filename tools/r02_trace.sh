#!/bin/bash
# kernel-trace stats of extract_loop under env variants: bash tools/r02_trace.sh <tag> "ENV=a" "ENV=b" ...
set -e -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r02tr}
shift
mkdir -p $O
cd /tmp
export TMPDIR=/tmp
i=0
for v in "$@"; do
  i=$((i+1))
  env $v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/t$i -o run --output-format csv -- python3 $R/tools/extract_loop.py 256 6 > $O/t$i.log 2>&1
  echo "== $v"
  python3 $R/tools/rocprof_summary.py $O/t$i/run_kernel_stats.csv | head -12
done
