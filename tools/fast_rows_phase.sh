#!/bin/bash
# k_fast_rows phase split (developer build, make OUT=../lib/dev DEV=1): ORBG_DBG stops every
# strip after a phase -- 31 window rows (loads + LDS ring), 32 + pretest, 33 + scoring, 34 + NMS
# (0: the whole kernel) -- and bench.py's serial pass times fast_cells.  Wrong outputs.  The last
# line is k_fast2 (ORBG_FAST_ROWS=0) on the product library for comparison.
#   gpurun -- bash tools/fast_rows_phase.sh <tag> [variant]
set -e -o pipefail
O=gpurun_out/${1:-frphase}
V=${2:-dev}
mkdir -p $O
for d in 31 32 33 34 0; do
  ORBG_FAST_ROWS=1 ORBG_LIB_VARIANT=$V ORBG_DBG=$d timeout -k 10 120 python bench.py --extract-only --steps 20 --warmup 3 --no-cpu > $O/p$d.json 2> $O/p$d.err
  echo "dbg $d fast_cells $(python3 -c 'import json;d=json.load(open("'$O'/p'$d'.json"));print(d["kernels"]["fast_cells"]["ms_per_step"])')"
done
ORBG_FAST_ROWS=0 timeout -k 10 120 python bench.py --extract-only --steps 20 --warmup 3 --no-cpu > $O/old.json 2> $O/old.err
echo "k_fast2 fast_cells $(python3 -c 'import json;d=json.load(open("'$O'/old.json"));print(d["kernels"]["fast_cells"]["ms_per_step"], d["ms_per_step"])')"
ORBG_FAST_ROWS=1 timeout -k 10 120 python bench.py --extract-only --steps 20 --warmup 3 --no-cpu > $O/new.json 2> $O/new.err
echo "k_fast_rows fast_cells $(python3 -c 'import json;d=json.load(open("'$O'/new.json"));print(d["kernels"]["fast_cells"]["ms_per_step"], d["ms_per_step"])')"
