#!/bin/bash
# k_fast2 phase split (developer build, make OUT=../lib/dev DEV=1): ORBG_DBG stops every cell
# after a phase -- 11 window staging, 14 + compass pretest, 12 + scoring, 13 + NMS/compaction
# (0: the whole kernel) -- and bench.py's serial pass times fast_cells.  Wrong outputs.
#   gpurun -- bash tools/fast_phase.sh <tag> [variant]
set -e -o pipefail
O=gpurun_out/${1:-fastphase}
V=${2:-dev}
mkdir -p $O
for d in 11 14 12 13 0; do
  ORBG_LIB_VARIANT=$V ORBG_DBG=$d timeout -k 10 120 python bench.py --extract-only --steps 20 --warmup 3 --no-cpu > $O/p$d.json 2> $O/p$d.err
  echo "dbg $d fast_cells $(python3 -c 'import json;d=json.load(open("'$O'/p'$d'.json"));print(d["kernels"]["fast_cells"]["ms_per_step"])')"
done
