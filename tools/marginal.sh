#!/bin/bash
# Marginal cost of each kernel inside the pipelined step (developer build, make OUT=../lib/dev
# DEV=1): ORBG_SKIP=<name> ORBG_SKIP_AFTER=<warm-up batches> stops issuing that launch after
# warm-up (what-if runs, wrong outputs); bench.py's pipelined ms_per_step with and without.
#   gpurun -- bash tools/marginal.sh <tag> [rounds]
set -e -o pipefail
O=gpurun_out/${1:-marginal}
R=${2:-2}
mkdir -p $O
for r in $(seq 1 $R); do
  for k in none fast_cells orient_desc blur resize octree knn2 init_cands init_resolve; do
    if [ $k = none ]; then S=""; else S="ORBG_SKIP=$k ORBG_SKIP_AFTER=8"; fi
    env $S ORBG_LIB_VARIANT=dev timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu --no-kernel-timing > $O/b.json 2> $O/b.err
    echo "$r $k $(python3 -c 'import json;print(json.load(open("'$O'/b.json"))["ms_per_step"])')"
  done
done
