#!/bin/bash
# Interleaved A/B of library variants on the default bench (ms_per_step per run):
#   gpurun -- bash tools/r02_abv.sh <tag> <rounds> <variant|default> ...
# "default" is the in-tree lib; other names are lib/<variant>/liborbg.so (csrc make OUT=).
set -e -o pipefail
O=gpurun_out/${1:-r02abv}
R=${2:-3}
shift 2
mkdir -p $O
for r in $(seq 1 $R); do
  for v in "$@"; do
    if [ "$v" = default ]; then unset ORBG_LIB_VARIANT; else export ORBG_LIB_VARIANT=$v; fi
    timeout -k 10 120 python bench.py --steps 40 --warmup 5 --no-cpu --no-kernel-timing > $O/b.json 2> $O/b.err
    echo "$r $v $(python -c 'import json;d=json.load(open("'$O'/b.json"));print(d["ms_per_step"], d["value"])')"
  done
done
unset ORBG_LIB_VARIANT
