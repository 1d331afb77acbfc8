#!/bin/bash
# Interleaved A/B of library variants on the stereo line (bench.py --stereo).
#   gpurun -- bash tools/abst.sh <tag> <rounds> <variant|default> ...
set -e -o pipefail
O=gpurun_out/${1:-abst}
R=${2:-2}
shift 2
mkdir -p $O
for r in $(seq 1 $R); do
  for v in "$@"; do
    if [ "$v" = default ]; then unset ORBG_LIB_VARIANT; else export ORBG_LIB_VARIANT=$v; fi
    timeout -k 10 120 python bench.py --stereo --steps 20 --warmup 4 --no-cpu > $O/b.json 2> $O/b.err
    echo "$r $v $(python -c 'import json;d=json.load(open("'$O'/b.json"));print(d["ms_per_step"], {k:round(v["ms_per_step"],4) for k,v in d["kernels"].items() if k.startswith("stereo")})')"
  done
done
unset ORBG_LIB_VARIANT
