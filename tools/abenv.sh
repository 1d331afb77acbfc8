#!/bin/bash
# Interleaved A/B of runtime settings: each argument is "name:ENV=VAL[,ENV=VAL...]" (or
# "name:" for the defaults), optionally "name:ENV=VAL@variant" to also load lib/<variant>;
# bench.py's pipelined ms_per_step beside the serial per-kernel times.
#   gpurun -- bash tools/abenv.sh <tag> <rounds> <spec> ...
set -e -o pipefail
O=gpurun_out/${1:-abenv}
R=${2:-2}
shift 2
mkdir -p $O
for r in $(seq 1 $R); do
  for spec in "$@"; do
    name=${spec%%:*}; rest=${spec#*:}; var=""
    if [[ "$rest" == *@* ]]; then var=${rest##*@}; rest=${rest%@*}; fi
    envs=$(echo "$rest" | tr ',' ' ')
    env $envs ${var:+ORBG_LIB_VARIANT=$var} timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu > $O/b.json 2> $O/b.err
    echo "$r $name $(python -c 'import json;d=json.load(open("'$O'/b.json"));print(d["ms_per_step"], {k:round(v["ms_per_step"],4) for k,v in d["kernels"].items()})')"
  done
done
