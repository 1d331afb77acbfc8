#!/bin/bash
# bench frames/s at several batch sizes, interleaved: bash tools/r02_batchab.sh <tag> <rounds> <B> ...
set -e -o pipefail
O=gpurun_out/${1:-r02bab}
R=${2:-2}
shift 2
mkdir -p $O
for r in $(seq 1 $R); do
  for b in "$@"; do
    timeout -k 10 120 python bench.py --batch $b --steps 30 --warmup 5 --no-cpu --no-kernel-timing > $O/b.json 2> $O/b.err
    echo "$r B=$b $(python -c 'import json;d=json.load(open("'$O'/b.json"));print(d["ms_per_step"], d["value"])')"
  done
done
