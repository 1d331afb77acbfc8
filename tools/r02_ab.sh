#!/bin/bash
# bench.py A/B under env variants (ms_per_step, frames/s): bash tools/r02_ab.sh <tag> "ENV=a" ...
set -e -o pipefail
O=gpurun_out/${1:-r02ab}
shift
mkdir -p $O
for v in "$@"; do
  env $v timeout -k 10 120 python bench.py --steps 40 --warmup 5 --no-cpu --no-kernel-timing > $O/b.json 2> $O/b.err
  echo "$v $(python -c 'import json;d=json.load(open("'$O'/b.json"));print(d["ms_per_step"], d["value"])')"
done
