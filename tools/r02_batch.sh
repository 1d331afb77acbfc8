#!/bin/bash
# bench.py ms per 256 frames at several batch sizes (pipelined)
set -e -o pipefail
O=gpurun_out/${1:-r02bs}
shift
mkdir -p $O
for b in "$@"; do
  timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu --no-kernel-timing --batch $b > $O/b.json 2> $O/b.err
  echo "batch $b $(python -c 'import json;d=json.load(open("'$O'/b.json"));print(d["ms_per_step"], d["value"], d["ms_per_step"]*256/'$b')')"
done
