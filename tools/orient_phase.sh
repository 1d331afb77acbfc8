#!/bin/bash
# k_orient_desc phase split (developer build, make OUT=../lib/dev DEV=1): ORBG_DBG stops every
# wave after a phase -- 21 IC_Angle moments (A), 22 + angle / sincos / keypoint records (B),
# (0: the whole kernel, + rBRIEF C) -- and bench.py's serial pass times orient_desc.  Wrong
# outputs.   gpurun -- bash tools/orient_phase.sh <tag> [variant]
set -e -o pipefail
O=gpurun_out/${1:-orientphase}
V=${2:-dev}
mkdir -p $O
for d in 21 22 0; do
  ORBG_LIB_VARIANT=$V ORBG_DBG=$d timeout -k 10 120 python bench.py --extract-only --steps 20 --warmup 3 --no-cpu > $O/p$d.json 2> $O/p$d.err
  echo "dbg $d orient_desc $(python3 -c 'import json;d=json.load(open("'$O'/p'$d'.json"));print(d["kernels"]["orient_desc"]["ms_per_step"])')"
done
