#!/bin/bash
# k_octree_lds phase split (developer build, make OUT=../lib/dev DEV=1): ORBG_DBG stops every
# (frame, level) after a phase -- 1 candidate count + bucket histogram, 2 + bucket scan and
# scatter, 3 + roots and phase-1 passes, 4 + phase-2 rounds (0: the whole kernel) -- and
# bench.py's serial pass times octree.  Also k_orient_desc's stops (21 after the angle phase,
# 22 after the descriptor phase).  Wrong outputs.
#   gpurun -- bash tools/octree_phase.sh <tag> [variant]
set -e -o pipefail
O=gpurun_out/${1:-octphase}
V=${2:-dev}
mkdir -p $O
for d in 1 2 3 4 0 21 22; do
  ORBG_LIB_VARIANT=$V ORBG_DBG=$d timeout -k 10 120 python bench.py --extract-only --steps 20 --warmup 3 --no-cpu > $O/p$d.json 2> $O/p$d.err
  echo "dbg $d $(python3 -c 'import json;d=json.load(open("'$O'/p'$d'.json"));k=d["kernels"];print(" ".join("%s %.4f"%(n,k[n]["ms_per_step"]) for n in ("octree","octree_big","orient_desc") if n in k))')"
done
