#!/bin/bash
# Round-end profiles: kernel trace + serial PMC passes of the mono (C3) and stereo (C4) bench
# lines and of the BA bench (C5), tools/profile.sh each.
#   gpurun --timeout 1200 -- bash tools/round_prof.sh <tag>
set -e -o pipefail
TAG=${1:-r03}
O=gpurun_out/$TAG
mkdir -p $O
SER="--serial --steps 3 --warmup 1 --no-kernel-timing --no-cpu"
echo "[prof] mono"
PMC_ARGS="$SER" PMC_STEPS=4 timeout -k 10 560 bash tools/profile.sh ${TAG}_prof bench.py \
    --steps 10 --warmup 3 --no-cpu > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 1; }
echo "[prof] stereo"
PMC_ARGS="$SER" PMC_STEPS=4 timeout -k 10 560 bash tools/profile.sh ${TAG}_sprof bench.py \
    --stereo --steps 10 --warmup 3 --no-cpu > $O/sprofile.log 2>&1 || { tail -20 $O/sprofile.log; exit 1; }
echo "[prof] done"
