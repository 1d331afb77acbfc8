#!/bin/bash
# Round-end measurement set, part 2: kernel trace + PMC passes of the mono bench line and of
# the stereo line (tools/r02_profile.sh each).
#   gpurun --timeout 1200 -- bash tools/r02g_prof.sh <tag>
set -e -o pipefail
TAG=${1:-r02g}
O=gpurun_out/$TAG
mkdir -p $O
echo "[prof] mono"
timeout -k 10 560 bash tools/r02_profile.sh ${TAG}_prof > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 1; }
echo "[prof] stereo"
timeout -k 10 560 bash tools/r02_profile.sh ${TAG}_sprof --stereo > $O/sprofile.log 2>&1 || { tail -20 $O/sprofile.log; exit 1; }
echo "[prof] done"
