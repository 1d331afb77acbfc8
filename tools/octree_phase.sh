#!/bin/bash
# k_octree_lds phase split at B = 1 (the single-frame drop-in, C++ loop), developer build
# (make OUT=../lib/dev DEV=1): ORBG_DBG stops every level after a phase -- 1 candidate
# histogram, 2 + bucket scan and scatter, 3 + DistributeOctTree's phase-1 passes, 4 + phase-2
# rounds (0: the whole kernel, winners included) -- rocprofv3 kernel stats of each run.
# Wrong outputs by design.
#   gpurun -- bash tools/octree_phase.sh <tag> [variant]
set -e -o pipefail
O=$(pwd)/gpurun_out/${1:-octphase}
V=${2:-dev}
R=$(pwd)
mkdir -p $O
python tools/single_frame_bench.py --write-frames /tmp/sf.raw 16
cd /tmp
export TMPDIR=/tmp
for d in 1 2 3 4 0; do
  ORBG_DBG=$d timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/d$d -o run --output-format csv \
      -- $R/orb_slam2_test_amd/lib/$V/compat_selftest bench 1241 376 /tmp/sf.raw 16 200 2000 > $O/d$d.json 2> $O/d$d.err
  echo "dbg $d $(python3 - $O/d$d/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'k_octree_lds' in r['Name']:
        print('k_octree_lds avg_us %.2f calls %s' % (float(r['AverageNs']) / 1e3, r['Calls']))
PY
)"
done
