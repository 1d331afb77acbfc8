#!/bin/bash
# HBM traffic per kernel: FETCH_SIZE and WRITE_SIZE passes (each its own run) over bench.py
#   gpurun -- bash tools/r02_traffic.sh <tag> [bench args]
set -e -o pipefail
TAG=${1:-r02t}
shift || true
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp
export TMPDIR=/tmp
i=2
for P in "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i + 1))
    timeout -s KILL 150 rocprofv3 --pmc $P -d "$O/pmc$i" -o run --output-format csv \
        -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu --no-kernel-timing "$@" > "$O/pmc$i.log" 2>&1
done
python3 "$R/tools/pmc_kernels.py" "$O" "$O/pmc_kernels.json" > /dev/null
python3 - "$O/pmc_kernels.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d.items():
    if k[0] != "_" and "hbm_bytes_per_launch" in v:
        print("  %-14s dispatches %3d  hbm MB/launch %8.1f" % (k, v["dispatches"], v["hbm_bytes_per_launch"] / 1e6))
PY
