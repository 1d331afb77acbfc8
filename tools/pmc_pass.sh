#!/bin/bash
# One rocprofv3 PMC pass (kernel-trace only beside it) over a short bench run.
#   bash tools/pmc_pass.sh <outdir-name> <counter> [<counter> ...]
set -e -o pipefail
R=$(pwd)
N=$1
shift
O=$R/gpurun_out/pmc/$N
mkdir -p "$O"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace -d "$O" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu --no-kernel-timing > "$O/bench.json" 2> "$O/err.log"
echo "pass $N ok"
