#!/bin/bash
# rocprofv3 of tools/ba_bench.py: kernel-trace summary, then MFMA/VALU counters (own pass)
set -e -o pipefail
R=$(pwd)
O=$R/gpurun_out/ba_prof
mkdir -p "$O"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv \
    -- python3 "$R/tools/ba_bench.py" --no-cpu --iters 10 > "$O/trace.json" 2> "$O/trace.err"
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_BUSY_CU_CYCLES SQ_INSTS_VALU \
    --kernel-trace -d "$O/pmc" -o run --output-format csv \
    -- python3 "$R/tools/ba_bench.py" --no-cpu --iters 3 --warmup 1 > "$O/pmc.json" 2> "$O/pmc.err"
echo "ba_prof ok"
