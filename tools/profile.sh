#!/bin/bash
# Kernel trace + PMC passes of one python workload (bench.py, tools/ba_bench.py, ...):
#   gpurun --timeout 1200 -- bash tools/profile.sh <tag> <script.py> [args]
# 1. rocprofv3 --kernel-trace --stats of `script args` (the committed *_kernel_stats.md,
#    *_kernel_phase.md for bench.py: its pipelined timed pass vs its serial timing pass);
# 2. one rocprofv3 --pmc run per counter group (never combined with tracing) of
#    `script args $PMC_ARGS`.  For bench.py pass PMC_ARGS="--serial --steps 3 --warmup 1
#    --no-kernel-timing": every kernel then runs as one dispatch per step on one stream, so
#    a dispatch is exactly the launch bench.py's roofline prices (PMC_STEPS = 4 steps);
# 3. tools/pmc_kernels.py: per-dispatch and per-step HBM bytes (2 FETCH_SIZE + WRITE_SIZE,
#    the gfx950 correction of MI355X_MICROARCH.md) and the SQ fractions.
set -e -o pipefail
TAG=${1:?tag}
SCRIPT=${2:?script}
shift 2
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp
export TMPDIR=/tmp
echo "[profile] kernel-trace: $SCRIPT $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv \
    -- python3 "$R/$SCRIPT" "$@" > "$O/run.json" 2> "$O/trace.err"
python3 "$R/tools/rocprof_summary.py" "$O/trace/run_kernel_stats.csv" "$O/kernel_stats.md" > /dev/null
if [ "$(basename $SCRIPT)" = bench.py ]; then
    python3 "$R/tools/rocprof_phase.py" "$O/trace/run_kernel_trace.csv" "$O/run.json" "$O/kernel_phase.md"
fi
P1="SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU"
P2="SQ_ACTIVE_INST_VALU SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for P in "$P1" "$P2" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i + 1))
    echo "[profile] pmc pass $i: $P"
    timeout -s KILL 240 rocprofv3 --pmc $P -d "$O/pmc$i" -o run --output-format csv \
        -- python3 "$R/$SCRIPT" "$@" $PMC_ARGS > "$O/pmc$i.log" 2>&1
done
python3 "$R/tools/pmc_kernels.py" "$O" "$O/pmc_kernels.json" ${PMC_STEPS:-0}
echo "[profile] done"
