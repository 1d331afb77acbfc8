#!/bin/bash
# Round-2 profile of the bench line: kernel-trace of bench.py (pipelined timed pass + serial
# kernel-timing pass), then PMC passes each in its own run.
#   gpurun --timeout 1200 -- bash tools/r02_profile.sh <tag> [bench args]
set -e -o pipefail
TAG=${1:-r02}
shift || true
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp
export TMPDIR=/tmp
echo "[profile] kernel-trace of bench.py $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu "$@" > "$O/bench.json" 2> "$O/trace.err"
python3 "$R/tools/rocprof_summary.py" "$O/trace/run_kernel_stats.csv" "$O/kernel_stats.md" > /dev/null
python3 "$R/tools/rocprof_phase.py" "$O/trace/run_kernel_trace.csv" "$O/bench.json" "$O/kernel_phase.md"
P1="SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU"
P2="SQ_ACTIVE_INST_VALU SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for P in "$P1" "$P2" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i + 1))
    echo "[profile] pmc pass $i: $P"
    timeout -s KILL 150 rocprofv3 --pmc $P -d "$O/pmc$i" -o run --output-format csv \
        -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu --no-kernel-timing "$@" > "$O/pmc$i.log" 2>&1
done
python3 "$R/tools/pmc_kernels.py" "$O" "$O/pmc_kernels.json"
echo "[profile] done"
