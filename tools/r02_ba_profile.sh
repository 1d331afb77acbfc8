#!/bin/bash
# BA linearisation (configs[4]) profile: kernel trace + PMC passes of tools/ba_bench.py
set -e -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r02ba}
shift || true
mkdir -p "$O"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv \
    -- python3 "$R/tools/ba_bench.py" --iters 10 --no-cpu "$@" > "$O/ba_bench.json" 2> "$O/trace.err"
python3 "$R/tools/rocprof_summary.py" "$O/trace/run_kernel_stats.csv" "$O/kernel_stats.md" > /dev/null
P1="SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU"
P2="SQ_ACTIVE_INST_VALU SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for P in "$P1" "$P2" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i + 1))
    timeout -s KILL 150 rocprofv3 --pmc $P -d "$O/pmc$i" -o run --output-format csv \
        -- python3 "$R/tools/ba_bench.py" --iters 3 --warmup 1 --no-cpu "$@" > "$O/pmc$i.log" 2>&1
done
python3 "$R/tools/pmc_kernels.py" "$O" "$O/pmc_kernels.json" > /dev/null
cd "$R"
timeout -k 10 300 python3 tools/ba_bench.py "$@" > "$O/ba_bench_plain.json"
cat "$O/ba_bench_plain.json"
