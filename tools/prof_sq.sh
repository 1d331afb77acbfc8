#!/bin/bash
# Extraction-kernel counters for one gpurun call (extraction alone, 256-frame batches, no
# matching, so every kernel's counters are its own):
#   kernel-trace summary, then two SQ passes (8 SQ counters each: the per-pass limit) and
#   the FETCH_SIZE / WRITE_SIZE passes, each in its own rocprofv3 run.
#   gpurun --timeout 900 -- bash tools/prof_sq.sh <tag>
set -e -o pipefail
TAG=${1:-r02_sq}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp
export TMPDIR=/tmp
echo "[prof_sq] kernel-trace"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv \
    -- python3 "$R/tools/extract_loop.py" 256 6 > "$O/trace.log" 2>&1
P1="SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVES"
i=0
for P in "$P1" "$P2" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i + 1))
    echo "[prof_sq] pmc pass $i: $P"
    timeout -s KILL 120 rocprofv3 --pmc $P -d "$O/pmc$i" -o run --output-format csv \
        -- python3 "$R/tools/extract_loop.py" 256 3 > "$O/pmc$i.log" 2>&1
done
echo "[prof_sq] done"
