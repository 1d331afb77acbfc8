#!/bin/bash
# SQ + traffic counters of extract_loop's kernels under one env setting:
#   bash tools/r02_pmc.sh <tag> "ENV=a ENV=b"
set -e -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r02pmc}
V=${2:-X=0}
mkdir -p $O
cd /tmp
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVES"
i=0
for P in "$P1" "$P2" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i + 1))
    env $V timeout -s KILL 120 rocprofv3 --pmc $P -d "$O/pmc$i" -o run --output-format csv \
        -- python3 "$R/tools/extract_loop.py" 256 3 > "$O/pmc$i.log" 2>&1
done
python3 $R/tools/pmc_table.py $O > $O/table.csv
python3 $R/tools/sq_summary.py $O/table.csv
