#!/bin/bash
# One gpurun call: GPU parity tests, smoke, bench, rocprofv3 kernel-trace summary and the
# two PMC passes (FETCH_SIZE, WRITE_SIZE in separate runs, kernel-trace only beside them).
# Every GPU step has its own time limit; the script stops at the first failure.
#   gpurun --timeout 1200 -- bash tools/gpu_round.sh <tag> [steps]
set -e -o pipefail
TAG=${1:-r01}
STEPS=${2:-20}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
echo "[gpu_round] pytest -m gpu"
timeout -k 10 600 python -m pytest tests -m gpu -x -q > "$O/pytest_gpu.log" 2>&1
tail -2 "$O/pytest_gpu.log"
echo "[gpu_round] smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
cat "$O/smoke.log"
echo "[gpu_round] bench"
timeout -k 10 500 python bench.py --steps "$STEPS" > "$O/bench.json" 2> "$O/bench.err"
cat "$O/bench.json"
cd /tmp
export TMPDIR=/tmp
echo "[gpu_round] rocprofv3 kernel-trace"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu > "$O/prof_bench.json" 2> "$O/prof.err"
for C in FETCH_SIZE WRITE_SIZE; do
    echo "[gpu_round] rocprofv3 --pmc $C"
    timeout -k 10 400 rocprofv3 --pmc "$C" --kernel-trace -d "$O/pmc_$C" -o run --output-format csv \
        -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu --no-kernel-timing \
        > "$O/pmc_$C.json" 2> "$O/pmc_$C.err"
done
echo "[gpu_round] done"
