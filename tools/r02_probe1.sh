#!/bin/bash
# round-2 first GPU call: new error-path tests, bench, sub-batch split probe, SQ counters
set -e -o pipefail
O=gpurun_out/r02a
mkdir -p $O
echo "[r02a] pytest errors"
timeout -k 10 300 python -u -m pytest tests/test_gpu_errors.py -x -v --timeout 120 --timeout-method thread > $O/pytest_err.log 2>&1 || { tail -40 $O/pytest_err.log; exit 1; }
tail -3 $O/pytest_err.log
echo "[r02a] bench"
timeout -k 10 300 python bench.py --steps 20 --no-cpu > $O/bench.json 2> $O/bench.err
cat $O/bench.json | head -c 600; echo
echo "[r02a] split probe"
timeout -k 10 300 python tools/split_probe.py > $O/split.log 2>&1
cat $O/split.log
echo "[r02a] prof_sq"
bash tools/prof_sq.sh r02a_sq
echo "[r02a] done"
