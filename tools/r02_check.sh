#!/bin/bash
# GPU check: the whole -m gpu suite, then the default bench line
#   gpurun --timeout 900 -- bash tools/r02_check.sh <tag> [bench args]
set -e -o pipefail
O=gpurun_out/${1:-r02c}
shift || true
mkdir -p $O
echo "[gpu] pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
echo "[gpu] bench $*"
timeout -k 10 300 python bench.py --steps 20 "$@" > $O/bench.json 2> $O/bench.err
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step']);print({k:v['ms_per_step'] for k,v in d['kernels'].items()})"
echo "[gpu] done"
