#!/bin/bash
# round-2 GPU check: the whole -m gpu suite, then the bench (A/B of the FAST kernels)
set -e -o pipefail
O=gpurun_out/${1:-r02b}
mkdir -p $O
echo "[gpu] pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
echo "[gpu] bench (k_fast2)"
timeout -k 10 300 python bench.py --steps 20 --no-cpu > $O/bench.json 2> $O/bench.err
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step']);print({k:v['ms_per_step'] for k,v in d['kernels'].items()})"
echo "[gpu] bench (k_fast_cells, ORBG_FAST_V=1)"
ORBG_FAST_V=1 timeout -k 10 300 python bench.py --steps 20 --no-cpu > $O/bench_v1.json 2> $O/bench_v1.err
python3 -c "import json;d=json.load(open('$O/bench_v1.json'));print(d['value'],d['ms_per_step']);print({k:v['ms_per_step'] for k,v in d['kernels'].items()})"
echo "[gpu] oct_timing serial"
ORBG_NOMATCH=1 timeout -k 10 200 python tools/oct_timing.py 256 0 > $O/serial.txt 2>&1 && cat $O/serial.txt
echo "[gpu] done"
