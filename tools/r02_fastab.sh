#!/bin/bash
# k_fast2 vs k_fast_cells: parity, phase timing (ORBG_DBG early exits), bench
set -e -o pipefail
O=gpurun_out/${1:-r02c}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_errors.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for V in 2 1; do
  echo "== ORBG_FAST_V=$V"
  ORBG_FAST_V=$V ORBG_NOMATCH=1 timeout -k 10 300 python tools/oct_timing.py 256 11 14 12 13 0 2>&1 | tee $O/phase_v$V.txt
  ORBG_FAST_V=$V timeout -k 10 300 python bench.py --steps 20 --no-cpu > $O/bench_v$V.json 2> $O/bench_v$V.err
  python3 -c "import json;d=json.load(open('$O/bench_v$V.json'));print(d['value'],d['ms_per_step']);print({k:v['ms_per_step'] for k,v in d['kernels'].items()})"
done
