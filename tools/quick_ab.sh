#!/bin/bash
# Quick check of the working tree on the GPU: the extraction parity tests (-m gpu, bench-step
# and extractor files), then bench.py twice (serial kernel times + pipelined step).
#   gpurun -- bash tools/quick_ab.sh <tag> [pytest -k expr]
set -e -o pipefail
O=gpurun_out/${1:-quick}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_bench_step.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 200 --timeout-method thread ${2:+-k "$2"} > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu > $O/b$r.json 2> $O/b$r.err
  python3 -c 'import json;d=json.load(open("'$O'/b'$r'.json"));print(d["ms_per_step"], {k:round(v["ms_per_step"],4) for k,v in d["kernels"].items()})'
done
