#!/bin/bash
# pipelined batches: parity tests, bench A/B, kernel timeline of the pipelined bench
set -e -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r02p}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_extract.py tests/test_gpu_stereo.py tests/test_gpu_errors.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for P in 1 0; do
  timeout -k 10 300 python bench.py --steps 20 --no-cpu --pipeline $P > $O/bench_p$P.json 2> $O/bench_p$P.err
  python3 -c "import json;d=json.load(open('$O/bench_p$P.json'));print('pipeline=$P',d['value'],d['ms_per_step']);print({k:v['ms_per_step'] for k,v in d['kernels'].items()})"
done
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tl -o run --output-format csv -- python3 $R/bench.py --steps 6 --warmup 2 --no-cpu --no-kernel-timing --pipeline 1 > $O/tl_bench.json 2> $O/tl.err
python3 $R/tools/timeline.py $O/tl/run_kernel_trace.csv 2 > $O/timeline.txt
tail -45 $O/timeline.txt
