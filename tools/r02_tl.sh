#!/bin/bash
# kernel trace of the bench pipeline (timeline per step)
set -e -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r02h}
mkdir -p $O
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tl -o run --output-format csv -- python3 $R/bench.py --steps 6 --warmup 2 --no-cpu --no-kernel-timing > $O/tl_bench.json 2> $O/tl.err
python3 $R/tools/timeline.py $O/tl/run_kernel_trace.csv 2
