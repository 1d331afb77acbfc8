#!/bin/bash
# k_pyramid: parity (extract + stereo levels), A/B against the k_resize chain, serial times
set -e -o pipefail
O=gpurun_out/${1:-r02pyr}
mkdir -p $O
echo "[pyr] pytest extract"
timeout -k 10 400 python -u -m pytest tests/test_gpu_extract.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in ORBG_PYR=1 ORBG_PYR=0 "ORBG_PYR=1 ORBG_PYR_NB=2" "ORBG_PYR=1 ORBG_PYR_NB=8"; do
  env $v timeout -k 10 120 python bench.py --steps 40 --warmup 5 --no-cpu --no-kernel-timing > $O/b.json 2> $O/b.err
  echo "$v $(python -c 'import json;d=json.load(open("'$O'/b.json"));print(d["ms_per_step"], d["value"])')"
done
for v in ORBG_PYR=1 ORBG_PYR=0; do
  env $v ORBG_NOMATCH=1 ORBG_FAST0=0 timeout -k 10 200 python tools/oct_timing.py 256 0 > $O/serial.txt 2>&1
  echo "serial $v: $(cat $O/serial.txt)"
done
