# developer A/B of the whole pipeline: bench.py ms_per_step under env variants
# usage: AB_ENV="ORBG_FAST0=0 ORBG_FAST0=1 ..." bash tools/ab_bench.sh
set -e -o pipefail
O=gpurun_out/abb; mkdir -p $O
echo "[ab] pytest"
timeout -k 10 600 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_match.py tests/test_gpu_stereo.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in ${AB_ENV:-X=0}; do
  env $v timeout -k 10 120 python bench.py --steps 40 --warmup 5 --no-cpu --no-kernel-timing > $O/b.json 2> $O/b.err
  echo "$v $(python -c 'import json;d=json.load(open("'$O'/b.json"));print(d["ms_per_step"], d["value"])')"
done
