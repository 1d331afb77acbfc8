set -e -o pipefail
O=gpurun_out/ab1; mkdir -p $O
echo "[ab] pytest"
timeout -k 10 600 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_match.py tests/test_gpu_stereo.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
echo "[ab] timing"
timeout -k 10 300 python tools/oct_timing.py 256 ${AB_VARIANTS:-0@base 0 0@base 0} > $O/ab.txt 2>&1
cat $O/ab.txt
