#!/bin/bash
# Round-end measurement set, part 1 (one gpurun call): the -m gpu suite, every bench line with its
# CPU baseline, the BA / single-frame / C1 benches (part 2, the profiles: tools/round_prof.sh).
#   gpurun --timeout 1200 -- bash tools/round_bench.sh <tag>
set -e -o pipefail
TAG=${1:-r03final}
O=gpurun_out/$TAG
mkdir -p $O
echo "[final] pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
echo "[final] bench (C3 mono)"
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d['cpu_baseline']['value'],d['cpu_baseline']['value_1core'])"
echo "[final] bench --extract-only (C2)"
timeout -k 10 300 python bench.py --extract-only > $O/c2.json 2> $O/c2.err
python3 -c "import json;d=json.load(open('$O/c2.json'));print(d['value'],d['ms_per_step'],d['cpu_baseline']['value'],d['cpu_baseline']['value_1core'])"
echo "[final] bench --stereo (C4)"
timeout -k 10 300 python bench.py --stereo > $O/stereo.json 2> $O/stereo.err
python3 -c "import json;d=json.load(open('$O/stereo.json'));print(d['value'],d['ms_per_step'],d['cpu_baseline']['value'],d['cpu_baseline']['value_1core'])"
echo "[final] bench --host-input (C3 fed from pinned host memory)"
timeout -k 10 300 python bench.py --host-input --no-cpu > $O/host.json 2> $O/host.err
python3 -c "import json;d=json.load(open('$O/host.json'));print(d['value'],d['ms_per_step'],d['host_input'])"
echo "[final] BA (C5)"
timeout -k 10 300 python tools/ba_bench.py > $O/ba.json 2> $O/ba.err
tail -c 400 $O/ba.json
echo "[final] single frame (KITTI, TUM)"
timeout -k 10 200 python tools/single_frame_bench.py 200 > $O/single.jsonl 2> $O/single.err
timeout -k 10 200 python tools/single_frame_bench.py 200 640 480 1000 >> $O/single.jsonl 2>> $O/single.err
echo "[final] single frame, C++ drop-in loop (compat_selftest bench)"
python tools/single_frame_bench.py --write-frames /tmp/sf.raw 16
timeout -k 10 120 orb_slam2_test_amd/lib/compat_selftest bench 1241 376 /tmp/sf.raw 16 500 2000 > $O/single_cpp.json
cat $O/single_cpp.json
echo "[final] SearchByBoW"
timeout -k 10 200 python tools/bow_match_bench.py > $O/bow_match.json 2> $O/bow_match.err
tail -c 300 $O/bow_match.json
echo "[final] Frame / MapPoint geometry"
timeout -k 10 300 python tools/frame_geom_bench.py > $O/frame_geom.jsonl 2> $O/frame_geom.err
echo "[final] LocalMapping matchers"
timeout -k 10 300 python tools/mapping_bench.py > $O/mapping.jsonl 2> $O/mapping.err
echo "[final] Relocalization / LoopClosing matchers"
timeout -k 10 300 python tools/loop_bench.py > $O/loop.jsonl 2> $O/loop.err
echo "[final] C1"
timeout -k 10 300 python tools/c1_bench.py 16 > $O/c1.json 2> $O/c1.err
cat $O/c1.json
echo "[final] done"
