#!/bin/bash
# k_fast2 only: parity, serial phase times, counters, bench
set -e -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r02g}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cd /tmp
export TMPDIR=/tmp
for DBG in 0 11 14 12; do
  ORBG_DBG=$DBG ORBG_FAST0=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace_d$DBG -o run --output-format csv -- python3 $R/tools/extract_loop.py 256 4 > /dev/null 2>&1
  python3 - $O/trace_d$DBG/run_kernel_stats.csv $DBG <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if "fast" in r["Name"] or sys.argv[2] == "0":
        print("  dbg=%s %-32s calls %3s avg_us %8.1f" % (sys.argv[2], r["Name"].split("(")[0][:32], r["Calls"], float(r["AverageNs"])/1e3))
PY
done
ORBG_FAST0=0 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU -d $O/pmc -o run --output-format csv -- python3 $R/tools/extract_loop.py 256 3 > $O/pmc.log 2>&1
python3 - $O/pmc/run_counter_collection.csv <<'PY'
import csv,sys,collections
acc=collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    n=r["Kernel_Name"].split("(")[0].replace("orbg::","")
    acc[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
for n,d in acc.items():
    if n.startswith("__"): continue
    print("  ", n[:24], " ".join("%s=%.3g" % (k.replace("SQ_",""), sum(v)/len(v)) for k,v in sorted(d.items())))
PY
cd $R
timeout -k 10 300 python bench.py --steps 20 --no-cpu > $O/bench.json 2> $O/bench.err
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step']);print({k:v['ms_per_step'] for k,v in d['kernels'].items()})"
