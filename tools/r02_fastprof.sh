#!/bin/bash
# serial kernel times (ORBG_FAST0=0: no concurrent streams) + SQ counters of both FAST kernels
set -e -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r02e}
mkdir -p $O
cd /tmp
export TMPDIR=/tmp
for V in 1 2; do
  echo "== ORBG_FAST_V=$V"
  ORBG_FAST_V=$V ORBG_FAST0=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace_v$V -o run --output-format csv -- python3 $R/tools/extract_loop.py 256 6 > $O/trace_v$V.log 2>&1
  python3 - $O/trace_v$V/run_kernel_stats.csv <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    print("  %-40s calls %4s avg_us %9.1f" % (r["Name"].split("(")[0][:40], r["Calls"], float(r["AverageNs"])/1e3))
PY
  for DBG in 11 14 12; do
    ORBG_DBG=$DBG ORBG_FAST_V=$V ORBG_FAST0=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace_v${V}_d$DBG -o run --output-format csv -- python3 $R/tools/extract_loop.py 256 4 > /dev/null 2>&1
    python3 - $O/trace_v${V}_d$DBG/run_kernel_stats.csv $DBG <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if "fast" in r["Name"]:
        print("  dbg=%s %-30s avg_us %9.1f" % (sys.argv[2], r["Name"].split("(")[0][:30], float(r["AverageNs"])/1e3))
PY
  done
  ORBG_FAST_V=$V ORBG_FAST0=0 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU -d $O/pmc_v$V -o run --output-format csv -- python3 $R/tools/extract_loop.py 256 3 > $O/pmc_v$V.log 2>&1
  python3 - $O/pmc_v$V/run_counter_collection.csv <<'PY'
import csv,sys,collections
acc=collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    n=r["Kernel_Name"].split("(")[0].replace("orbg::","")
    if "fast" in n: acc[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
for n,d in acc.items():
    print("  ", n[:30], " ".join("%s=%.3g" % (k.replace("SQ_",""), sum(v)/len(v)) for k,v in sorted(d.items())))
PY
done
