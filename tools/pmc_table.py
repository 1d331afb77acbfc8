#!/usr/bin/env python3
"""Average PMC counter values per orbg kernel over all pmc passes under a directory."""
import csv
import glob
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(list))
for path in glob.glob(sys.argv[1] + "/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("orbg::", "").strip()
        if not name.startswith("k_"):
            continue
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
cols = sorted({c for k in acc.values() for c in k})
print("kernel," + ",".join(cols))
for k, d in sorted(acc.items()):
    print(k + "," + ",".join("%.4g" % (sum(d[c]) / len(d[c])) if d.get(c) else "" for c in cols))
