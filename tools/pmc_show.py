#!/usr/bin/env python3
"""Per-launch averages of the counters in rocprofv3 counter_collection.csv files."""
import csv
import sys
from collections import defaultdict

for path in sys.argv[1:]:
    vals = defaultdict(list)
    names = {}
    for r in csv.DictReader(open(path)):
        vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
        names[r["Counter_Name"]] = r.get("Kernel_Name", "")[:60]
    for k, v in sorted(vals.items()):
        print(f"{k:28s} avg {sum(v)/len(v):16.1f}  n={len(v)}  {names[k]}")
