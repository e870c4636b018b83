#!/usr/bin/env python3
"""Prints the top kernels of a rocprofv3 kernel_stats.csv (per-call averages)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
calls_div = int(sys.argv[2]) if len(sys.argv) > 2 else 1
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[: int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    print(f"{r['Name'][:80]:80s} calls={int(r['Calls']):7d} total/run={float(r['TotalDurationNs'])/1e6/calls_div:9.3f} ms "
          f"avg={float(r['AverageNs'])/1e3:10.1f} us {100*float(r['TotalDurationNs'])/tot:5.1f}%")
