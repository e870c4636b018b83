#!/usr/bin/env python3
"""Summarize the SSS phase's FETCH_SIZE / WRITE_SIZE passes (tools/gpu_pmc_sss.sh) per call:
python3 tools/pmc_sss.py <rr|genome> <fetch.csv> <write.csv> -> JSON (the format bench.py's
pmc_traffic reads).  gfx950 FETCH_SIZE counts half the bytes of wide streaming reads
(MI355X_MICROARCH.md, HBM section): doubled; WRITE_SIZE as read.  prof_step.py 1 runs two calls."""
import csv
import json
import sys
from collections import defaultdict

CALLS = 2


def per_kernel(path, counter):
    acc = defaultdict(float)
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != counter:
            continue
        name = r["Kernel_Name"].split("(")[0]
        acc[name] += float(r["Counter_Value"])
    return {k: round(v / CALLS, 1) for k, v in acc.items()}


wl, fpath, wpath = sys.argv[1:4]
f = per_kernel(fpath, "FETCH_SIZE")
w = per_kernel(wpath, "WRITE_SIZE")
fk, wk = sum(f.values()), sum(w.values())
corr = 2.0
print(json.dumps({
    "kernels": "SSS phase: " + ", ".join(sorted(set(f) | set(w))), "workload": wl, "n": 1 << 30,
    "fetch_size_kib_per_call": round(fk, 1), "write_size_kib_per_call": round(wk, 1),
    "fetch_by_kernel_kib": f, "write_by_kernel_kib": w, "fetch_correction": corr,
    "hbm_bytes_per_launch": int((fk * corr + wk) * 1024)}, indent=1))
