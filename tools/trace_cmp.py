#!/usr/bin/env python3
"""Per-kernel time of the last factorization step in two rocprofv3 kernel traces:
python3 tools/trace_cmp.py <trace_dir_a> <trace_dir_b> [top]"""
import csv
import glob
import re
import sys
from collections import defaultdict


def last_step(d):
    f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    a = [i for i, r in enumerate(rows) if "k_sss_stream<false" in r["Kernel_Name"]][-1]
    agg = defaultdict(lambda: [0, 0.0])
    t0 = int(rows[a]["Start_Timestamp"])
    end = t0
    for r in rows[a:]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        nm = re.sub(r"rocprim::ROCPRIM_400200_NS::detail::", "", re.sub(r"\(.*", "", r["Kernel_Name"]))[:64]
        agg[nm][0] += 1
        agg[nm][1] += (e - s) / 1e3
        end = max(end, e)
    return agg, (end - t0) / 1e3


A, sa = last_step(sys.argv[1])
B, sb = last_step(sys.argv[2])
print(f"span us: {sa:.1f} -> {sb:.1f}; busy {sum(v[1] for v in A.values()):.1f} -> {sum(v[1] for v in B.values()):.1f}")
keys = sorted(set(A) | set(B), key=lambda k: -abs(B.get(k, [0, 0])[1] - A.get(k, [0, 0])[1]))
for k in keys[: int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    a, b = A.get(k, [0, 0.0]), B.get(k, [0, 0.0])
    print(f"{a[1]:9.1f} ({a[0]:3d}) -> {b[1]:9.1f} ({b[0]:3d})  {k}")
