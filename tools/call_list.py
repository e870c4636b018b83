#!/usr/bin/env python3
"""Kernels of one factorization call in launch order (start offset, duration, gap before, name)
from a rocprofv3 kernel trace: python3 tools/call_list.py <run_kernel_trace.csv> [call index, default last]
A call starts at each launch of SSS pass 1 (its preceding fill included)."""
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
first = "k_sss_stream<false, true>"
starts = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
ci = int(sys.argv[2]) if len(sys.argv) > 2 else -1
a = starts[ci]
b = starts[ci + 1] if ci != -1 and ci + 1 < len(starts) else len(rows)
t0 = int(rows[a]["Start_Timestamp"])
prev = t0
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    nm = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("rocprim::ROCPRIM_400200_NS::detail::", "rp::")
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {(s - prev) / 1e3:7.1f}  {nm[:110]}")
    prev = e
