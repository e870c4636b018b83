#!/usr/bin/env python3
"""Per-factorization span vs busy time from a rocprofv3 kernel trace:
python3 tools/trace_calls.py <run_kernel_trace.csv> [first-kernel substring]
A call starts at each launch of the first kernel (default: SSS pass 1)."""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
first = sys.argv[2] if len(sys.argv) > 2 else "k_sss_stream<false, true>"
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
for a, b in zip(starts, starts[1:] + [len(rows)]):
    c = rows[a:b]
    s = int(c[0]["Start_Timestamp"])
    e = max(int(r["End_Timestamp"]) for r in c)
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in c)
    gaps = defaultdict(float)
    for x, y in zip(c, c[1:]):
        g = int(y["Start_Timestamp"]) - int(x["End_Timestamp"])
        if g > 20000:
            gaps[x["Kernel_Name"][:50] + " -> " + y["Kernel_Name"][:40]] += g / 1e3
    print(f"launches={len(c)} span_us={(e - s) / 1e3:.1f} busy_us={busy / 1e3:.1f}")
    for k, v in sorted(gaps.items(), key=lambda kv: -kv[1])[:8]:
        print(f"   gap {v:8.1f} us  {k}")
