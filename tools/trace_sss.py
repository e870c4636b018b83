#!/usr/bin/env python3
"""SSS-phase kernels of the last step of a rocprofv3 kernel trace, from the last pass-1 launch
(k_sss_stream<false, true>) through the last k_sss_compact:
python3 tools/trace_sss.py <kernel_trace.csv>"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
p1 = [i for i, r in enumerate(rows) if "k_sss_stream<false, true>" in r["Kernel_Name"]]
a = p1[-1]
# the buffer fills just before pass 1 belong to the phase (the counters' clear)
while a > 0 and "fillBuffer" in rows[a - 1]["Kernel_Name"]:
    a -= 1
b = max(i for i, r in enumerate(rows) if "k_sss_compact" in r["Kernel_Name"] and i > a)
t0 = int(rows[a]["Start_Timestamp"])
tot = 0
print("# SSS phase of the last call: start offset, duration (us), kernel")
for r in rows[a:b + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    tot += e - s
    nm = re.sub(r"\(.*", "", r["Kernel_Name"])[:100]
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:9.1f}  {nm}")
print(f"# kernel time {tot / 1e3:.1f} us, span {(int(rows[b]['End_Timestamp']) - t0) / 1e3:.1f} us")
