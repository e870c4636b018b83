#!/usr/bin/env python3
"""SSS-phase kernels of the last step of a trace: python3 tools/trace_sss.py <kernel_trace.csv>"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
st = [i for i, r in enumerate(rows) if "k_sss_stream" in r["Kernel_Name"] or "k_q_anchors" in r["Kernel_Name"]]
# first SSS kernel of the last step: walk back from the last one while gaps are small
a = st[-1]
while a > 0 and ("k_sss" in rows[a - 1]["Kernel_Name"] or "k_q_anchors" in rows[a - 1]["Kernel_Name"]
                 or "k_run" in rows[a - 1]["Kernel_Name"] or "k_flag_list" in rows[a - 1]["Kernel_Name"]
                 or "rocprim" in rows[a - 1]["Kernel_Name"] or "rocclr" in rows[a - 1]["Kernel_Name"]):
    a -= 1
t0 = int(rows[a]["Start_Timestamp"])
for r in rows[a:a + int(sys.argv[2]) if len(sys.argv) > 2 else a + 16]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    nm = re.sub(r"\(.*", "", r["Kernel_Name"])[:90]
    print(f"{(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:8.1f}  {nm}")
