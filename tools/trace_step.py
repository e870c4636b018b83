#!/usr/bin/env python3
"""Timeline of the last factorization step in a rocprofv3 kernel trace (tools/gpu_trace.sh):
python3 tools/trace_step.py gpurun_out/trace_<tag>_<wl>/run_kernel_trace.csv [steps] [--list]"""
import csv
import re
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# a step starts at a k_q_anchors launch
starts = [i for i, r in enumerate(rows) if "k_q_anchors" in r["Kernel_Name"] or "k_sss_stream_fused" in r["Kernel_Name"]]
a = starts[-1]
step = rows[a:]
t0 = int(step[0]["Start_Timestamp"])
busy = 0
prev_end = t0
agg = defaultdict(lambda: [0, 0.0])
lines = []
for r in step:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    nm = re.sub(r"\(.*", "", r["Kernel_Name"])[:70]
    busy += e - s
    agg[nm][0] += 1
    agg[nm][1] += (e - s) / 1e3
    lines.append(f"{(s - t0)/1e3:9.1f} us  gap {(s - prev_end)/1e3:7.1f}  dur {(e - s)/1e3:8.1f}  {nm}")
    prev_end = max(prev_end, e)
wall = (prev_end - t0) / 1e3
print(f"last step: {len(step)} kernels, wall {wall:.1f} us, busy {busy/1e3:.1f} us ({100*busy/1e3/wall:.0f}%)")
for nm, (c, d) in sorted(agg.items(), key=lambda x: -x[1][1])[:40]:
    print(f"  {d:9.1f} us  x{c:4d}  {nm}")
if "--list" in sys.argv:
    print("\n".join(lines))
