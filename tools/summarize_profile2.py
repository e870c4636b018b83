#!/usr/bin/env python3
"""profiles/<tag>_<wl>_* from the outputs of tools/gpu_profile2.sh:

  <tag>_<wl>_kernel_stats.csv   rocprofv3 --kernel-trace --stats (as produced)
  <tag>_<wl>_kernels.txt        top kernels per factorization (4 calls: 1 warmup + 3 timed)
  <tag>_<wl>_sss_phase.txt      the SSS-phase kernels of the last call, in launch order
  <tag>_<wl>_pmc_sss.json       HBM bytes per factorization call of the SSS-phase kernels

FETCH_SIZE on gfx950 is calibrated per MI355X_MICROARCH.md (HBM section): a streaming
read's bytes are 2 x FETCH_SIZE for 16-B-per-lane loads; other widths are uncalibrated,
so the raw KiB are kept beside the corrected total.
"""
import csv
import json
import re
import shutil
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
tag, wl = sys.argv[1], sys.argv[2]
n = int(sys.argv[3]) if len(sys.argv) > 3 else 1 << 30
src = ROOT / "gpurun_out"
dst = ROOT / "profiles"
dst.mkdir(exist_ok=True)
calls = 4

ks = src / f"prof_{tag}_{wl}" / "run_kernel_stats.csv"
shutil.copy(ks, dst / f"{tag}_{wl}_kernel_stats.csv")
rows = list(csv.DictReader(open(ks)))
with open(dst / f"{tag}_{wl}_kernels.txt", "w") as f:
    f.write(f"# rocprofv3 --kernel-trace --stats -- python3 tools/prof_step.py {wl} 3 (1 GiB, 4 factorize calls)\n")
    f.write("# per factorization = TotalDuration / 4\n")
    for r in rows[:40]:
        f.write(f"{r['Name'][:90]:90s} calls={int(r['Calls']):7d} per_factorization_ms="
                f"{float(r['TotalDurationNs']) / 1e6 / calls:9.3f} avg_us={float(r['AverageNs']) / 1e3:10.2f} "
                f"pct={float(r['Percentage']):5.1f}\n")

tr = sorted(csv.DictReader(open(src / f"prof_{tag}_{wl}" / "run_kernel_trace.csv")),
            key=lambda r: int(r["Start_Timestamp"]))
p1 = [i for i, r in enumerate(tr) if "k_sss_stream<false, true>" in r["Kernel_Name"]]
a = p1[-1] - 1
while a > 0 and "fillBuffer" not in tr[a]["Kernel_Name"]:
    a -= 1
t0 = int(tr[a]["Start_Timestamp"])
with open(dst / f"{tag}_{wl}_sss_phase.txt", "w") as f:
    f.write("# SSS phase of the last call: start offset, duration (us), kernel\n")
    tot = 0.0
    for r in tr[a:a + 40]:
        nm = re.sub(r"\(.*", "", r["Kernel_Name"])
        if "k_key" in nm or "k_iota" in nm:
            break
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        tot += (e - s) / 1e3
        f.write(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:9.1f}  {nm[:100]}\n")
    f.write(f"# kernel time {tot:.1f} us\n")


def per_call(path, name):
    tot = defaultdict(float)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == name:
            tot[re.sub(r"\(.*", "", r["Kernel_Name"])[:60]] += float(r["Counter_Value"])
    return {k: v / 3 for k, v in tot.items()}  # prof_step.py ... 2: 3 calls


fetch = per_call(src / f"pmc_{tag}_{wl}_fetch" / "run_counter_collection.csv", "FETCH_SIZE")
write = per_call(src / f"pmc_{tag}_{wl}_write" / "run_counter_collection.csv", "WRITE_SIZE")
fk, wk = sum(fetch.values()), sum(write.values())
out = {"kernels": "SSS phase: " + ", ".join(sorted(fetch)), "workload": wl, "n": n,
       "fetch_size_kib_per_call": round(fk, 1), "write_size_kib_per_call": round(wk, 1),
       "fetch_by_kernel_kib": {k: round(v, 1) for k, v in fetch.items()},
       "write_by_kernel_kib": {k: round(v, 1) for k, v in write.items()},
       "fetch_correction": 2.0,
       "hbm_bytes_per_launch": int(2 * fk * 1024 + wk * 1024)}
(dst / f"{tag}_{wl}_pmc_sss.json").write_text(json.dumps(out, indent=1) + "\n")
print(json.dumps(out))
