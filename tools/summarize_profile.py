#!/usr/bin/env python3
"""Turns the rocprofv3 outputs of tools/gpu_profile.sh into committed summaries under profiles/.

  profiles/<tag>_<wl>_kernel_stats.csv   rocprofv3 --kernel-trace --stats (as produced)
  profiles/<tag>_<wl>_kernels.txt        top kernels, per-bench-step totals
  profiles/<tag>_<wl>_pmc_sss.json       HBM bytes per launch of k_sss_stream from the two PMC passes

HBM bytes follow MI355X_MICROARCH.md (HBM/rocprofv3): FETCH_SIZE and WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reports half the bytes of a 16-B-per-lane streaming read (k_sss_stream
stages its tile with one uint4 load per lane), so it is doubled; WRITE_SIZE is taken as is.
"""
import csv
import json
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
tag, wl = sys.argv[1], sys.argv[2]
n = int(sys.argv[3]) if len(sys.argv) > 3 else 1 << 30
src = ROOT / "gpurun_out"
dst = ROOT / "profiles"
dst.mkdir(exist_ok=True)

ks = src / f"prof_{tag}_{wl}" / "run_kernel_stats.csv"
shutil.copy(ks, dst / f"{tag}_{wl}_kernel_stats.csv")
rows = list(csv.DictReader(open(ks)))
steps = 4  # bench.py --steps 3 --warmup 1
with open(dst / f"{tag}_{wl}_kernels.txt", "w") as f:
    f.write(f"# rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 3 --warmup 1 --workload {wl}\n")
    f.write("# per factorization = TotalDuration / 4 (3 timed + 1 warmup calls)\n")
    for r in rows[:30]:
        f.write(f"{r['Name'][:90]:90s} calls={int(r['Calls']):7d} per_factorization_ms="
                f"{float(r['TotalDurationNs']) / 1e6 / steps:9.3f} avg_us={float(r['AverageNs']) / 1e3:10.2f} "
                f"pct={float(r['Percentage']):5.1f}\n")


def counter(path, name):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path)) if r["Counter_Name"] == name]
    return sum(vals) / len(vals), len(vals)


fetch, nf = counter(src / f"pmc_{tag}_{wl}_fetch" / "run_counter_collection.csv", "FETCH_SIZE")
write, nw = counter(src / f"pmc_{tag}_{wl}_write" / "run_counter_collection.csv", "WRITE_SIZE")
sss_avg_ns = [float(r["AverageNs"]) for r in rows if "k_sss_stream" in r["Name"]][0]
hbm = 2 * fetch * 1024 + write * 1024
out = {"kernel": "k_sss_stream", "workload": wl, "n": n, "launches": {"fetch": nf, "write": nw},
       "fetch_size_kib": fetch, "write_size_kib": write, "fetch_correction": 2.0,
       "hbm_bytes_per_launch": int(hbm), "avg_launch_ns_kernel_trace": sss_avg_ns}
(dst / f"{tag}_{wl}_pmc_sss.json").write_text(json.dumps(out, indent=1) + "\n")
print(json.dumps(out))
