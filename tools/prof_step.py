#!/usr/bin/env python3
"""Factorization steps only (no decode / containers), for rocprofv3 kernel traces:
python3 tools/prof_step.py <rr|genome> [steps] [size_mib]"""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "lz77-sss_amd"))
import lz77sss as lz  # noqa: E402

wl = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
n = (int(sys.argv[3]) if len(sys.argv) > 3 else 1024) << 20
T = lz.gen_random_repetitive(n, n, 42, 0.5, 0.05) if wl == "rr" else lz.gen_genome(n, 64 << 20, 0.001, 7)
with lz.Session(n) as s:
    s.load(T)
    for k in range(steps + 1):
        t0 = time.perf_counter()
        z = s.factorize()
        dt = time.perf_counter() - t0
        print(f"step {k}: z={z} {dt*1e3:.3f} ms  phases={ {a: round(b, 3) for a, b in s.phase_times().items()} } "
              f"stats={s.stats()[:22]}", flush=True)
