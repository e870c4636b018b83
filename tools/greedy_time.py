#!/usr/bin/env python3
"""Greedy phase timing of a variant build: python3 tools/greedy_time.py <rr|genome> [reps]
(LZ77SSS_LIB selects the library)."""
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "lz77-sss_amd"))
import lz77sss as lz  # noqa: E402

wl = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
n = 1 << 30
T = lz.gen_random_repetitive(n, n, 42, 0.5, 0.05) if wl == "rr" else lz.gen_genome(n, 64 << 20, 0.001, 7)
with lz.Session(n) as s:
    s.load(T)
    ts = []
    for k in range(reps + 1):
        z = s.factorize()
        if k:
            ts.append(s.phase_times()["greedy"])
    print(f"{os.path.basename(os.environ.get('LZ77SSS_LIB', 'product'))} {wl}: z={z} greedy ms "
          f"min={min(ts):.2f} med={sorted(ts)[len(ts) // 2]:.2f}", flush=True)
