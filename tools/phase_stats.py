#!/usr/bin/env python3
"""Min / median phase times over K factorization steps (after one warmup):
python3 tools/phase_stats.py <rr|genome> [K] [size_mib]   (LZ77SSS_LIB selects a build)"""
import os
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "lz77-sss_amd"))
import lz77sss as lz  # noqa: E402

wl = sys.argv[1]
K = int(sys.argv[2]) if len(sys.argv) > 2 else 5
n = (int(sys.argv[3]) if len(sys.argv) > 3 else 1024) << 20
T = lz.gen_random_repetitive(n, n, 42, 0.5, 0.05) if wl == "rr" else lz.gen_genome(n, 64 << 20, 0.001, 7)
rows = []
with lz.Session(n) as s:
    s.load(T)
    for k in range(K + 1):
        t0 = time.perf_counter()
        z = s.factorize()
        dt = (time.perf_counter() - t0) * 1e3
        if k:
            ph = s.phase_times()
            ph["step"] = dt
            rows.append(ph)
tag = os.path.basename(os.environ.get("LZ77SSS_LIB", "product"))
out = " ".join(f"{k}={min(r[k] for r in rows):.3f}/{statistics.median(r[k] for r in rows):.3f}" for k in rows[0])
print(f"{tag} {wl} z={z} min/median ms: {out}", flush=True)
