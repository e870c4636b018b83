#!/usr/bin/env python3
"""SSS phase timing only (timing experiments): python3 tools/sss_time.py <rr|genome> [reps]
(LZ77SSS_LIB selects a variant build)."""
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "lz77-sss_amd"))
import lz77sss as lz  # noqa: E402

wl = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
n = 1 << 30
T = lz.gen_random_repetitive(n, n, 42, 0.5, 0.05) if wl == "rr" else lz.gen_genome(n, 64 << 20, 0.001, 7)
with lz.Session(n) as s:
    s.load(T)
    ts = []
    for k in range(reps):
        S, runs = s.sss()
        ts.append(s.sss_kernel_time()[0])
    print(f"{os.path.basename(os.environ.get('LZ77SSS_LIB', 'product'))} {wl}: |S|={len(S)} runs={runs} "
          f"sss kernel ms min={min(ts):.3f} med={sorted(ts)[len(ts)//2]:.3f}", flush=True)
