#!/usr/bin/env python3
"""Per-phase times of the approximate factorization (timing experiments):
python3 tools/phase_time.py <rr|genome> [reps]; prints the median of each phase."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "lz77-sss_amd"))
import os  # noqa: E402

import lz77sss as lz  # noqa: E402

wl = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
n = 1 << 30
T = lz.gen_random_repetitive(n, n, 42, 0.5, 0.05) if wl == "rr" else lz.gen_genome(n, 64 << 20, 0.001, 7)
with lz.Session(n) as s:
    s.load(T)
    runs = []
    for k in range(reps + 1):
        z = s.factorize()
        if k:
            runs.append(s.phase_times())
    med = {k: sorted(r[k] for r in runs)[len(runs) // 2] for k in runs[0]}
    knobs = {k: v for k, v in os.environ.items() if k.startswith("LZ77SSS_")}
    print(f"{wl} z={z} {knobs} " + " ".join(f"{k}={v:.3f}" for k, v in med.items()), flush=True)
