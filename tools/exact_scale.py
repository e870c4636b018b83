#!/usr/bin/env python3
"""exact-smpl phase times over text sizes (one line per run, flushed):
python3 tools/exact_scale.py <rr|genome> <mib,...> [transf_mode]"""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "lz77-sss_amd"))
import lz77sss as lz  # noqa: E402

kind = sys.argv[1]
sizes = [int(x) for x in sys.argv[2].split(",")]
tm = int(sys.argv[3]) if len(sys.argv) > 3 else lz.WITHOUT_SAMPLES
for mib in sizes:
    n = mib << 20
    T = lz.gen_random_repetitive(n, n, 42, 0.5, 0.05) if kind == "rr" else lz.gen_genome(n, min(n, 64 << 20) // 16 * 16 if n < (64 << 20) else 64 << 20, 0.001, 7)
    with lz.Session(n) as s:
        s.load(T)
        t = time.time()
        z = s.factorize_exact(tm)
        dt = time.time() - t
        st = s.stats()
        ph = {k: round(v, 1) for k, v in s.phase_times().items() if k.startswith("smpl")}
        print(f"{kind} {mib} MiB tm={tm} z={z} {dt * 1e3:.0f} ms {n / dt / 1e6:.1f} MB/s samples={st[24] if len(st) > 24 else '?'} "
              f"tasks={st[26] if len(st) > 26 else '?'} rounds/walks={st[27] >> 32 if len(st) > 27 else '?'}/"
              f"{st[27] & 0xFFFFFFFF if len(st) > 27 else '?'} {ph}", flush=True)
