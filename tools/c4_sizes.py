#!/usr/bin/env python3
"""Validity of the pos_t = uint64_t one-GPU factorization of chr19-style texts at growing sizes, each in a
fresh session, checked in HBM (Session.verify: bad positions and the first one):
python3 tools/c4_sizes.py <gib> [<gib> ...]"""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "lz77-sss_amd"))
import lz77sss as lz  # noqa: E402

ok = True
for g in (float(x) for x in sys.argv[1:]):
    n = int(g * (1 << 30))
    with lz.Session(n, pos64=True) as s:
        s.gen_genome(n, 59 << 20, 0.001, 7)
        t = time.time()
        z = s.factorize()
        dt = time.time() - t
        st = s.stats()
        bad, first = s.verify(first=True)
        print(f"[c4_sizes] {g} GiB n={n}: z={z} {dt:.1f} s, |S|={st[0]} phrases={st[2]} log2_h={st[11]} "
              f"windows={st[21]}; verify: bad={bad} first={first} phases={ {k: round(v, 1) for k, v in s.phase_times().items()} }",
              flush=True)
        ok = ok and bad == 0
sys.exit(0 if ok else 1)
