"""Debug probe: pos_t = uint64_t factorization of a chr19-style text generated in HBM.
argv: size in MiB, mutation rate, greedy window (0 = auto).  Prints window hand-overs (LZ77SSS_DEBUG)."""
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "lz77-sss_amd"))
import lz77sss as lz  # noqa: E402

mib = int(sys.argv[1]) if len(sys.argv) > 1 else 4099
mut = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0001
win = int(sys.argv[3]) if len(sys.argv) > 3 else 0
if win:
    os.environ["LZ77SSS_GREEDY_WINDOW"] = str(win)
n = mib << 20
with lz.Session(n, pos64=True) as s:
    s.gen_genome(n, 59 << 20, mut, 7)
    t = time.time()
    z = s.factorize()
    dt = time.time() - t
    F = s.factors(z)
    st = s.stats()
    ln = np.maximum(F[:, 1], 1).astype(np.uint64)
    cs = np.cumsum(ln)
    print("stats", st[:12], flush=True)
    print(f"n={n} z={z} sum={int(cs[-1])} ok={int(cs[-1]) == n} windows={st[21]} outer={st[12]} t={dt:.2f}s "
          f"phases={s.phase_times()}", flush=True)
    bad = np.nonzero(F[:, 0] >= np.concatenate([[0], cs[:-1]]).astype(np.uint64) & (F[:, 1] > 0))[0]
    print("forward refs:", bad[:5].tolist(), flush=True)
