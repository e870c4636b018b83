"""Debug probe: greedy windows vs the oracle on one C1 text (prints the window hand-overs)."""
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "lz77-sss_amd"))
sys.path.insert(0, str(ROOT / "oracle"))
import lz77sss as lz  # noqa: E402
import oracle  # noqa: E402

T = lz.gen_random_repetitive(10000, 200000, int(sys.argv[1]) if len(sys.argv) > 1 else 1)
F_ref, _ = oracle.factorize(T)
pos = np.concatenate([[0], np.cumsum(np.maximum(F_ref[:, 1].astype(np.int64), 1))])
print("n", T.size, "z_ref", len(F_ref), flush=True)
os.environ["LZ77SSS_GREEDY_WINDOW"] = sys.argv[2] if len(sys.argv) > 2 else "65536"
os.environ["LZ77SSS_DEBUG"] = "1"
with lz.Session(T.size) as s:
    s.load(T)
    F = s.factors(s.factorize())
m = min(len(F), len(F_ref))
d = np.nonzero(np.any(F[:m] != F_ref[:m], axis=1))[0]
k = int(d[0]) if d.size else m
print("z", len(F), "first diff", k, "at pos", int(pos[k]) if k < len(pos) else -1)
print("ref", F_ref[max(0, k - 2):k + 3].tolist())
print("gpu", F[max(0, k - 2):k + 3].tolist())
