#!/usr/bin/env python3
"""Which greedy path reproduces the short-chunk divergence on the c1_seed2 fixture
(DESIGN.md 4.5 known defect): LZ77SSS_GAP_CHUNK=128 under path knobs, vs the fixture stream."""
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "lz77-sss_amd"))
import lz77sss as lz  # noqa: E402

g = np.load(ROOT / "tests/golden/c1_seed2.npz")
T, Fg = g["text"], g["factors"]
knobs = [{}, {"LZ77SSS_PRED": "1"}, {"LZ77SSS_NO_PRED": "1"}, {"LZ77SSS_NO_DENSE": "1"},
         {"LZ77SSS_GREEDY_MAX_OUTER": "1"}, {"LZ77SSS_GREEDY_MAX_OUTER": "2"}, {"LZ77SSS_GREEDY_MAX_OUTER": "0"},
         {"LZ77SSS_NO_IPOSR": "1"}]
with lz.Session(T.size) as s:
    s.load(T)
    for ch in ["128", "512"]:
        for kn in knobs:
            env = {"LZ77SSS_GAP_CHUNK": ch, **kn}
            for k, v in env.items():
                os.environ[k] = v
            z = s.factorize()
            F = s.factors(z)
            d = np.nonzero(np.any(F != Fg, axis=1))[0] if F.shape == Fg.shape else "shape"
            st = s.stats()
            print(f"CH={ch} {kn}: {'ok' if isinstance(d, np.ndarray) and d.size == 0 else 'DIFF at ' + str(d[:4])} "
                  f"outer={st[12]} link={st[13]} completion={st[19]}@{st[20]}", flush=True)
            for k in env:
                del os.environ[k]
