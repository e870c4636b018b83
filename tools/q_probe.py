"""SSS pass on 256 MiB texts of different structure (run under rocprofv3 --kernel-trace --stats):
which text regime makes k_q_anchors slow."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lz77-sss_amd"))
import lz77sss as lz  # noqa: E402

n = 256 << 20
rng = np.random.default_rng(1)
texts = {
    "random256": rng.integers(0, 256, n, dtype=np.uint8),
    "zeros": np.zeros(n, np.uint8),
    "period50": np.tile(rng.integers(0, 256, 50, dtype=np.uint8), n // 50 + 1)[:n],
    "period150": np.tile(rng.integers(0, 256, 150, dtype=np.uint8), n // 150 + 1)[:n],
    "period1000": np.tile(rng.integers(0, 256, 1000, dtype=np.uint8), n // 1000 + 1)[:n],
    "rr": lz.gen_random_repetitive(n, n, 42, 0.5, 0.05),
    "genome": lz.gen_genome(n, 16 << 20, 0.001, 7),
}
which = sys.argv[1:] or list(texts)
with lz.Session(n) as s:
    for k in which:
        s.load(texts[k])
        for _ in range(3):
            S, runs = s.sss()
        print(f"{k}: |S|={S.size} runs={runs}", flush=True)
