#!/usr/bin/env python3
"""exact-smpl walk profile on a generated text: python3 tools/smpl_prof.py <rr|genome> [size_mib] [runs]
(LZ77SSS_SMPL_PROF=1 prints per-walk clock statistics of k_chunk_walks / k_bridge_walks)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "lz77-sss_amd"))
import lz77sss as lz  # noqa: E402

wl = sys.argv[1]
n = int(sys.argv[2] if len(sys.argv) > 2 else 1024) << 20
with lz.Session(n) as s:
    # the texts of bench.py's make_text
    s.load(lz.gen_genome(n, 64 << 20, 0.001, 7) if wl == "genome" else lz.gen_random_repetitive(n, n, 42, 0.5, 0.05))
    for it in range(int(sys.argv[3]) if len(sys.argv) > 3 else 2):
        t = time.time()
        z = s.factorize_exact(transf_mode=lz.WITH_SAMPLES, log=1)
        print(f"{wl} n={n} exact z={z} {time.time() - t:.3f} s", flush=True)
