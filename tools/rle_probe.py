#!/usr/bin/env python3
"""Greedy base-set diagnostics (LZ77SSS_DEBUG lines) for rr texts: python3 tools/rle_probe.py <mib> [seed]"""
import os
import sys
from pathlib import Path

os.environ["LZ77SSS_DEBUG"] = "1"
sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "lz77-sss_amd"))
import lz77sss as lz  # noqa: E402

n = int(sys.argv[1]) << 20
seed = int(sys.argv[2]) if len(sys.argv) > 2 else 42
T = lz.gen_random_repetitive(n, n, seed, 0.5, 0.05)
with lz.Session(n) as s:
    s.load(T)
    z = s.factorize()
    st = s.stats()
    print(f"n={n} z={z} stats={st}", flush=True)
