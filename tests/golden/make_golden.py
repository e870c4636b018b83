#!/usr/bin/env python3
"""Regenerates tests/golden/*.npz from the CPU oracle (oracle/oracle.hpp).

The reference ships no golden vectors for this path and cannot
be built here, so these fixtures pin the oracle restatement itself: every
fixture holds the input text and the oracle's outputs (S, SA_S, LCP, LPF_opt
phrases, the factor stream and the approximation statistics).  The exact-mode stream (factors_exact) follows the oracle's
PSV/NSV source rule (oracle.hpp, "Exact greedy LZ77").  Texts come
from numpy's PCG64 or the seeded random_repetitive_string restatement; each
fixture stores its text, so the fixtures do not depend on any generator.

Usage: python tests/golden/make_golden.py   (writes next to this script)
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path.insert(0, str(ROOT / "oracle"))
sys.path.insert(0, str(ROOT / "lz77-sss_amd"))
import oracle  # noqa: E402
import lz77sss  # noqa: E402  (host-side generator only)


def texts():
    rng = np.random.Generator(np.random.PCG64(2024))
    out = {}
    for seed in (1, 2, 3, 4):
        out[f"c1_seed{seed}"] = lz77sss.gen_random_repetitive(10000, 200000, seed)
    for n in (1, 2, 100, 511, 512, 1023, 1024, 1025, 1535, 1536, 2047, 2048, 2049, 4096, 5000):
        out[f"edge_n{n}"] = rng.integers(0, 256, n, dtype=np.uint8)
    out["binary_30k"] = rng.integers(0, 2, 30000, dtype=np.uint8)
    out["zeros_10k"] = np.zeros(10000, np.uint8)
    # runs and periodic regions of periods around the Q threshold (tau/3 = 170)
    parts = []
    for p in (1, 2, 3, 7, 64, 169, 170, 171, 172, 200, 341):
        parts.append(rng.integers(0, 4, 700, dtype=np.uint8))
        unit = rng.integers(0, 4, p, dtype=np.uint8)
        parts.append(np.tile(unit, 2000 // p + 2)[:2000 + 37 * (p % 5)])
    out["periodic"] = np.concatenate(parts)
    # blocks copied with point mutations (genome-like, small)
    base = rng.integers(0, 4, 20000, dtype=np.uint8)
    blocks = []
    for _ in range(6):
        b = base.copy()
        idx = rng.integers(0, b.size, 20)
        b[idx] = rng.integers(0, 4, idx.size, dtype=np.uint8)
        blocks.append(b)
    out["genome_small"] = np.concatenate(blocks)
    return out


def main():
    for name, T in texts().items():
        T = np.ascontiguousarray(T, np.uint8)
        F, st = oracle.factorize(T)
        assert np.array_equal(oracle.decode(F, T.size), T)
        F3, st3 = oracle.factorize(T, phr_mode=oracle.LPF_LNF_OPT)
        S, has_runs = oracle.sss(T)
        _, SA, LCP = oracle.sa_s(T)
        P = oracle.lpf_opt(T)
        FX = oracle.factorize_exact(T)
        assert np.array_equal(oracle.decode(FX, T.size), T)
        np.savez_compressed(HERE / f"{name}.npz", text=T, factors=F, stats=st, factors_lnf=F3, stats_lnf=st3,
                            sss=S, has_runs=np.array([has_runs]), sa_s=SA, lcp=LCP, lpf=P, factors_exact=FX,
                            gap_bases_seed42=np.array(oracle.gap_bases(42), np.uint64))
        print(f"{name}: n={T.size} z={F.shape[0]} z_lnf={F3.shape[0]} z_exact={FX.shape[0]} |S|={S.size} lpf={P.shape[0]}")


if __name__ == "__main__":
    main()
