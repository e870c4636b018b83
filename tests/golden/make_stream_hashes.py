#!/usr/bin/env python3
"""Writes tests/golden/stream_hashes.json: SHA-256 pins of the p = 1 oracle factor streams of the
full-size texts the GPU tests cannot afford to re-run the oracle on (test infrastructure only).

Each entry: the generator call that makes the text (the same seeded generators the GPU side uses,
so the box regenerates the bytes instead of loading them), the text's SHA-256, n, z, the oracle's
stats and the SHA-256 of the factor stream as little-endian (src, len) pairs of pos_t (mode
"exact_lengths": of the exact parse's length column, little-endian uint32).

    python3 tests/golden/make_stream_hashes.py [names...]      (default: all; ~2-6 min each)

The oracle runs here in the container (oracle/_build/liboracle.so, a CPU restatement of the
reference path); tests/test_stream_hashes.py compares the device streams with it.
"""
from __future__ import annotations

import hashlib
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "lz77-sss_amd"))
sys.path.insert(0, str(ROOT / "oracle"))
import lz77sss as lz  # noqa: E402
import oracle  # noqa: E402

OUT = Path(__file__).resolve().parent / "stream_hashes.json"

# name -> (generator, args, pos_t bits)
STREAMS = {
    # BASELINE configs[1] headline text (bench.py --workload rr)
    "rr_1gib": ("random_repetitive", dict(n=1 << 30, seed=42, rep=0.5, run=0.05), 32),
    # the realistic C2 text (bench.py --workload genome)
    "genome_1gib": ("genome", dict(n=1 << 30, base_len=64 << 20, mut=0.001, seed=7), 32),
    # C4-style: chr19-like 59 MiB ACGT block, 0.1 % mutations, positions past 2^32 (pos_t = uint64_t)
    "chr19_4gib_u64": ("genome_pos", dict(n=(1 << 32) + (3 << 20) + 12345, base_len=59 << 20, mut=0.001, seed=7), 64),
    # configs[2]: the headline text with LPF/LNF phrases (factorize_approximate<greedy, lpf_lnf_opt>)
    "rr_1gib_lpf_lnf": ("random_repetitive", dict(n=1 << 30, seed=42, rep=0.5, run=0.05), 32, "lpf_lnf_opt"),
    # configs[4]: exact greedy LZ77 of the headline and genome texts -- the length column only (the
    # canonical lengths; sources follow the range structure's visit order)
    "rr_1gib_exact_lengths": ("random_repetitive", dict(n=1 << 30, seed=42, rep=0.5, run=0.05), 32, "exact_lengths"),
    "genome_1gib_exact_lengths": ("genome", dict(n=1 << 30, base_len=64 << 20, mut=0.001, seed=7), 32,
                                  "exact_lengths"),
}


def make_text(kind, a, pad=0):
    if kind == "random_repetitive":
        T = lz.gen_random_repetitive(a["n"], a["n"], a["seed"], a["rep"], a["run"])
        return np.concatenate([T, np.zeros(pad, np.uint8)]) if pad else T
    if kind == "genome":
        T = lz.gen_genome(a["n"], a["base_len"], a["mut"], a["seed"])
        return np.concatenate([T, np.zeros(pad, np.uint8)]) if pad else T
    if kind == "genome_pos":
        return lz.gen_genome_pos(a["n"], a["base_len"], a["mut"], a["seed"], pad=pad)
    raise ValueError(kind)


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).view(np.uint8)).hexdigest()


def main(names):
    db = json.loads(OUT.read_text()) if OUT.exists() else {}
    for name in names:
        kind, a, bits, *rest = STREAMS[name]
        mode = rest[0] if rest else "lpf_opt"
        t0 = time.time()
        T = make_text(kind, a, pad=4096)
        n = a["n"]
        st = []
        if mode == "exact_lengths":  # oracle.hpp factorize_exact (SA-IS + PSV/NSV): the length column
            F = oracle.factorize_exact(T[:n])[:, 1].astype("<u4")
        elif bits == 32:
            F, st = oracle.factorize(T[:n], phr_mode=oracle.LPF_LNF_OPT if mode == "lpf_lnf_opt" else oracle.LPF_OPT)
            F = F.astype("<u4")
        else:
            F, st = oracle.factorize64(T[:n], buf=T)
            F = F.astype("<u8")
        db[name] = {"kind": kind, "args": a, "pos_bits": bits, "mode": mode, "n": n, "text_sha256": sha(T[:n]),
                    "z": int(F.shape[0]), "stats": [int(x) for x in st[:12]], "stream_sha256": sha(F),
                    "oracle_seconds": round(time.time() - t0, 1)}
        print(name, json.dumps(db[name]), flush=True)
        OUT.write_text(json.dumps(db, indent=1) + "\n")


if __name__ == "__main__":
    main(sys.argv[1:] or list(STREAMS))
