#!/usr/bin/env python3
"""configs[3] one-GPU factorize (no sharded run before it) of a chr19-style text, pos_t = uint64_t:
python3 tools/c4_plain.py <size-gib> — prints the phase times and validates by device decode."""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "lz77-sss_amd"))
import lz77sss as lz  # noqa: E402

gib = float(sys.argv[1]) if len(sys.argv) > 1 else 8.0
n = int(gib * (1 << 30))
with lz.Session(n, pos64=True) as s:
    t = time.time()
    s.gen_genome(n, 59 << 20, 0.001, 7)
    print(f"text {n} bytes generated in HBM", flush=True)
    t = time.time()
    z = s.factorize()
    dt = time.time() - t
    print(f"factorize: z={z} {dt:.2f} s {n / dt / 1e6:.1f} MB/s phases={s.phase_times()}", flush=True)
    _, mism = s.decode(out=False)
    print(f"device decode mismatches: {mism}", flush=True)
