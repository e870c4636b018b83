"""Parity sweep (GPU): many generated texts, device 3-aprx stream vs the oracle and the device
exact-smpl stream vs the restated reference transform; prints one line per text and FAIL lines.
usage: python tools/sweep_parity.py <seconds budget>"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "lz77-sss_amd"), os.path.join(ROOT, "oracle")]
import lz77sss as lz  # noqa: E402
import oracle as orc  # noqa: E402

budget = float(sys.argv[1]) if len(sys.argv) > 1 else 500
t_end = time.time() + budget
cases = []
for seed in range(100, 140):
    mib = [1, 2, 3, 6][seed % 4]
    rep, run = [(0.5, 0.05), (0.9, 0.2), (0.3, 0.5), (0.7, 0.01)][(seed // 4) % 4]
    cases.append(("rr", mib, seed, rep, run))
    if seed % 3 == 0:
        cases.append(("genome", mib, seed, 0, 0))
fails = 0
with lz.Session(6 << 20) as s:
    for kind, mib, seed, rep, run in cases:
        if time.time() > t_end:
            break
        n = (mib << 20) - 12345 * (seed % 5)
        T = lz.gen_random_repetitive(n, n, seed, rep, run) if kind == "rr" else lz.gen_genome(n, 1 << 19, 0.002, seed)
        s.load(T)
        z = s.factorize()
        F = s.factors(z)
        Fo = orc.factorize(T)
        Fo = Fo[0] if isinstance(Fo, tuple) else Fo
        ok_a = F.shape == Fo.shape and np.array_equal(F, Fo)
        ze = s.factorize_exact(transf_mode=1)
        E = s.factors(ze)
        Eo = orc.factorize_exact_smpl(T, 1, 1)
        ok_e = E.shape == Eo.shape and np.array_equal(E, Eo)
        line = f"{kind} n={n} seed={seed} rep={rep} run={run}: approx z={z} {'ok' if ok_a else 'FAIL'}; exact z={ze} {'ok' if ok_e else 'FAIL'}"
        if not (ok_a and ok_e):
            fails += 1
            line = "FAIL " + line
        print(line, flush=True)
print(f"done, {fails} failing texts", flush=True)
