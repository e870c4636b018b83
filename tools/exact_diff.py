"""Diagnostic: device exact-smpl vs the oracle on one text; prints the first differing phrase.
usage: python tools/exact_diff.py rr|genome MIB SEED [MODES, default 3,1,2,0]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "lz77-sss_amd"), os.path.join(ROOT, "oracle")]
import lz77sss as lz  # noqa: E402
import oracle as orc  # noqa: E402

kind, mib, seed = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
n = mib << 20
T = lz.gen_random_repetitive(n, n, seed, 0.5, 0.05) if kind == "rr" else lz.gen_genome(n, 1 << 20, 0.001, seed)
Fc = orc.factorize_exact(T)
print("canonical z", len(Fc), flush=True)
pos_c = np.concatenate([[0], np.cumsum(np.maximum(Fc[:, 1].astype(np.int64), 1))])
with lz.Session(n) as s:
    s.load(T)
    za = s.factorize()
    Fa = s.factors(za)
    Fo = orc.factorize(T)
    Fo = Fo[0] if isinstance(Fo, tuple) else Fo
    print(f"approx: z={za} oracle z={len(Fo)} equal={Fa.shape == Fo.shape and np.array_equal(Fa, Fo)}", flush=True)
    for tm in [int(x) for x in (sys.argv[4] if len(sys.argv) > 4 else "3,1,2,0").split(",")]:
        z = s.factorize_exact(transf_mode=tm)
        F = s.factors(z)
        st = s.stats()
        ok = F.shape == Fc.shape and np.array_equal(F[:, 1], Fc[:, 1])
        print(f"mode {tm}: z={z} lengths-equal={ok} stats24..={st[24:]}", flush=True)
        if not ok:
            k = min(len(F), len(Fc))
            d = int(np.nonzero(F[:k, 1] != Fc[:k, 1])[0][0])
            p = int(pos_c[d])
            print(f"  first diff phrase {d} at pos {p}: device {F[d - 1:d + 2].tolist()} canonical "
                  f"{Fc[d - 1:d + 2].tolist()}", flush=True)
