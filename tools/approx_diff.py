"""Diagnostic: device 3-approximation vs the oracle on one text, stage by stage (S, has_runs, SA_S,
LPF phrases, factors); prints the first difference.
usage: python tools/approx_diff.py rr|genome MIB SEED"""
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


def first_diff(a, b):
    k = min(len(a), len(b))
    d = np.nonzero(a[:k] != b[:k])[0] if k else []
    return int(d[0]) if len(d) else k


S_o, hr_o = orc.sss(T)
with lz.Session(n) as s:
    s.load(T)
    z = s.factorize()
    S_d, hr_d = s.sss()
    i = first_diff(S_d, S_o)
    print(f"S: device {len(S_d)} oracle {len(S_o)} runs {hr_d}/{hr_o} equal={len(S_d) == len(S_o) and i == len(S_d)}"
          + ("" if i == min(len(S_d), len(S_o)) else f" first diff at {i}: dev {S_d[i - 2:i + 3].tolist()} "
                                                     f"orc {S_o[i - 2:i + 3].tolist()}"), flush=True)
    L_d = s.lpf()
    L_o = orc.lpf_opt(T)
    print(f"LPF: device {L_d.shape} oracle {L_o.shape} equal={L_d.shape == L_o.shape and np.array_equal(L_d, L_o)}",
          flush=True)
    if not (L_d.shape == L_o.shape and np.array_equal(L_d, L_o)):
        k = min(len(L_d), len(L_o))
        d = np.nonzero(np.any(L_d[:k] != L_o[:k], axis=1))[0]
        j = int(d[0]) if len(d) else k
        print(f"  first LPF diff {j}: dev {L_d[j - 1:j + 2].tolist()} orc {L_o[j - 1:j + 2].tolist()}", flush=True)
        os.makedirs("gpurun_out", exist_ok=True)
        np.savez(f"gpurun_out/lpf_{kind}_{mib}_{seed}.npz", dev=L_d, orc=L_o)
    F = s.factors(z)
    Fo = orc.factorize(T)
    Fo = Fo[0] if isinstance(Fo, tuple) else Fo
    j = first_diff(F[:, 1], Fo[:, 1]) if F.shape == Fo.shape else -1
    eq = F.shape == Fo.shape and np.array_equal(F, Fo)
    print(f"factors: device {len(F)} oracle {len(Fo)} equal={eq}", flush=True)
    if not eq:
        k = min(len(F), len(Fo))
        d = np.nonzero(np.any(F[:k] != Fo[:k], axis=1))[0]
        j = int(d[0]) if len(d) else k
        pos = int(np.sum(np.maximum(Fo[:j, 1].astype(np.int64), 1)))
        print(f"  first factor diff {j} at pos {pos}: dev {F[j - 1:j + 2].tolist()} orc {Fo[j - 1:j + 2].tolist()}",
              flush=True)
        _, mism = s.decode(out=False)
        print(f"  device decode mismatches: {mism}", flush=True)
