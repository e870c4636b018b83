"""Debug probe: the pos_t = uint64_t engine against the oracle and the uint32_t engine with the same
gap-index size, on genome-like texts of growing size; prints the first differing factor."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "lz77-sss_amd"))
sys.path.insert(0, str(ROOT / "oracle"))
import lz77sss as lz  # noqa: E402
import oracle  # noqa: E402


def first_diff(a, b):
    m = min(len(a), len(b))
    d = np.nonzero(np.any(a[:m] != b[:m], axis=1))[0]
    return int(d[0]) if d.size else (m if len(a) != len(b) else -1)


for mib, base in [(1, 256 << 10), (2, 512 << 10), (4, 1 << 20), (8, 1 << 20), (16, 2 << 20)]:
    n = mib << 20
    T = lz.gen_genome(n, base, 0.001, 11)
    F_ref, st_ref = oracle.factorize64(T)
    with lz.Session(n, pos64=True) as s:
        s.load(T)
        F64 = s.factors(s.factorize())
        st = s.stats()
        lg = st[11]
    with lz.Session(n) as s:
        s.load(T)
        F32 = s.factors(s.factorize(index_log2_size=lg)).astype(np.uint64)
        st32 = s.stats()
    d1, d2 = first_diff(F64, F_ref), first_diff(F64, F32)
    print(f"{mib} MiB: z64={len(F64)} zref={len(F_ref)} z32(log2={lg})={len(F32)} diff_ref@{d1} diff_32@{d2} "
          f"outer={st[12]} rounds={st[13]} outer32={st32[12]} compl={st[19]}", flush=True)
    if d1 >= 0:
        pos = np.concatenate([[0], np.cumsum(np.maximum(F_ref[:, 1], 1))])
        print("  at text pos", int(pos[d1]), "ref", F_ref[d1 - 1:d1 + 2].tolist(), "gpu64", F64[d1 - 1:d1 + 2].tolist())
