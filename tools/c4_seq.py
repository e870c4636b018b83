#!/usr/bin/env python3
"""configs[3] sequence on ONE pos_t = uint64_t session: the resident sharded
path at world 1 (sss_range, set_sss, prepare, greedy_block), then a plain factorize of the same text,
both streams compared on the device and checked against the text in HBM (Session.verify).

python3 tools/c4_seq.py <size-gib> [--plain-first]
"""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "lz77-sss_amd"))
import torch  # noqa: E402

import lz77sss as lz  # noqa: E402
import sharded  # noqa: E402

gib = float(sys.argv[1]) if len(sys.argv) > 1 else 8.0
n = int(gib * (1 << 30))


def mem(tag):
    f, t = torch.cuda.mem_get_info(0)
    print(f"[c4_seq] {tag}: HBM free {f / 2**30:.1f} GiB of {t / 2**30:.1f}", flush=True)


torch.zeros(1, device="cuda")
with lz.Session(n, pos64=True) as s:
    s.gen_genome(n, 59 << 20, 0.001, 7)
    mem("text generated")
    t = time.time()
    tm = {}
    F1 = sharded.factorize_sharded_resident(s, n, 0, 1, 0, timings=tm)
    torch.cuda.synchronize()
    pm_p, pm_g = tm.pop("mem_prepare", {}), tm.pop("mem_greedy", {})
    print(f"[c4_seq] sharded (world 1): z={F1.shape[0]} {time.time() - t:.2f} s {tm}", flush=True)
    for ph, m in list(pm_p.items()) + list(pm_g.items()):
        print(f"[c4_seq]   sharded phase {ph}: held {m['held'] / 2**30:.1f} GiB, peak {m['peak'] / 2**30:.1f} GiB, "
              f"HBM free {m['hbm_free'] / 2**30:.1f} GiB", flush=True)
    mem("after sharded")
    bad1 = s.verify()
    print(f"[c4_seq] sharded stream verify: bad positions {bad1}", flush=True)
    t = time.time()
    z = s.factorize()
    print(f"[c4_seq] plain factorize: z={z} {time.time() - t:.2f} s phases={s.phase_times()}", flush=True)
    for ph, m in s.phase_mem().items():
        print(f"[c4_seq]   plain phase {ph}: held {m['held'] / 2**30:.1f} GiB, peak {m['peak'] / 2**30:.1f} GiB, "
              f"HBM free {m['hbm_free'] / 2**30:.1f} GiB", flush=True)
    mem("after plain")
    F2 = torch.empty(max(z, 1) * 2, dtype=torch.int64, device="cuda:0")
    if z:
        s.copy_factors(F2.data_ptr(), z * 16)
    same = z == F1.shape[0] and bool(torch.equal(F2[: 2 * z].view(-1, 2), F1))
    bad2 = s.verify()
    print(f"[c4_seq] plain stream verify: bad positions {bad2}; equal to the sharded stream: {same}", flush=True)
    ok = same and bad1 == 0 and bad2 == 0
print(f"[c4_seq] {'OK' if ok else 'FAILED'}", flush=True)
sys.exit(0 if ok else 1)
