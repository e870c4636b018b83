"""Times the exact mode (csrc/exact.hip) on a 1 GiB workload and checks the round trip on the device."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lz77-sss_amd"))
import lz77sss as lz  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "rr"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 30
T = lz.gen_random_repetitive(n, n, 42, 0.5, 0.05) if kind == "rr" else lz.gen_genome(n, 64 << 20, 0.001, 7)
with lz.Session(n) as s:
    s.load(T)
    for rep in range(2):
        t = time.time()
        z = s.factorize_exact()
        dt = time.time() - t
        print(f"{kind} n={n} z={z} {dt*1e3:.1f} ms  {n/dt/1e6:.1f} MB/s  phases={s.phase_times()}", flush=True)
    _, mism = s.decode(out=False)
    print("device decode mismatches:", mism, flush=True)
