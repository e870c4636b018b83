"""Times the device decode (csrc/decode.hip) on a 1 GiB workload; run under rocprofv3 for per-kernel times."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lz77-sss_amd"))
import lz77sss as lz  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "rr"
n = (int(sys.argv[2]) if len(sys.argv) > 2 else 1024) << 20
T = lz.gen_random_repetitive(n, n, 42, 0.5, 0.05) if kind == "rr" else lz.gen_genome(n, 64 << 20, 0.001, 7)
with lz.Session(n) as s:
    s.load(T)
    z = s.factorize()
    for i in range(3):
        t0 = time.perf_counter()
        _, m = s.decode(out=False)
        dt = time.perf_counter() - t0
        print(f"{kind} z={z} decode#{i}: wall {dt*1e3:.1f} ms, timed {s.phase_times()['decode']:.1f} ms, "
              f"rounds {s.stats()[18]}, mismatches {m}", flush=True)
