"""Runs only the SSS pass (k_q_anchors + k_sss_stream + compaction) a few times on a 1 GiB workload;
used under rocprofv3 --pmc to read the instruction mix of the SSS kernels."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lz77-sss_amd"))
import lz77sss as lz  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "rr"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
n = 1 << 30
T = lz.gen_random_repetitive(n, n, 42, 0.5, 0.05) if kind == "rr" else lz.gen_genome(n, 64 << 20, 0.001, 7)
with lz.Session(n) as s:
    s.load(T)
    for _ in range(reps):
        S, runs = s.sss()
    print(f"{kind}: |S|={S.size} has_runs={runs} kernel {s.sss_kernel_time()}", flush=True)
