#!/usr/bin/env python3
"""Headline benchmark: 3-approximate LZ77 factorization MB/s on a 1 GiB text.

Metric (BASELINE.json): "factorization MB/s + factor count, 3-aprx on 1 GiB
repetitive text".  One *step* = one full ``factorize_approximate<greedy,
lpf_opt, 512>`` of the text (SSS -> SA_S/LCP/RMQ -> LPF_opt -> greedy emitter,
factors left in HBM), the text already resident in HBM when the timed region
starts.  MB = 10^6 bytes as the reference's
``throughput`` helper (utils.hpp:88-91).

Workloads:
  rr      random_repetitive_string(2^30, 2^30) with repetition 0.5, run 0.05,
          seed 42 (+rank) -- configs[1] of BASELINE.json (default)
  genome  4-letter 64 MiB base block repeated with 0.1% point mutations, seed 7

Multi-GPU (``--gpus N`` under torch.distributed.run): the texts are
independent objects, one 1 GiB text per rank (seed 42 + rank); no data-path
collective, the barrier/max-over-ranks timing only (weak scaling).  The same
line carries ``strong_scaling_one_text``: rank 0's text split over all ranks
through the sharded path's collectives (sync set by block + all-gather,
rank-ordered chain blocks with the state hand-over, gathered emission;
strong scaling, max over ranks), checked against rank 0's one-GPU stream.

Also reported:
  roofline      the SSS kernel sequence (k_sss_stream pass 1 with the periodicity
                filter, k_sss_runs on the stripes pass 1 stopped, the exact Q pass on
                marked tiles and the re-run of stripes that see Q windows, the run-record
                segments, the compaction of S), algorithmic bytes n + 4|S| per call over
                its HIP-event time on the library's own stream (two windows: the
                phase's one host read is not kernel time),
                against the 8 TB/s HBM3E peak; ``traffic`` from the committed
                rocprofv3 PMC summary (profiles/) when one exists for this
                workload, else null.
  cpu_baseline  the CPU oracle (a port of the reference algorithm, OpenMP) on
                rank 0 at N=1, on a bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "lz77-sss_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
GIB = 1 << 30


def make_text(lz, workload: str, n: int, rank: int):
    if workload == "rr":
        return lz.gen_random_repetitive(n, n, 42 + rank, 0.5, 0.05)
    if workload == "genome":
        return lz.gen_genome(n, 64 << 20, 0.001, 7 + rank)
    raise SystemExit(f"unknown workload {workload}")


def aggregate(dt_local: float, n_per_rank: int, world: int, dist=None, device="cpu"):
    """Max step time over ranks and the whole-job MB/s (every rank processed its own n bytes)."""
    dt = dt_local
    if dist is not None and world > 1:
        import torch

        if dist.get_backend() != "nccl":
            device = "cpu"  # (gloo rehearsal runs: host tensors)
        t = torch.tensor([dt_local], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dt, world * n_per_rank / dt / 1e6


# the SSS kernel set the roofline covers; a PMC summary counts only if it measured
# all of them (older summaries predate k_sss_runs and cover a different kernel sequence)
SSS_KERNELS = ("k_sss_stream<false, true>", "k_sss_runs", "k_sss_compact_scan")


def pmc_traffic(workload: str, n: int, mode: str = "approx"):
    """Per-call HBM bytes of the SSS kernels from profiles/*_pmc_sss.json (rocprofv3 --pmc passes), for
    this workload, size and mode (a summary without "mode" is a 3-aprx one), measured over the current
    kernel set; None when no such summary exists."""
    best = None
    for p in sorted((ROOT / "profiles").glob("*_pmc_sss.json")):
        try:
            d = json.loads(p.read_text())
        except (OSError, ValueError):
            continue
        if d.get("workload") != workload or int(d.get("n", -1)) != n or d.get("mode", "approx") != mode:
            continue
        if not all(any(k in name for name in d.get("fetch_by_kernel_kib", {})) for k in SSS_KERNELS):
            continue
        best = d
    return None if best is None else best.get("hbm_bytes_per_launch")


PHR = {"lpf_opt": 2, "lpf_lnf_opt": 3}
TRANSF = {"naive": 0, "with_samples": 1, "without_samples": 2, "full_sa": 3}


def cpu_model() -> str:
    """lscpu's model name (read from /proc/cpuinfo, the same field)."""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(lz, workload: str, sample_mib: int, phr_mode: int = 2, runs: int = 3):
    """the oracle timed at p = the host's OpenMP thread count and at
    p = 1, median of `runs` each; `value` is the p = nproc median."""
    import statistics

    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle  # the CPU port (test/bench infrastructure only)

    n = sample_mib << 20
    T = make_text(lz, workload, n, 0)
    p = oracle.num_threads()
    res = {}
    par = False
    for threads in (p, 1):
        secs, z = [], 0
        for r in range(runs):
            z, sec, _, par_r = oracle.factorize_timed_p(T, threads, phr_mode=phr_mode)
            par = par or (threads == p and par_r)
            secs.append(sec)
            print(f"cpu_baseline {workload} p={threads} run {r + 1}/{runs}: {sec:.2f} s", file=sys.stderr, flush=True)
        res[threads] = (statistics.median(secs), z, secs)
    sec_p, z_p, _ = res[p]
    sec_1, z_1, _ = res[1]
    greedy = ("the reference's racy parallel greedy, greedy_parallel.cpp:31-285, selected as lz77_sss.hpp:467-474"
              if par else "sequential greedy: lz77_sss.hpp:467-474 does not select the parallel one for this text")
    desc = ("full 1 GiB workload text" if n == GIB else f"{sample_mib} MiB instance of the same generator")
    return {"value": round(n / sec_p / 1e6, 2), "unit": "MB/s", "cores": p, "kind": "port",
            "cpu_model": cpu_model(), "runs": runs,
            "p1": {"value": round(n / sec_1 / 1e6, 2), "cores": 1, "median_s": round(sec_1, 3), "factors": z_1},
            "sample": f"{workload}: {desc} (n={n}), oracle factorize_approximate<greedy,"
                      f"{'lpf_opt' if phr_mode == 2 else 'lpf_lnf_opt'}> median of {runs}: p={p} threads "
                      f"{sec_p:.2f} s (z={z_p}; OpenMP SSS/sort stages, LPF in {p} partitions as "
                      f"lpf_opt.cpp:46-56, {greedy}), p=1 {sec_1:.2f} s (z={z_1})",
            "greedy_parallel": par}


CHR19_SAMPLE_N = (1 << 32) + (3 << 20) + 12345  # the instance tests/golden/stream_hashes.json pins (chr19_4gib_u64)


def cpu_baseline_chr19(lz, n: int):
    """configs[3]'s CPU leg: the oracle (pos_t = uint64_t) at p = the host's OpenMP threads on a chr19-style
    instance of n bytes (default the 4 GiB + 3 MiB one whose p = 1 stream is SHA-pinned), one run."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle  # the CPU port (test/bench infrastructure only)

    buf = lz.gen_genome_pos(n, 59 << 20, 0.001, 7, pad=4096)
    p = oracle.num_threads()
    print(f"cpu_baseline chr19 p={p}: n={n} ...", file=sys.stderr, flush=True)
    z, sec, _, par = oracle.factorize_timed_p64(buf[:n], p, buf=buf)
    print(f"cpu_baseline chr19 p={p}: {sec:.1f} s z={z}", file=sys.stderr, flush=True)
    greedy = ("the reference's racy parallel greedy, greedy_parallel.cpp:31-285, selected as lz77_sss.hpp:467-474"
              if par else "sequential greedy")
    return {"value": round(n / sec / 1e6, 2), "unit": "MB/s", "cores": p, "kind": "port", "cpu_model": cpu_model(),
            "runs": 1, "sample": f"chr19-style (59 MiB ACGT block, 0.1% mutations, position-hashed as the GPU's), "
                                 f"n={n} ({n / GIB:.3f} GiB, pos_t=uint64), oracle factorize_approximate<greedy,lpf_opt> "
                                 f"at p={p}: {sec:.1f} s, z={z} ({greedy})",
            "greedy_parallel": par}


def cpu_baseline_exact(lz, workload: str, sample_mib: int, transf_mode: str):
    """configs[4]'s CPU leg: the restatement of the reference's own transform (oracle/oracle_exact.hpp:
    factorize_exact<greedy, lpf_opt, with_samples | without_samples>, its 3-approximation included) at
    p = min(16, host threads) on the workload's text (default the full one), one run."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle  # the CPU port (test/bench infrastructure only)

    n = sample_mib << 20
    T = make_text(lz, workload, n, 0)
    p = min(16, oracle.num_threads())
    mode = oracle.WITHOUT_SAMPLES if transf_mode == "without_samples" else oracle.WITH_SAMPLES
    mname = "without_samples" if mode == oracle.WITHOUT_SAMPLES else "with_samples"
    print(f"cpu_baseline exact p={p}: n={n} {mname} ...", file=sys.stderr, flush=True)
    z, sec, sec_aprx = oracle.factorize_exact_smpl_timed(T, mode, p)
    print(f"cpu_baseline exact p={p}: {sec:.1f} s z={z}", file=sys.stderr, flush=True)
    return {"value": round(n / sec / 1e6, 2), "unit": "MB/s", "cores": p, "kind": "port", "cpu_model": cpu_model(),
            "runs": 1,
            "sample": f"{workload}: {sample_mib} MiB instance of the same generator (n={n}); the restatement of "
                      f"the reference's transform_to_exact_{mname} (oracle_exact.hpp: sample set, PA/SA by stable "
                      f"sort, interval samples, decomposed weighted square grid, 16 p sections) after its "
                      f"3-approximation, p={p}: {sec:.2f} s ({sec_aprx:.2f} s approximation), z={z} "
                      f"(sections restart the greedy parse: z >= the canonical z)",
            "device_transform": "one device implementation serves with_samples and without_samples (csrc/smpl.hip: "
                                "sparse-table interval lifting replaces with_samples' interval samples), so the "
                                "two modes time the same device code; naive drops the approximate lower bound "
                                "and the Pi / Psi scans"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="rr", choices=["rr", "genome", "chr19"],
                    help="chr19 (--shard only): configs[3]'s chr19-style text of --size-gib GiB generated in "
                         "HBM (59 MiB ACGT base block, 0.1%% mutations per copy), pos_t = uint64_t")
    ap.add_argument("--size-mib", type=int, default=1024)
    ap.add_argument("--phr-mode", default="lpf_opt", choices=["lpf_opt", "lpf_lnf_opt"],
                    help="lpf_opt = configs[1]; lpf_lnf_opt = configs[2] (LPF/LNF phrases)")
    ap.add_argument("--mode", default="approx", choices=["approx", "exact", "sss"],
                    help="approx = configs[1]/[2] (3-aprx); exact = configs[4] (exact factorization); "
                         "sss = the sharded pos_t=uint64 sync-set pass of configs[3] (chr19-style text)")
    ap.add_argument("--transf-mode", default="with_samples", choices=["naive", "with_samples", "without_samples", "full_sa"],
                    help="--mode exact: factorize_exact's transform_mode (configs[4]: with_samples, the sample index; "
                         "full_sa is the device extension)")
    ap.add_argument("--size-gib", type=float, default=50.0,
                    help="--mode sss / --workload chr19: text size in GiB (configs[3]: 50)")
    ap.add_argument("--cpu-sample-mib", type=int, default=-1,
                    help="oracle sample size in MiB (default: the full workload text, 2-30 s of CPU work)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--shard", action="store_true",
                    help="--mode approx: ONE text split across the ranks (sharded.factorize_sharded_resident: "
                         "sync set by block + all-gather, replicated phrases, rank-ordered greedy blocks, "
                         "rank-ordered emission; strong scaling) instead of one independent text per rank")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the N > 1 path on a one-GPU box: every rank on device 0, gloo between the ranks
    # (LZ77SSS_BENCH_SHARE_GPU=1); the driver's runs use one GPU per rank and RCCL
    share_gpu = os.environ.get("LZ77SSS_BENCH_SHARE_GPU") == "1"
    if share_gpu:
        local_rank = 0
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)

    import torch
    import lz77sss as lz

    torch.cuda.set_device(local_rank)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if share_gpu:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    if args.mode == "sss":
        return main_sss(args, lz, torch, dist, world, rank, local_rank)
    if args.shard:
        if args.mode != "approx" or args.phr_mode != "lpf_opt":
            raise SystemExit("--shard runs the 3-aprx with lpf_opt (configs[1])")
        return main_shard(args, lz, torch, dist, world, rank, local_rank)
    if args.workload == "chr19":
        raise SystemExit("--workload chr19 runs with --shard (configs[3])")

    n = args.size_mib << 20
    T = make_text(lz, args.workload, n, rank)
    sess = lz.Session(n, device=local_rank)
    t_load0 = time.perf_counter()
    sess.load(T)
    t_load = time.perf_counter() - t_load0

    exact = args.mode == "exact"

    # the factors reach the caller in host memory inside the timed step (the span
    # includes the output callback into a preallocated vector): a pinned buffer sized after warmup
    out_buf = [None]

    def step():
        z = sess.factorize_exact(TRANSF[args.transf_mode], device=local_rank) if exact else \
            sess.factorize(device=local_rank, phr_mode=PHR[args.phr_mode])
        if out_buf[0] is not None and z * 8 <= out_buf[0].numel():
            sess.copy_factors(out_buf[0].data_ptr(), out_buf[0].numel())
        return z

    z_w = 0
    for _ in range(max(args.warmup, 1)):
        z_w = step()
    out_buf[0] = torch.empty(max(z_w * 8, 8) + (1 << 20), dtype=torch.uint8, pin_memory=True)

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    kern_ms, kern_bytes = [], []
    barrier()
    t0 = time.perf_counter()
    z = 0
    for _ in range(args.steps):
        z = step()
        ms, b = sess.sss_kernel_time()
        kern_ms.append(ms)
        kern_bytes.append(b)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier()
    dt, value = aggregate((t1 - t0) / args.steps, n, world, dist, device="cuda")

    phases = sess.phase_times()
    pmem = sess.phase_mem()
    st = sess.stats()
    # N > 1: also ONE text (rank 0's, seed 42) split over all ranks through the sharded path's
    # collectives (sync set by block + all-gather, rank-ordered chain blocks with the
    # state hand-over, gathered emission), timed the same way -- strong scaling beside the weak line
    strong = None
    if world > 1 and not exact and args.phr_mode == "lpf_opt" and not os.environ.get("LZ77SSS_BENCH_NO_STRONG"):
        try:
            strong = strong_scaling_line(args, lz, torch, dist, world, rank, local_rank, n, sess, int(z))
        except Exception as e:  # (reported in the line; the weak measurement above stands)
            strong = {"error": f"{type(e).__name__}: {e}"}
    # PCIe-inclusive rate of one call (host text in, factors out), reported beside the HBM-resident value
    t_out0 = time.perf_counter()
    F = sess.factors(z)
    t_out = time.perf_counter() - t_out0
    del F
    # device decode of the same factors, compared in HBM with the input (outside the timed region)
    _, mism = sess.decode(out=False)
    dec_ms = sess.phase_times().get("decode", float("nan"))
    dec_rounds = sess.stats()[18]
    # the Huffman factor container of the same factors (csrc/huffman.hip), host copy included
    t_h0 = time.perf_counter()
    hbytes = int(sess.huffman().size)
    t_h = time.perf_counter() - t_h0

    if rank == 0:
        avg_ms = sum(kern_ms) / len(kern_ms)
        bytes_launch = kern_bytes[-1]
        achieved = bytes_launch / (avg_ms * 1e-3) / 1e9
        out = {
            "metric": f"factorization MB/s (exact greedy LZ77, factorize_exact<greedy, lpf_opt, {args.transf_mode}>, "
                      f"tau=512)" if exact else
                      f"factorization MB/s (3-aprx LZ77, greedy + {args.phr_mode}, tau=512)",
            "value": round(value, 2),
            "unit": "MB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded restatement of the reference's random_repetitive_string)"
            if args.workload == "rr" else "synthetic (genome-like: 64 MiB ACGT base block, 0.1% mutations)",
            "config": {
                "workload": f"{args.workload} n={n} ({args.size_mib} MiB) per GPU, pos_t=uint32",
                "n": n, "tau": 512, "phr_mode": args.phr_mode, "fact_mode": "greedy", "virtual_p": 1,
                "mode": f"exact (configs[4]), transf_mode={args.transf_mode}" if exact else
                        ("3-aprx (configs[2])" if args.phr_mode == "lpf_lnf_opt" else "3-aprx (configs[1])"),
                "parallelism": f"independent-texts x{world}" if world > 1 else "single GPU",
                "factors_to_host_in_step": True,
                "factors": int(z), "comp_ratio": round(n / max(z, 1), 2),
                "sss_size": int(st[0]) if st else None, "has_runs": bool(st[1]) if st else None,
                "lpf_phrases": int(st[2]) if st else None,
                "greedy": None if exact or not st else {
                    "outer_rounds": int(st[12]), "link_rounds": int(st[13]), "walked": int(st[15]),
                    "segments": int(st[16]), "completion_used": bool(st[19]),
                    "completion_start": int(st[20]), "windows": int(st[21])},
                "phase_ms": {k: round(v, 3) for k, v in phases.items()},
                "pcie_inclusive_mbps": round(n / (dt + t_load + t_out) / 1e6, 2),
                "device_decode": {"mismatches": int(mism), "ms": round(dec_ms, 3), "jump_rounds": int(dec_rounds),
                                  "mbps": round(n / (dec_ms * 1e-3) / 1e6, 1)},
                "huffman_container": {"bytes": hbytes, "ms_incl_d2h": round(t_h * 1e3, 3)},
                "phase_mem_gib": {ph: {k: round(v / GIB, 3) for k, v in m.items()} for ph, m in pmem.items()},
            },
            "roofline": {
                "kernel": "SSS phase kernels (DESIGN.md 4.1): k_sss_stream pass 1, k_sss_runs, [Q-anchor pass + re-run "
                          "where a tile is marked], k_blk_seg_tiles/info, compaction; HIP events in two windows "
                          "around the phase's one host read",
                "bound": "hbm",
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": pmc_traffic(args.workload, n, "exact" if exact else "approx"),
                "algorithmic_bytes_per_launch": int(bytes_launch),
                "avg_launch_ms": round(avg_ms, 4),
            },
            "cpu_baseline": None,
        }
        if not exact and st and phases.get("sss"):
            # the whole SSS phase (Q anchors + run table + stream + compaction), same algorithmic bytes
            sb = n + 4 * int(st[0])
            out["roofline_sss_phase"] = {
                "phase": "sss (k_q_anchors + run table + k_sss_stream + compaction)", "bound": "hbm",
                "achieved": round(sb / (phases["sss"] * 1e-3) / 1e9, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(sb / (phases["sss"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                "algorithmic_bytes": sb, "ms": round(phases["sss"], 4),
                "ms_per_gib": round(phases["sss"] * GIB / n, 4)}
            pipe = sum(v for k, v in phases.items() if k != "decode")
            out["roofline_pipeline"] = {
                "bound": "hbm", "note": "text bytes per step over the whole pipeline's phase time",
                "achieved": round(n / (pipe * 1e-3) / 1e9, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(n / (pipe * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "ms": round(pipe, 3)}
        if strong is not None:
            out["strong_scaling_one_text"] = strong
        if world == 1 and not args.no_cpu_baseline:
            sample = args.cpu_sample_mib if args.cpu_sample_mib > 0 else args.size_mib
            if exact:
                out["cpu_baseline"] = cpu_baseline_exact(lz, args.workload, sample, args.transf_mode)
            else:
                out["cpu_baseline"] = cpu_baseline(lz, args.workload, sample, PHR[args.phr_mode])
        print(json.dumps(out), flush=True)
    sess.close()
    if dist is not None:
        dist.destroy_process_group()


def strong_scaling_line(args, lz, torch, dist, world, rank, local_rank, n, sess_weak, z_weak):
    """The N > 1 extra of the default line: rank 0's text (seed 42) factorized by all ranks together
    (sharded.factorize_sharded_resident: collectives (1)-(4) of SURVEY.md 8e), max step time over
    ranks; rank 0 compares the stream with its own one-GPU factorization of that text (the weak run's
    last step, still in its session).  Returns the dict rank 0 adds to the JSON line (else None)."""
    import sharded

    T0 = make_text(lz, args.workload, n, 0)
    s2 = lz.Session(n, device=local_rank)
    s2.load(T0)
    del T0
    steps = max(2, args.steps // 4)
    F = None
    for _ in range(max(args.warmup, 1)):
        F = sharded.factorize_sharded_resident(s2, n, rank, world, local_rank)
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        F = sharded.factorize_sharded_resident(s2, n, rank, world, local_rank)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    dist.barrier()
    dt, _ = aggregate((t1 - t0) / steps, n, world, dist, device="cuda")
    out = None
    if rank == 0:
        zw = int(F.shape[0])
        ok = False
        if zw == z_weak:
            ref = torch.empty(max(zw, 1) * 2, dtype=torch.int32, device=f"cuda:{local_rank}")
            if zw:
                sess_weak.copy_factors(ref.data_ptr(), zw * 8)
            ok = bool(torch.equal(ref[: 2 * zw].view(-1, 2), F))
        out = {"value": round(n / dt / 1e6, 2), "unit": "MB/s", "ms_per_step": round(dt * 1e3, 3), "steps": steps,
               "scaling": "strong", "n": n,
               "workload": f"{args.workload} n={n}: rank 0's text split over {world} ranks",
               "parallelism": f"sharded x{world}: S by block + all-gather, replicated phrases, rank-ordered greedy "
                              f"blocks with the chain-state hand-over, gathered emission",
               "factors": int(zw), "equals_one_gpu_stream": ok}
    s2.close()
    return out


def main_shard(args, lz, torch, dist, world, rank, local_rank):
    """One text factorized by all ranks together: one step = sharded.factorize_sharded_resident
    (collectives (1)-(4) of SURVEY.md 8e).  rr / genome: the seed-42 text of the default mode
    (--size-mib); chr19: configs[3]'s chr19-style text of --size-gib GiB generated in HBM with
    pos_t = uint64_t (every rank holds the whole text: the phrases are replicated).  The greedy
    chain is walked block by block in rank order (speculative concurrent blocks are opt-in,
    LZ77SSS_SPECULATE=1: sharded.py); total work is fixed (strong scaling).  After the timed
    region rank 0 checks the stream against a one-GPU factorize of the same text on the same session, and
    both against the text in HBM."""
    import sharded

    chr19 = args.workload == "chr19"
    n = int(args.size_gib * GIB) if chr19 else args.size_mib << 20
    pos64 = chr19 or n > (1 << 32) - 16
    sess = lz.Session(n, device=local_rank, pos64=pos64)
    t_gen0 = time.perf_counter()
    if chr19:
        sess.gen_genome(n, 59 << 20, 0.001, 7)
    else:
        T = make_text(lz, args.workload, n, 0)
        sess.load(T)
        del T
    torch.cuda.synchronize()
    t_gen = time.perf_counter() - t_gen0
    print(f"[bench --shard] rank {rank}: text of {n} bytes in HBM ({t_gen:.1f} s)", file=sys.stderr, flush=True)
    tm = {}

    def step():
        t = time.perf_counter()
        F = sharded.factorize_sharded_resident(sess, n, rank, world, local_rank, timings=tm)
        print(f"[bench --shard] rank {rank}: step {time.perf_counter() - t:.2f} s, phases "
              f"{ {k: (round(v, 3) if isinstance(v, float) else v) for k, v in tm.items()} }", file=sys.stderr,
              flush=True)
        return F

    for _ in range(args.warmup):
        step()

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    barrier()
    t0 = time.perf_counter()
    F = None
    for _ in range(args.steps):
        F = step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier()
    dt, _ = aggregate((t1 - t0) / args.steps, n, world, dist, device="cuda")  # max over ranks
    mem = {}
    for key in ("mem_prepare", "mem_greedy"):
        for ph, m in (tm.pop(key, None) or {}).items():
            mem[ph] = {k: round(v / GIB, 2) for k, v in m.items()}
    phases = {k: (round(v * 1e3, 3) if isinstance(v, float) else v) for k, v in tm.items()}
    z = int(F.shape[0])
    same = None
    st = sess.stats()
    verified = None
    if rank == 0:
        # the one-GPU stream of the same text on the same session (round 3 took it from a fresh session
        # to dodge a fault whose cause, 2^32+ work-item launches past 2^26 sync positions, is fixed:
        # DESIGN.md 8), both streams checked against the text in HBM (lz77sss_session_verify)
        bad_sharded = sess.verify() if world == 1 else None
        t_1 = time.perf_counter()
        z1 = sess.factorize(device=local_rank)
        print(f"[bench --shard] one-GPU factorize {time.perf_counter() - t_1:.2f} s, z={z1}", file=sys.stderr,
              flush=True)
        ref = torch.empty(max(z1, 1) * 2, dtype=torch.int64 if pos64 else torch.int32, device=f"cuda:{local_rank}")
        if z1:
            sess.copy_factors(ref.data_ptr(), z1 * (16 if pos64 else 8))
        same = bool(z1 == z and torch.equal(ref[: 2 * z1].view(-1, 2), F))
        verified = {"one_gpu_stream_bad_positions": int(sess.verify()),
                    "sharded_stream_bad_positions": None if bad_sharded is None else int(bad_sharded)}
    if rank == 0:
        if chr19:
            data = "synthetic chr19-style (59 MiB ACGT base block, 0.1% mutations per copy), generated in HBM"
        elif args.workload == "rr":
            data = "synthetic (seeded restatement of the reference's random_repetitive_string)"
        else:
            data = "synthetic (genome-like: 64 MiB ACGT base block, 0.1% mutations)"
        out = {
            "metric": "factorization MB/s (3-aprx LZ77, greedy + lpf_opt, tau=512)",
            "value": round(n / dt / 1e6, 2), "unit": "MB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt * 1e3, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "u8", "data": data,
            "config": {"workload": (f"chr19 n={n} ({args.size_gib} GiB)" if chr19 else
                                    f"{args.workload} n={n} ({args.size_mib} MiB)") +
                       f", ONE text split over {world} rank(s), pos_t={'uint64' if pos64 else 'uint32'}",
                       "n": n, "tau": 512, "phr_mode": "lpf_opt", "fact_mode": "greedy",
                       "parallelism": f"sharded x{world}: S by block + all-gather, replicated phrases, "
                                      f"rank-ordered greedy blocks (speculative blocks opt-in: "
                                      f"LZ77SSS_SPECULATE=1), gathered emission",
                       "factors": z, "equals_one_gpu_stream": same, "verify_in_hbm": verified,
                       "sss_size": int(st[0]) if st else None, "lpf_phrases": int(st[2]) if st else None,
                       "text_gen_s": round(t_gen, 3), "rank0_phase_ms": phases,
                       "rank0_phase_mem_gib": {"note": "per phase: the session's device buffers when the phase was "
                                                       "enqueued (held) and their peak in it (peak), text excluded; "
                                                       "the GPU's free memory then (hbm_free)", **mem}},
            "roofline": None, "cpu_baseline": None,
        }
        if chr19 and world == 1 and not args.no_cpu_baseline:
            sess.close()  # (the host copy of the sample needs no device memory; free it anyway)
            sess = None
            out["cpu_baseline"] = cpu_baseline_chr19(lz, args.cpu_sample_mib << 20 if args.cpu_sample_mib > 0
                                                     else CHR19_SAMPLE_N)
        print(json.dumps(out), flush=True)
    if sess is not None:
        sess.close()
    if dist is not None:
        dist.destroy_process_group()


def main_sss(args, lz, torch, dist, world, rank, local_rank):
    """configs[3]'s sharded pass: the sync set (pos_t = uint64_t) of one chr19-style text of
    --size-gib GiB split over the ranks (lz77-sss_amd/sharded.py).  Each rank generates its
    block plus the 2tau-1 halo directly in HBM; one step = S n block on every rank + the
    rank-ordered all-gather of the blocks (RCCL when N > 1).  Total work is fixed: strong
    scaling."""
    import sharded

    n = int(args.size_gib * GIB)
    base_len = 59 << 20  # chr19-sized random ACGT "chromosome", 0.1% mutations per copy
    b, e = sharded.partition(n, world)[rank]
    lo, hi = sharded.block_bytes(n, b, e)
    sess = lz.Session(max(hi - lo, 1), device=local_rank)
    sess.gen_genome(hi - lo, base_len, 0.001, 7, offset=lo)
    gathered = [None]

    def step():
        cnt, runs = sess.sss_range(0, e - b, base=b) if e > b else (0, False)
        if dist is None:
            return cnt
        out = torch.empty(max(cnt, 1), dtype=torch.int64, device=f"cuda:{local_rank}")
        if cnt:
            sess.copy_sync_set64(out.data_ptr(), cnt)
        gathered[0] = sharded.gather_blocks(out[:cnt])
        return int(gathered[0].numel())

    for _ in range(args.warmup):
        step()

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    barrier()
    t0 = time.perf_counter()
    total = 0
    for _ in range(args.steps):
        total = step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier()
    dt = (t1 - t0) / args.steps
    if dist is not None:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    kms, kbytes = sess.sss_kernel_time()
    if dist is not None and gathered[0] is not None:
        g = gathered[0]
        ok = bool(g.numel() < 2 or bool((g[1:] > g[:-1]).all().item()))
    else:
        ok = True
    if rank == 0:
        achieved = kbytes / (kms * 1e-3) / 1e9 if kms > 0 else 0.0
        out = {
            "metric": "sync-set pass MB/s (pos_t=uint64, sharded by text block, tau=512)",
            "value": round(n / dt / 1e6, 2), "unit": "MB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt * 1e3, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic chr19-style (59 MiB ACGT base block, 0.1% mutations per copy), generated in HBM",
            "config": {"workload": f"chr19-style n={n} ({args.size_gib} GiB) split over {world} rank(s), pos_t=uint64",
                       "n": n, "tau": 512, "sss_size": int(total),
                       "sss_over_2n_tau": round(total / (2 * n / 512), 4),
                       "parallelism": f"text blocks x{world} + RCCL all-gather" if world > 1 else "single GPU",
                       "gathered_sorted": ok},
            "roofline": {"kernel": "k_sss_stream (per window launch, averaged)", "bound": "hbm", "achieved": round(achieved, 2),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": None, "algorithmic_bytes_per_launch": int(kbytes),
                         "avg_launch_ms": round(kms, 4)},
            "cpu_baseline": None,
        }
        print(json.dumps(out), flush=True)
    sess.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
