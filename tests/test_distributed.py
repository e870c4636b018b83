"""world_size-2 gloo test of bench.py's multi-rank path: independent texts per rank (no data-path
collective), max-over-ranks step time and the whole-job aggregate."""
from __future__ import annotations

import os
import socket
import sys

import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "lz77-sss_amd"))
    import bench
    import lz77sss

    T = bench.make_text(lz77sss, "rr", 1 << 16, rank)
    dt, value = bench.aggregate(0.5 + rank, 1 << 20, world, dist, device="cpu")
    q.put((rank, dt, value, int(T[:4096].sum())))
    dist.destroy_process_group()


def test_bench_aggregate_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    (_, dt0, v0, h0), (_, dt1, v1, h1) = res
    assert dt0 == dt1 == 1.5                      # max over ranks
    assert abs(v0 - 2 * (1 << 20) / 1.5 / 1e6) < 1e-9 and v0 == v1
    assert h0 != h1                               # each rank factorizes its own text
