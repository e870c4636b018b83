"""Sharded sync set over the ranks of one node (collective (1)).

The decisions of the text are split into contiguous blocks, one per rank.  Rank r
holds only T[b_r, e_r + 2tau - 1) -- its block plus the 2tau - 1 byte halo that the
last decision of the block reads -- computes S n [b_r, e_r) on its GPU
(Session.sss_range with base = b_r, pos_t = uint64_t), and the blocks are
all-gathered in rank order: the counts first, then the positions padded to the
largest count.  Phi and Q depend on window contents only, so the concatenation is
the sync set of T and the halo replaces any boundary exchange.

Backend "nccl" (RCCL over xGMI) gathers GPU to GPU from the session's HBM result;
"gloo" goes through host memory (the CPU tests, or several ranks sharing a GPU).
The per-block compute is injectable so the CPU tests can drive the same
partition/gather logic with the oracle as the block function.
"""
from __future__ import annotations

from typing import Callable

import numpy as np

TAU = 512
ALIGN = 4096  # block starts stay 4096-aligned (aligned text views on the device)


def num_decisions(n: int, tau: int = TAU) -> int:
    """Decisions i in [0, n - 2tau] (lce_sss.hpp:53, the K&K definition of DESIGN.md 4.1)."""
    return n - 2 * tau + 1 if n >= 2 * tau else 0


def partition(n: int, world: int, tau: int = TAU, align: int = ALIGN) -> list[tuple[int, int]]:
    """Contiguous decision blocks [b_r, e_r), one per rank (trailing ranks may be empty)."""
    d = num_decisions(n, tau)
    blk = -(-d // world) if world else d
    blk = -(-blk // align) * align if blk else 0
    return [(min(d, r * blk), min(d, (r + 1) * blk)) for r in range(world)]


def block_bytes(n: int, b: int, e: int, tau: int = TAU) -> tuple[int, int]:
    """Text bytes [lo, hi) a rank needs for decisions [b, e): the block and its halo."""
    if e <= b:
        return b, b
    return b, min(n, e + 2 * tau - 1)


def hip_block(text, b: int, e: int, n: int, device: int = 0, window: int = 0, keep_on_device: bool = False):
    """S n [b, e) on `device` through the C-ABI; returns (positions, has_runs).

    `text` is the whole text (host array) or a callable fill(session, offset, length)
    that materialises bytes [offset, offset + length) in the session (e.g.
    Session.gen_genome).  With keep_on_device the positions come back as an int64
    torch tensor on the device (for an RCCL gather), else as a uint64 numpy array."""
    import lz77sss as L

    lo, hi = block_bytes(n, b, e)
    with L.Session(max(hi - lo, 1), device) as s:
        if callable(text):
            text(s, lo, hi - lo)
        else:
            s.load(np.ascontiguousarray(text[lo:hi]))
        cnt, runs = s.sss_range(0, e - b, base=b, window=window) if e > b else (0, False)
        if keep_on_device:
            import torch

            out = torch.empty(max(cnt, 1), dtype=torch.int64, device=f"cuda:{device}")
            if cnt:
                s.copy_sync_set64(out.data_ptr(), cnt)
            return out[:cnt], runs
        return s.sync_set64(cnt), runs


def gather_blocks(local, group=None):
    """All-gather variable-length int64 blocks in rank order (torch.distributed)."""
    import torch
    import torch.distributed as dist

    dev = local.device
    world = dist.get_world_size(group)
    cnt = torch.tensor([local.numel()], dtype=torch.int64, device=dev)
    cnts = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(cnts, cnt, group=group)
    cnts = [int(c.item()) for c in cnts]
    m = max(max(cnts), 1)
    pad = torch.zeros(m, dtype=torch.int64, device=dev)
    pad[: local.numel()] = local
    parts = [torch.empty(m, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(parts, pad, group=group)
    return torch.cat([p[:c] for p, c in zip(parts, cnts)])


def sss_sharded(text, n: int, rank: int, world: int, device: int | None = None,
                compute: Callable | None = None, group=None, window: int = 0):
    """The sync set of T (uint64 numpy array) and has_runs, computed block-wise on
    `world` ranks and all-gathered.  Call on every rank of the process group.

    compute(text, b, e, n) -> (uint64 positions of S n [b, e), has_runs) defaults to
    the HIP path on `device` (fails loudly if the library or the GPU is missing)."""
    import torch
    import torch.distributed as dist

    b, e = partition(n, world)[rank]
    nccl = dist.is_initialized() and dist.get_backend(group) == "nccl"
    if compute is None:
        dev = rank if device is None else device
        local, runs = hip_block(text, b, e, n, device=dev, window=window, keep_on_device=nccl)
        if not nccl:
            local = torch.from_numpy(local.astype(np.int64))
    else:
        pos, runs = compute(text, b, e, n)
        local = torch.from_numpy(np.asarray(pos, dtype=np.uint64).astype(np.int64))
        if nccl:
            local = local.to(f"cuda:{rank if device is None else device}")
    if world == 1 or not dist.is_initialized():
        allp = local
        any_runs = bool(runs)
    else:
        allp = gather_blocks(local, group)
        flag = torch.tensor([1 if runs else 0], dtype=torch.int64, device=local.device)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
        any_runs = bool(flag.item())
    return allp.cpu().numpy().astype(np.uint64), any_runs
