"""Sharded sync set and sharded 3-approximation over the ranks of one node.

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


# ---------------------------------------------------------------------------
# Sharded 3-approximation (SURVEY.md 8e collectives (1)-(4)).
#   (1) S by text block on every rank + all-gather (sss_sharded above);
#   (2) SA_S / LCP / LCE and the LPF phrases replicated on every rank from the
#       gathered S (lz77sss_session_prepare with external_sss);
#   (3) the greedy chain block by block in rank order: rank r receives the exact
#       chain state and the carried table (last insert per gap-index slot before its
#       block) from rank r - 1, walks its block, sends both on;
#   (4) the blocks' factors gathered to every rank in rank order.
# The concatenation is bit-identical to a one-GPU factorization of the whole text.
TAIL_GUARD = 4160  # a non-last chain block ends at or below n - 4160 (greedy.hip)


def chain_bounds(n: int, world: int, tau: int = TAU) -> list[int]:
    """g_0 = 0 <= g_1 <= ... <= g_world = n: the chain blocks [g_r, g_{r+1}) (the sync-set
    blocks' starts, clamped so a non-last block ends at or below n - 4160)."""
    parts = partition(n, world, tau)
    lim = n - TAIL_GUARD if n > TAIL_GUARD else 0
    inner = [min(b, lim) for b, _ in parts[1:]]
    return [0] + inner + [n]


class HipBlocks:
    """Block compute on one device through the C-ABI (a session holding the whole text)."""

    def __init__(self, text, n: int, device: int = 0, pos64: bool = False, **params):
        import lz77sss as L

        self.L = L
        self.params = params
        self.s = L.Session(max(n, 1), device, pos64=pos64)
        if callable(text):
            text(self.s, 0, n)
        else:
            self.s.load(np.ascontiguousarray(text))
        self.table_bytes = 0

    def prepare(self, S, runs: bool) -> int:
        self.s.set_sss(S, runs)
        self.table_bytes = self.s.prepare(external_sss=True, **self.params)
        return self.table_bytes

    def run(self, state, end: int, table):
        start, idxpos, zmask = state
        if table is not None:
            self.s.carried_set(table)
        z, ex = self.s.greedy_block(start, idxpos, zmask, table is not None, end, **self.params)
        F = self.s.factors(z).astype(np.uint64)
        return F, ex, self.s.carried_get(self.table_bytes)

    def close(self):
        self.s.close()


def _send_bytes(arr: np.ndarray, dst: int, device=None, group=None):
    import torch
    import torch.distributed as dist

    t = torch.from_numpy(np.ascontiguousarray(arr).view(np.uint8).copy())
    n = torch.tensor([t.numel()], dtype=torch.int64)
    if device is not None:
        t, n = t.to(device), n.to(device)
    dist.send(n, dst, group=group)
    if t.numel():
        dist.send(t, dst, group=group)


def _recv_bytes(src: int, device=None, group=None) -> np.ndarray:
    import torch
    import torch.distributed as dist

    n = torch.zeros(1, dtype=torch.int64, device=device)
    dist.recv(n, src, group=group)
    t = torch.empty(int(n.item()), dtype=torch.uint8, device=device)
    if t.numel():
        dist.recv(t, src, group=group)
    return t.cpu().numpy()


def factorize_sharded(text, n: int, rank: int, world: int, device: int | None = None, blocks=None, group=None,
                      sss_compute: Callable | None = None, timings: dict | None = None):
    """The 3-approximation of T (uint64 (z, 2) factors, on every rank) computed with `world`
    ranks.  `blocks` (HipBlocks, or the tests' oracle form with the same interface) holds the whole text; defaults to HipBlocks
    on `device` (rank if None).  Call on every rank of the process group."""
    import time

    import torch
    import torch.distributed as dist

    dev = rank if device is None else device
    nccl = dist.is_initialized() and dist.get_backend(group) == "nccl"
    comm_dev = f"cuda:{dev}" if nccl else None
    t0 = time.perf_counter()
    # (1) sharded sync set
    S, runs = sss_sharded(text, n, rank, world, device=dev, compute=sss_compute, group=group)
    t1 = time.perf_counter()
    # (2) replicated phrases
    if blocks is None:
        blocks = HipBlocks(text, n, device=dev)
    blocks.prepare(S, runs)
    t2 = time.perf_counter()
    # (3) rank-ordered greedy chain
    g = chain_bounds(n, world)
    if rank == 0:
        state, table = (0, 0, 0), None
    else:
        st = _recv_bytes(rank - 1, comm_dev, group).view(np.uint64)
        state = (int(st[0]), int(st[1]), int(st[2]))
        table = _recv_bytes(rank - 1, comm_dev, group)
        if table.size == 0:  # no block before this one ran: nothing inserted yet
            table = None
    # walk only while the chain has not passed this block: g[world] == n, so a chain that an earlier
    # block's last factor carried to n (a text ending in a long repeat) ends without a last walk
    if state[0] < g[rank + 1]:
        F, ex, table = blocks.run(state, g[rank + 1], table)
    else:  # an earlier block's last factor covered this whole block: pass the state on
        F, ex = np.zeros((0, 2), np.uint64), state
    if rank + 1 < world:
        _send_bytes(np.array(ex, np.uint64), rank + 1, comm_dev, group)
        _send_bytes(table if table is not None else np.zeros(0, np.uint8), rank + 1, comm_dev, group)
    t3 = time.perf_counter()
    # (4) emission: the blocks' factors in rank order
    if world > 1 and dist.is_initialized():
        flat = torch.from_numpy(F.reshape(-1).astype(np.int64))
        if nccl:
            flat = flat.to(comm_dev)
        allf = gather_blocks(flat, group).cpu().numpy().astype(np.uint64).reshape(-1, 2)
    else:
        allf = F.reshape(-1, 2)
    if timings is not None:
        timings.update(sss=t1 - t0, prepare=t2 - t1, greedy_chain=t3 - t2, emit=time.perf_counter() - t3)
    return allf


def spec_parts() -> int:
    """Parts of a speculative block (LZ77SSS_SPEC_PARTS, 1..16, default 8): each is
    confirmed on its own, so a difference late in the block costs only the parts from there on."""
    import os

    return max(1, min(16, int(os.environ.get("LZ77SSS_SPEC_PARTS", "8"))))


def spec_lead(n: int, g: list[int], rank: int) -> int:
    """Lead-in length of rank `rank`'s speculative block: a third of its block, at
    least 64 MiB, at most everything before it (LZ77SSS_SPEC_LEAD overrides, for the tests)."""
    import os

    env = os.environ.get("LZ77SSS_SPEC_LEAD")
    lead = int(env) if env else max(64 << 20, (g[rank + 1] - g[rank]) // 3)
    return max(1, min(lead, g[rank]))


def factorize_sharded_resident(sess, n: int, rank: int, world: int, device: int, group=None,
                               timings: dict | None = None, speculate: bool | None = None, **params):
    """Collectives (1)-(4) with everything in HBM: `sess` is a Session on `device` holding the
    whole text (every rank loads it; phrases are replicated), pos_t = uint32_t or, for texts
    past 4 GiB (configs[3]), uint64_t (Session(pos64=True); the reference's choice at
    cli/lz77_sss_3_aprx.cpp:73-83).  Returns the factors as an int32 (uint32 session) or int64
    (uint64 session) (z, 2) torch tensor on `device`, identical on every rank.

    With backend "nccl" the sync-set blocks, the chain state, the carried table and the
    factor blocks move GPU to GPU (RCCL over xGMI); with "gloo" they go through host
    memory (several ranks sharing a GPU in the tests).  The session's own stream is
    synchronized before any buffer changes hands, and torch's current stream before the
    session reads a received buffer."""
    import os
    import time

    import torch
    import torch.distributed as dist

    multi = world > 1 and dist.is_initialized()
    nccl = multi and dist.get_backend(group) == "nccl"
    dev = torch.device("cuda", device)
    cdev = dev if nccl else torch.device("cpu")

    def ready():  # received device buffers are complete before the session stream reads them
        torch.cuda.current_stream(dev).synchronize()

    t0 = time.perf_counter()
    # (1) S n [b_r, e_r) on this rank, all-gathered in rank order
    b, e = partition(n, world)[rank]
    cnt, runs = sess.sss_range(b, e) if e > b else (0, False)
    local = torch.empty(max(cnt, 1), dtype=torch.int64, device=dev)
    if cnt:
        sess.copy_sync_set64(local.data_ptr(), cnt)
    local = local[:cnt]
    if multi:
        S = gather_blocks(local.to(cdev), group)
        flag = torch.tensor([1 if runs else 0], dtype=torch.int64, device=cdev)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
        runs = bool(flag.item())
        S = S.to(dev)
    else:
        S = local
    ready()
    sess.set_sss(S.numel(), runs, device_ptr=S.data_ptr())
    t1 = time.perf_counter()
    # (2) replicated SA_S / LCP / LPF phrases
    tab_bytes = sess.prepare(external_sss=True, **params)
    t2 = time.perf_counter()
    if timings is not None and hasattr(sess, "phase_mem"):
        timings["mem_prepare"] = sess.phase_mem()
    # (3) the greedy chain.  With speculation (world > 1) every rank r > 0 first walks its block
    # concurrently from a speculated entry: a lead-in walk of the text before g_r from a table
    # of the gap positions before it gives the chain state at the first hand-over point >= g_r
    # and the table of the inserts before it; the block then runs as consecutive parts, the
    # slots each part's lookups take from that table tracked.  In rank order, the true (state,
    # table) from r - 1 confirms the leading parts whose used slots all agree (given an equal
    # state); the rest of the block is walked again from the exit state of the last confirmed
    # part, with their writes over the true table, exactly as without speculation.
    g = chain_bounds(n, world)
    if speculate is None:  # off by default; LZ77SSS_SPECULATE=1: lead-in, =2: ring
        speculate = {"1": True, "2": "ring"}.get(os.environ.get("LZ77SSS_SPECULATE", "0"), False)
    ring = speculate == "ring" and multi
    spec = bool(speculate) and multi and rank > 0 and g[rank] > 0
    t_spec = 0.0
    spec_state, parts = None, []  # parts: (entry state, exit state, factors)
    F0 = None  # ring: rank 0's block (its round-A walk is the true chain)
    state0 = None

    def take():  # the session's last factors, as a device tensor
        fb = sess.factor_bytes()
        F = torch.empty(max(fb // 8, 1), dtype=torch.int64, device=dev)
        if fb:
            sess.copy_factors(F.data_ptr(), fb)
        return F[: fb // 8]

    def table_out():  # the session's carried table as a device tensor (uint8 view)
        t = torch.empty(max(tab_bytes, 1), dtype=torch.uint8, device=dev)
        sess.carried_get(tab_bytes, device_ptr=t.data_ptr())
        return t

    wide = getattr(sess, "pos64", False)

    def as_pos(t):  # table bytes -> int64 positions + 1 (uint32 tables widened)
        return t.view(torch.int64) if wide else t.view(torch.int32).to(torch.int64) & 0xFFFFFFFF

    def as_bytes(v):
        return v.view(torch.uint8) if wide else v.to(torch.int32).view(torch.uint8)

    def send_state(st, tab):
        hdr = torch.tensor([st[0], st[1], st[2], 1], dtype=torch.int64, device=cdev)
        dist.send(hdr, rank + 1, group=group)
        dist.send(tab.to(cdev), rank + 1, group=group)

    def recv_state():
        hdr = torch.zeros(4, dtype=torch.int64, device=cdev)
        dist.recv(hdr, rank - 1, group=group)
        tab = torch.empty(max(tab_bytes, 1), dtype=torch.uint8, device=cdev)
        dist.recv(tab, rank - 1, group=group)
        if nccl:
            ready()
        return (int(hdr[0]), int(hdr[1]), int(hdr[2])), tab.to(dev)

    if ring:
        # round A (every rank at once): rank 0 walks its block exactly; rank r > 0 walks a lead-in
        # and its block from the lead-in's exit.  The prefix max over the ranks of the tables of
        # each block's own inserts (rank 0: its whole exit table), passed along the ranks, is the
        # speculated entry table of round B; the previous rank's round-A exit state its entry state
        ts = time.perf_counter()
        if rank == 0:
            st = (0, 0, 0)
            if g[1] > 0:
                _, st = sess.greedy_block(0, 0, 0, False, g[1], **params)
            state0, F0 = tuple(st), take()
            prefix = table_out()
            if world > 1:
                send_state(state0, prefix)
        else:
            st = (0, 0, 0)
            if g[rank] > 0:
                lead0 = g[rank] - spec_lead(n, g, rank)
                _, st = sess.greedy_block(lead0, lead0, 0, False, g[rank], seed=True, **params)
                st = tuple(st)
                if st[0] < g[rank + 1]:
                    _, st = sess.greedy_block(*st, True, g[rank + 1], **params)
                    st = tuple(st)
            mine = as_pos(table_out())
            own = torch.where(mine > g[rank], mine, torch.zeros_like(mine))  # inserts at or after g_r
            del mine
            spec_state, tin = recv_state()
            if rank + 1 < world:
                send_state(st, as_bytes(torch.maximum(as_pos(tin), own)))
            del own
            sess.carried_set(nbytes=tab_bytes, device_ptr=tin.data_ptr())
            del tin
        t_spec = time.perf_counter() - ts
    if spec:
        import lz77sss as L

        ts = time.perf_counter()
        if not ring:
            lead0 = g[rank] - spec_lead(n, g, rank)
            _, spec_state = sess.greedy_block(lead0, lead0, 0, False, g[rank], seed=True, **params)
        spec_state = st = tuple(spec_state)
        npart = spec_parts()
        for k in range(npart):
            e_k = g[rank + 1] if k == npart - 1 else g[rank] + (g[rank + 1] - g[rank]) * (k + 1) // npart
            if st[0] < e_k:
                try:
                    sess.spec_begin(len(parts), spec_state[0])
                except L.Lz77SssError as err:  # no HBM for another part snapshot: stop speculating
                    if err.code != L.ENOMEM:
                        raise
                    break
                _, st2 = sess.greedy_block(*st, True, e_k, **params)
                parts.append((st, tuple(st2), take()))
                st = tuple(st2)
        t_spec += time.perf_counter() - ts
    t_wait = time.perf_counter()
    state, carried = (0, 0, 0), False
    accepted = None  # speculation: the number of parts that stood
    if ring and rank == 0:
        state, carried = state0, True  # block 0 is done (round A)
    if rank > 0:
        hdr = torch.zeros(4, dtype=torch.int64, device=cdev)
        dist.recv(hdr, rank - 1, group=group)
        state, carried = (int(hdr[0]), int(hdr[1]), int(hdr[2])), bool(hdr[3])
        if carried:
            tab = torch.empty(max(tab_bytes, 1), dtype=torch.uint8, device=cdev)
            dist.recv(tab, rank - 1, group=group)
            if nccl:
                ready()
            if parts:
                same = state == spec_state
                accepted = sess.spec_resolve(nbytes=tab_bytes, parts=len(parts) if same else 0,
                                             device_ptr=tab.data_ptr())
                if timings is not None:
                    timings.update(spec_state_ok=same, spec_parts=len(parts))
                if accepted:
                    state = parts[accepted - 1][1]
            else:
                sess.carried_set(nbytes=tab_bytes, device_ptr=tab.data_ptr())
            del tab
    keep = [F for (_, _, F) in parts[: accepted or 0]]  # factors of the confirmed parts
    F_rest = F0
    if F0 is None and not (parts and accepted == len(parts)) and state[0] < g[rank + 1]:
        _, state = sess.greedy_block(*state, carried, g[rank + 1], **params)
        state, carried = tuple(state), True
        F_rest = take()
    if multi and rank + 1 < world:
        hdr = torch.tensor([state[0], state[1], state[2], int(carried)], dtype=torch.int64, device=cdev)
        dist.send(hdr, rank + 1, group=group)
        if carried:
            tab = torch.empty(max(tab_bytes, 1), dtype=torch.uint8, device=cdev)
            sess.carried_get(tab_bytes, device_ptr=tab.data_ptr())
            dist.send(tab, rank + 1, group=group)
            del tab
    t3 = time.perf_counter()
    if timings is not None:
        timings.update(spec_walk=t_spec, chain_wait=t3 - t_wait, spec_accepted=accepted)
        if hasattr(sess, "phase_mem"):
            timings["mem_greedy"] = sess.phase_mem()
    # (4) emission: the blocks' factors gathered in rank order
    blocks = keep + ([F_rest] if F_rest is not None else [])
    F = torch.cat(blocks) if blocks else torch.empty(0, dtype=torch.int64, device=dev)
    if multi:
        F = gather_blocks(F.to(cdev), group).to(dev)
    if timings is not None:
        timings.update(sss=t1 - t0, prepare=t2 - t1, greedy_chain=t3 - t2, emit=time.perf_counter() - t3)
    if getattr(sess, "pos64", False):
        return F.view(-1, 2)  # (src, len) as uint64 pairs; positions < 2^63
    return F.view(torch.int32).view(-1, 2)
