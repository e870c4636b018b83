"""Sharded / windowed sync set (pos_t = uint64_t, SURVEY.md section 8e collective (1)).

CPU: the block partition, the halo argument checked with the oracle itself (the sync
set of T[b, e + 2tau - 1) shifted by b is S n [b, e)), and the world_size-2 gloo
gather driven by the oracle as the block function.  GPU: windowed/ranged
build_sss_range against the one-shot pass, the sharded path through the C-ABI on
two ranks sharing the GPU, device text generation by offset, and a text past 2^32.
"""
from __future__ import annotations

import os
import socket
import sys

import numpy as np
import pytest

from conftest import ROOT

sys.path.insert(0, str(ROOT / "lz77-sss_amd"))
import sharded  # noqa: E402

TAU = 512


def _texts():
    import oracle

    rng = np.random.default_rng(5)
    yield "random", rng.integers(0, 256, 40000).astype(np.uint8)
    # runs (Q windows) straddling the block boundaries
    t = rng.integers(0, 4, 50000).astype(np.uint8) + 65
    t[8000:16000] = np.tile(np.frombuffer(b"ACGTTGCA" * 3, np.uint8), 8000 // 24 + 1)[:8000]
    t[20000:21500] = 67
    yield "runs", t
    yield "genome", _genome(60000)


def _genome(n):
    import lz77sss

    return lz77sss.gen_genome(n, 7000, 0.01, 3)


def test_partition_covers_decisions():
    for n in [0, 1000, 1023, 1024, 5000, 1 << 20, (1 << 20) + 12345]:
        for world in [1, 2, 3, 8]:
            parts = sharded.partition(n, world)
            d = sharded.num_decisions(n)
            assert len(parts) == world
            assert parts[0][0] == 0 and parts[-1][1] == d
            for (b0, e0), (b1, e1) in zip(parts, parts[1:]):
                assert e0 == b1
            for b, e in parts:
                assert b <= e and (b % sharded.ALIGN == 0 or b == d)
                lo, hi = sharded.block_bytes(n, b, e)
                if e > b:
                    assert lo == b and hi == min(n, e + 2 * TAU - 1)
                    assert hi - lo >= 2 * TAU  # the view has >= 1 decision


def _oracle_block(text, b, e, n):
    import oracle

    lo, hi = sharded.block_bytes(n, b, e)
    if e <= b:
        return np.zeros(0, np.uint64), False
    s, runs = oracle.sss(np.ascontiguousarray(text[lo:hi]))
    s = s.astype(np.uint64) + np.uint64(b)
    assert s.size == 0 or int(s[-1]) < e
    return s, runs


@pytest.mark.parametrize("world", [2, 3, 7])
def test_oracle_halo_blocks(world):
    import oracle

    for name, T in _texts():
        full, runs = oracle.sss(T)
        parts = [_oracle_block(T, b, e, T.size) for b, e in sharded.partition(T.size, world, align=256)]
        cat = np.concatenate([p[0] for p in parts]) if parts else np.zeros(0, np.uint64)
        assert np.array_equal(cat, full.astype(np.uint64)), name
        assert any(p[1] for p in parts) == runs, name


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q, use_gpu, T):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, str(ROOT / "lz77-sss_amd"))
    sys.path.insert(0, str(ROOT / "oracle"))
    sys.path.insert(0, str(ROOT / "tests"))
    import sharded as SH

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        if use_gpu:
            S, runs = SH.sss_sharded(T, T.size, rank, world, device=0)
        else:
            S, runs = SH.sss_sharded(T, T.size, rank, world, compute=_oracle_block)
        q.put((rank, S, runs))
    finally:
        dist.destroy_process_group()


def _run_ranks(world, use_gpu, T):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, use_gpu, T)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=180) for _ in procs), key=lambda x: x[0])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    return res


def test_gloo_two_ranks_oracle_blocks():
    import oracle

    T = dict(_texts())["runs"]
    full, runs = oracle.sss(T)
    res = _run_ranks(2, False, T)
    for _, S, r in res:
        assert np.array_equal(S, full.astype(np.uint64))
        assert r == runs


# ---------------------------------------------------------------- GPU
@pytest.mark.gpu
def test_sss_range_windows_match_one_shot(lz, orc):
    import lz77sss

    for name, T in _texts():
        with lz77sss.Session(T.size) as s:
            s.load(T)
            full, runs = s.sss()
            full = full.astype(np.uint64)
            for window in [4096, 8192, 12288, 0]:
                c, r = s.sss_range(window=window)
                assert np.array_equal(s.sync_set64(c), full), (name, window)
                assert r == runs
            # sub-ranges with unaligned bounds and a base offset
            d = sharded.num_decisions(T.size)
            for first, end in [(1, d), (777, 20001), (4096, 4097), (d - 5, d + 100), (0, 0)]:
                c, _ = s.sss_range(first, end, base=1 << 40, window=4096)
                want = full[(full >= first) & (full < min(end, d))] + np.uint64(1 << 40)
                assert np.array_equal(s.sync_set64(c), want), (name, first, end)


@pytest.mark.gpu
def test_sss_range_large_rr(lz, orc):
    import lz77sss

    T = lz77sss.gen_random_repetitive(1 << 22, 1 << 22, 9, 0.5, 0.05)
    with lz77sss.Session(T.size) as s:
        s.load(T)
        full, _ = s.sss()
        c, _ = s.sss_range(window=1 << 20)
        assert np.array_equal(s.sync_set64(c), full.astype(np.uint64))
    import oracle

    assert np.array_equal(oracle.sss(T)[0], full)


@pytest.mark.gpu
def test_sharded_two_ranks_on_gpu(lz, orc):
    import oracle

    T = dict(_texts())["runs"]
    full, runs = oracle.sss(T)
    for _, S, r in _run_ranks(2, True, T):
        assert np.array_equal(S, full.astype(np.uint64))
        assert r == runs


@pytest.mark.gpu
def test_gen_genome_blocks_and_past_4gib(lz, orc):
    import lz77sss

    n = (1 << 32) + (3 << 20) + 12345  # positions past 2^32: pos_t = uint64_t
    with lz77sss.Session(n) as s:
        s.gen_genome(n, 59 << 20, 0.001, 7)
        c1, _ = s.sss_range(window=1 << 30)
        S1 = s.sync_set64(c1)
        c2, _ = s.sss_range(window=(1 << 28) + 4096)
        S2 = s.sync_set64(c2)
        assert np.array_equal(S1, S2)
        assert S1.size > 0 and int(S1[-1]) > (1 << 32)
        assert np.all(np.diff(S1.astype(np.int64)) > 0)
        # |S| near 2n/tau for a random-like text
        assert 0.5 < S1.size / (2 * n / TAU) < 1.5
    # a block generated alone by offset equals the same range of the whole text
    b = (1 << 32) - (1 << 20)
    e = b + (2 << 20)
    with lz77sss.Session(e - b + 2 * TAU - 1) as s:
        s.gen_genome(e - b + 2 * TAU - 1, 59 << 20, 0.001, 7, offset=b)
        c, _ = s.sss_range(0, e - b, base=b)
        blk = s.sync_set64(c)
    want = S1[(S1 >= b) & (S1 < e)]
    assert np.array_equal(blk, want)


# ---------------------------------------------------------------- sharded 3-approximation
def test_chain_bounds():
    for n in [100, 5000, 100000, (1 << 20) + 7]:
        for world in [1, 2, 3, 8]:
            g = sharded.chain_bounds(n, world)
            assert len(g) == world + 1 and g[0] == 0 and g[-1] == n
            assert all(a <= b for a, b in zip(g, g[1:]))
            assert all(x <= n - sharded.TAIL_GUARD or x in (0, n) for x in g[1:-1])


def _fact_worker(rank, world, port, q, use_gpu, T, wide):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, str(ROOT / "lz77-sss_amd"))
    sys.path.insert(0, str(ROOT / "oracle"))
    sys.path.insert(0, str(ROOT / "tests"))
    import sharded as SH
    from oracle_blocks import OracleBlocks
    from test_sharded_sss import _oracle_block

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        if use_gpu:
            blocks = SH.HipBlocks(T, T.size, device=0, pos64=wide)
            F = SH.factorize_sharded(T, T.size, rank, world, device=0, blocks=blocks)
            blocks.close()
        else:
            blocks = OracleBlocks(T, T.size, pos64=wide)
            F = SH.factorize_sharded(T, T.size, rank, world, blocks=blocks, sss_compute=_oracle_block)
        q.put((rank, F))
    finally:
        dist.destroy_process_group()


def _run_fact_ranks(world, use_gpu, T, wide=False):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fact_worker, args=(r, world, port, q, use_gpu, T, wide)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=300) for _ in procs), key=lambda x: x[0])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("world,wide", [(2, False), (3, False), (2, True)])
def test_gloo_sharded_factorization_oracle_blocks(world, wide):
    """Collectives (1)-(4) on CPU ranks (gloo) with the oracle as the block compute: sharded
    sync set + all-gather, replicated phrases, the rank-ordered greedy chain with the carried
    gap-index table, rank-ordered emission == the one-process p = 1 stream."""
    import lz77sss
    import oracle

    T = lz77sss.gen_random_repetitive(60000, 60000, 11)
    F_ref = oracle.factorize64(T)[0] if wide else oracle.factorize(T)[0].astype(np.uint64)
    for _, F in _run_fact_ranks(world, False, T, wide):
        assert np.array_equal(F, F_ref)


def _tail_repeat_text(n: int = 60000):
    """A text whose second half is a copy of the first: the chain's last factor starts in the
    first rank's block and reaches n, so the last rank receives a state already at n."""
    import lz77sss

    h = lz77sss.gen_random_repetitive(n // 2, n // 2, 13)
    return np.concatenate([h, h])


def test_gloo_sharded_factorization_tail_repeat():
    """a last rank whose incoming chain state is already n must not walk (greedy_block
    rejects start >= end) -- the concatenation still equals the one-process stream."""
    import oracle

    T = _tail_repeat_text()
    F_ref = oracle.factorize(T)[0].astype(np.uint64)
    assert int(F_ref[-1, 1]) >= T.size // 2 - 64  # one factor covers (nearly) the whole copy
    for _, F in _run_fact_ranks(2, False, T):
        assert np.array_equal(F, F_ref)


def test_oracle_greedy_blocks_any_bounds():
    import lz77sss
    import oracle

    T = lz77sss.gen_genome(200000, 20000, 0.01, 4)
    F_ref = oracle.factorize(T)[0].astype(np.uint64)
    for bounds in [[0, T.size], [0, 5000, T.size], [0, 17000, 23000, 120000, T.size]]:
        st, tab, parts = (0, 0), None, []
        for r in range(len(bounds) - 1):
            F, st, tab = oracle.greedy_block(T, st[0], st[1], bounds[r + 1], tab)
            parts.append(F)
        assert np.array_equal(np.concatenate(parts), F_ref), bounds


@pytest.mark.gpu
@pytest.mark.parametrize("world,wide", [(2, False), (3, True)])
def test_sharded_factorization_ranks_on_gpu(lz, orc, world, wide):
    """The sharded 3-approximation through the C-ABI, ranks sharing the GPU (gloo between them)."""
    T = lz.gen_genome(3 << 20, 1 << 20, 0.001, 19)
    F_ref = orc.factorize64(T)[0] if wide else orc.factorize(T)[0].astype(np.uint64)
    for _, F in _run_fact_ranks(world, True, T, wide):
        assert F.shape == F_ref.shape and np.array_equal(F, F_ref)


@pytest.mark.gpu
@pytest.mark.parametrize("bounds_kind", ["two", "many"])
def test_greedy_blocks_one_session(lz, orc, bounds_kind):
    """lz77sss_session_greedy_block in sequence on one session == lz77sss_session_factorize."""
    T = lz.gen_genome(4 << 20, 1 << 20, 0.001, 29)
    n = T.size
    bounds = [0, n // 2, n] if bounds_kind == "two" else [0, 100000, 100001, 1 << 20, 3 << 20, n]
    F_ref = orc.factorize(T)[0]
    with lz.Session(n) as s:
        s.load(T)
        S, runs = s.sss()
        nb = s.prepare(external_sss=False)
        state, parts, tab = (0, 0, 0), [], None
        for b in bounds[1:]:
            if state[0] >= b and b < n:
                continue
            if tab is not None:
                s.carried_set(tab)
            z, ex = s.greedy_block(*state, tab is not None, b)
            parts.append(s.factors(z))
            tab = s.carried_get(nb)
            state = ex
    assert np.array_equal(np.concatenate(parts), F_ref)


def _resident_worker(rank, world, port, q, T, wide=False, gen=None, env=None, speculate=True):
    import hashlib

    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ.update(env or {})
    sys.path.insert(0, str(ROOT / "lz77-sss_amd"))
    import lz77sss as L
    import sharded as SH

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = T.size if gen is None else gen["n"]
        with L.Session(n, 0, pos64=wide) as s:
            if gen is None:
                s.load(T)
            else:  # generated in HBM (the seeded chr19-style generator)
                s.gen_genome(n, gen["base_len"], gen["mut"], gen["seed"])
            tm = {}
            F = SH.factorize_sharded_resident(s, n, rank, world, 0, timings=tm, speculate=speculate)
            if gen is None:
                # a second step on the same session
                F2 = SH.factorize_sharded_resident(s, n, rank, world, 0, speculate=speculate)
                q.put((rank, F.cpu().numpy().astype(np.uint64), bool(torch.equal(F, F2)), sorted(tm),
                       (tm.get("spec_accepted"), tm.get("spec_parts"))))
            else:  # the stream's SHA-256 in the fixture layout (little-endian uint64 pairs)
                h = hashlib.sha256(F.cpu().numpy().astype("<u8").view(np.uint8)).hexdigest()
                q.put((rank, int(F.shape[0]), h, sorted(tm), tm.get("spec_accepted"),
                       {k: (round(v, 3) if isinstance(v, float) else v) for k, v in tm.items()}))
    finally:
        dist.destroy_process_group()


def _run_resident(world, T, wide=False, gen=None, env=None, speculate=True):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    qq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_resident_worker, args=(r, world, port, qq, T, wide, gen, env, speculate))
             for r in range(world)]
    for p in procs:
        p.start()
    import queue
    import time

    got, t0 = [], time.time()
    while len(got) < world:  # a rank that dies fails the test instead of leaving the others waiting
        try:
            got.append(qq.get(timeout=5))
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            if dead or time.time() - t0 > 900:
                for p in procs:
                    p.kill()
                raise AssertionError(f"rank failed (exit codes {[p.exitcode for p in procs]})")
    res = sorted(got, key=lambda x: x[0])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    return res


@pytest.mark.gpu
@pytest.mark.parametrize("world,wide", [(1, False), (2, False), (3, False), (2, True)])
def test_sharded_resident_ranks_on_gpu(lz, orc, world, wide):
    """factorize_sharded_resident (the bench's --shard step: every buffer stays in HBM, handed
    over through the process group) == the one-process stream, on every rank, twice; also on
    pos_t = uint64_t sessions (configs[3])."""
    T = lz.gen_genome(3 << 20, 1 << 20, 0.001, 23)
    F_ref = orc.factorize64(T)[0] if wide else orc.factorize(T)[0].astype(np.uint64)
    for _, F, same, keys, _acc in _run_resident(world, T, wide):
        assert same and {"emit", "greedy_chain", "prepare", "sss"} <= set(keys)
        assert F.shape == F_ref.shape and np.array_equal(F, F_ref)


@pytest.mark.gpu
@pytest.mark.parametrize("speculate", [False, True])
def test_sharded_resident_tail_repeat(lz, orc, speculate):
    """ADVICE r3 on the device path: 2 ranks, the chain reaches n inside rank 0's block, so rank 1
    must not walk (with and without the speculative parts)."""
    T = _tail_repeat_text(1 << 20)
    F_ref = orc.factorize(T)[0].astype(np.uint64)
    for _, F, same, _keys, _acc in _run_resident(2, T, False, speculate=speculate):
        assert same and F.shape == F_ref.shape and np.array_equal(F, F_ref)


@pytest.mark.gpu
@pytest.mark.parametrize("world,lead,parts", [(2, None, None), (3, None, None), (2, 100000, None), (3, 4096, 3),
                                              (2, 1, None), (3, 30000, 1), (2, 200000, 16)])
def test_sharded_resident_speculative_blocks(lz, orc, world, lead, parts):
    """Speculative chain blocks: every rank > 0 walks its block, as consecutive
    parts, from a lead-in's exit state and table while the ranks before it work, and keeps the
    leading parts all of whose used carried slots agree with the true table (given the true
    state); the rest is re-walked.  The stream equals the one-process stream whatever the
    lead-in and the part count (a lead-in from position 0 -- the default on a text this short
    -- is the true chain, so every part must be accepted; short lead-ins may lose parts), and
    equals the non-speculative run."""
    T = lz.gen_genome(3 << 20, 1 << 20, 0.001, 29)
    F_ref = orc.factorize(T)[0].astype(np.uint64)
    env = {} if lead is None else {"LZ77SSS_SPEC_LEAD": str(lead)}
    if parts is not None:
        env["LZ77SSS_SPEC_PARTS"] = str(parts)
    res = _run_resident(world, T, False, env=env)
    for rank, F, same, keys, (acc, npart) in res:
        assert same and {"spec_walk", "chain_wait", "spec_accepted"} <= set(keys)
        assert F.shape == F_ref.shape and np.array_equal(F, F_ref)
        if rank > 0:
            assert npart is not None and 1 <= npart <= (parts or 8) and 0 <= acc <= npart
            if lead is None:
                assert acc == npart
    plain = _run_resident(world, T, False, speculate=False)
    assert all(np.array_equal(a[1], b[1]) for a, b in zip(res, plain))


@pytest.mark.gpu
@pytest.mark.parametrize("world,lead,parts", [(2, None, None), (3, None, None), (3, 100000, None), (4, 30000, 3),
                                              (3, 1, 1)])
def test_sharded_resident_ring_speculation(lz, orc, world, lead, parts):
    """Ring speculation: round A walks every block at once (rank 0 exactly, the others
    after a lead-in), the prefix max of the blocks' own-insert tables along the ranks is each rank's
    round-B entry table (the previous rank's round-A exit its entry state); round B's parts are then
    confirmed against the true table in rank order.  The stream equals the one-process stream and
    the non-speculative run whatever the lead-in and the part count; rank 1 (entered from rank 0's
    true exit) keeps every part."""
    T = lz.gen_genome(4 << 20, 1 << 20, 0.001, 37)
    F_ref = orc.factorize(T)[0].astype(np.uint64)
    env = {} if lead is None else {"LZ77SSS_SPEC_LEAD": str(lead)}
    if parts is not None:
        env["LZ77SSS_SPEC_PARTS"] = str(parts)
    res = _run_resident(world, T, False, env=env, speculate="ring")
    for rank, F, same, keys, (acc, npart) in res:
        assert same and {"spec_walk", "chain_wait", "spec_accepted"} <= set(keys)
        assert F.shape == F_ref.shape and np.array_equal(F, F_ref)
        if rank == 1:
            assert npart is not None and acc == npart


@pytest.mark.gpu
@pytest.mark.slow
@pytest.mark.parametrize("world,speculate", [(2, True), (3, "ring")])
def test_sharded_resident_u64_past_4gib_hash(world, speculate):
    """configs[3] at C4's mutation rate past 2^32: a 4 GiB + 3 MiB chr19-style text (0.1 %
    mutations, pos_t = uint64_t) factorized by 2 ranks (gloo, sharing the GPU) with
    factorize_sharded_resident == the oracle's stream (SHA-256 fixture of
    tests/golden/make_stream_hashes.py, entry chr19_4gib_u64) on both ranks."""
    import json

    e = json.loads((ROOT / "tests" / "golden" / "stream_hashes.json").read_text())["chr19_4gib_u64"]
    gen = dict(n=e["n"], base_len=e["args"]["base_len"], mut=e["args"]["mut"], seed=e["args"]["seed"])
    for rank, z, h, keys, acc, tm in _run_resident(world, np.zeros(0, np.uint8), True, gen, speculate=speculate):
        print(f"rank {rank}: speculation {speculate}: accepted={acc} times={tm}")
        assert {"emit", "greedy_chain", "prepare", "sss"} <= set(keys)
        assert z == e["z"] and h == e["stream_sha256"]


def _plain_after_sharded_worker(q, wide, window):
    # (its own process, as the rank workers: the pytest process's HIP state stays out of it)
    import torch

    sys.path.insert(0, str(ROOT / "lz77-sss_amd"))
    import lz77sss as L
    import sharded as SH

    torch.zeros(1, device="cuda")
    T = L.gen_genome(6 << 20, 1 << 20, 0.001, 31)
    n = T.size
    with L.Session(n, 0, pos64=wide) as s:
        s.load(T)
        F1 = SH.factorize_sharded_resident(s, n, 0, 1, 0).cpu().numpy().astype(np.uint64)
        if window:
            os.environ["LZ77SSS_GREEDY_WINDOW"] = window
        z = s.factorize()
        F2 = np.asarray(s.factors(z)).astype(np.uint64)
        os.environ.pop("LZ77SSS_GREEDY_WINDOW", None)
        F3 = SH.factorize_sharded_resident(s, n, 0, 1, 0).cpu().numpy().astype(np.uint64)
    q.put((T, F1, F2, F3))


@pytest.mark.gpu
@pytest.mark.parametrize("wide,window", [(False, None), (True, None), (False, "1048576"), (True, "1048576")])
def test_plain_factorize_after_sharded_same_session(lz, orc, wide, window):
    """A session that ran the resident sharded path (world 1: sss_range, set_sss, prepare,
    greedy_block) and then a plain factorize -- also in greedy windows, the form a 50 GiB text
    takes -- and the sharded path again: all three streams equal the oracle's."""
    import queue

    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    qq = ctx.Queue()
    p = ctx.Process(target=_plain_after_sharded_worker, args=(qq, wide, window))
    p.start()
    try:
        T, F1, F2, F3 = qq.get(timeout=150)
    except queue.Empty:
        p.kill()
        raise AssertionError(f"worker failed (exit code {p.exitcode})")
    p.join(60)
    assert p.exitcode == 0
    F_ref = orc.factorize64(T)[0] if wide else orc.factorize(T)[0].astype(np.uint64)
    for F in (F1, F2, F3):
        assert F.shape == F_ref.shape and np.array_equal(F, F_ref)
