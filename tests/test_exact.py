"""Exact mode (factorize_exact, lz77_sss.hpp:188-200): canonical greedy LZ77.

The reference's own tests check its exact modes only by decode(factorize(T)) == T
(tests/test_lz77_sss.cpp:95-133).  Here the lengths are pinned harder: the
oracle's exact restatement is checked against a brute-force longest-previous-
factor parse; the sample-index path (transf_mode naive / with_samples /
without_samples, csrc/smpl.hip) must give the oracle's lengths with valid sources,
and FULL_SA (csrc/exact.hip) the oracle's stream bit for bit (lengths and the
PSV/NSV source rule).  Sources are not the reference's (its PA / SA tie order comes
from an unstable parallel sort): "parity unpinned" for sources, pinned by
definition for lengths.
"""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

from conftest import golden_names, load_golden


def brute_force_lengths(T):
    t = bytes(T)
    n, p, out = len(t), 0, []
    while p < n:
        best = 0
        for j in range(p):
            k = 0
            while p + k < n and t[j + k] == t[p + k]:
                k += 1
            best = max(best, k)
        out.append(best)
        p += max(1, best)
    return out


def check_valid(T, F):
    ln = F[:, 1].astype(np.int64)
    pos = np.concatenate([[0], np.cumsum(np.maximum(ln, 1))[:-1]])
    assert pos[-1] + max(ln[-1], 1) == T.size
    lit = ln == 0
    assert np.array_equal(F[lit, 0].astype(np.uint8), T[pos[lit]])
    assert np.all(F[~lit, 0].astype(np.int64) < pos[~lit])


@pytest.mark.parametrize("seed,sigma,n", [(1, 2, 400), (2, 3, 500), (3, 4, 600), (4, 26, 700), (5, 1, 300)])
def test_oracle_exact_lengths_are_longest_previous_factors(orc, seed, sigma, n):
    rng = np.random.Generator(np.random.PCG64(seed))
    T = rng.integers(0, sigma, n, dtype=np.uint8)
    T[n // 3:n // 3 + 120] = np.tile(T[:7], 18)[:120]  # a run and a long repeat
    F = orc.factorize_exact(T)
    assert [int(x) for x in F[:, 1]] == brute_force_lengths(T)
    check_valid(T, F)
    assert np.array_equal(orc.decode(F, T.size), T)


@pytest.mark.parametrize("name", ["c1_seed1", "c1_seed2", "periodic", "genome_small", "binary_30k", "zeros_10k",
                                  "edge_n1", "edge_n2", "edge_n1025"])
def test_oracle_exact_golden(orc, name):
    g = load_golden(name)
    F = orc.factorize_exact(g["text"])
    assert np.array_equal(F, g["factors_exact"])
    assert np.array_equal(orc.decode(F, g["text"].size), g["text"])


@pytest.mark.parametrize("name", ["c1_seed1", "periodic", "genome_small"])
def test_exact_never_longer_than_approx(name):
    """The exact parse is optimal among greedy parses: never more factors than the 3-approximation."""
    g = load_golden(name)
    assert g["factors_exact"].shape[0] <= g["factors"].shape[0]


SMPL_FIXTURES = ["c1_seed1", "c1_seed2", "c1_seed4", "periodic", "genome_small", "binary_30k", "zeros_10k",
                 "edge_n1", "edge_n2", "edge_n511", "edge_n1025", "edge_n5000"]


@pytest.mark.parametrize("transf_mode", [1, 2])
@pytest.mark.parametrize("name", SMPL_FIXTURES)
def test_oracle_exact_smpl_restatement(orc, name, transf_mode):
    """The restatement of the reference's transform (oracle_exact.hpp) at p = 1: one section, so
    its lengths are the canonical greedy ones (pinned by brute force above), and it decodes."""
    g = load_golden(name)
    F = orc.factorize_exact_smpl(g["text"], transf_mode, 1)
    assert np.array_equal(F[:, 1], g["factors_exact"][:, 1])
    check_valid(g["text"], F)
    assert np.array_equal(orc.decode(F, g["text"].size), g["text"])


@pytest.mark.parametrize("seed", [1, 5, 9, 13])
def test_oracle_exact_smpl_c1_seeds(orc, lz, seed):
    T = lz.gen_random_repetitive(10000, 200000, seed)
    F_ref = orc.factorize_exact(T)
    for tm in (1, 2):
        F = orc.factorize_exact_smpl(T, tm, 1)
        assert np.array_equal(F[:, 1], F_ref[:, 1])
        check_valid(T, F)


@pytest.mark.parametrize("p", [2, 3, 8])
@pytest.mark.parametrize("name", ["binary_30k", "genome_small", "c1_seed1"])
def test_oracle_exact_smpl_sections(orc, name, p):
    """At p > 1 the reference splits the parse into 16 p sections that restart the greedy parse
    (common.cpp:48-75; every extension stops at its section end e, with_samples.cpp:50-53): a
    valid parse, never shorter than the canonical one."""
    g = load_golden(name)
    for tm in (1, 2):
        F = orc.factorize_exact_smpl(g["text"], tm, p)
        check_valid(g["text"], F)
        assert np.array_equal(orc.decode(F, g["text"].size), g["text"])
        assert F.shape[0] >= g["factors_exact"].shape[0]


def run_exact(session, T, **kw):
    s = session(max(T.size, 1))
    s.load(T)
    z = s.factorize_exact(**kw)
    return s, s.factors(z)


def check_exact(lz, T, F, F_ref):
    """Exact-smpl stream: the canonical lengths (the oracle's), valid sources, decodes to T."""
    assert F.shape == F_ref.shape
    assert np.array_equal(F[:, 1], F_ref[:, 1])
    check_valid(T, F)
    if T.size:
        ln = F[:, 1].astype(np.int64)
        pos = np.concatenate([[0], np.cumsum(np.maximum(ln, 1))[:-1]])
        cp = ln > 0
        # every copy's source is an earlier occurrence (checked by decoding)
        assert np.array_equal(lz.decode(F, T.size), T)
        assert np.all(F[cp, 0].astype(np.int64) < pos[cp])


SMPL_MODES = [0, 1, 2]  # naive, with_samples, without_samples (lz77_sss.hpp:60-64)


@pytest.mark.gpu
@pytest.mark.parametrize("name", golden_names())
def test_gpu_exact_golden(session, name):
    """FULL_SA (LPF over the full suffix array): bit-exact with the oracle, sources included."""
    g = load_golden(name)
    _, F = run_exact(session, g["text"], transf_mode=3)
    assert np.array_equal(F, g["factors_exact"])


@pytest.mark.gpu
@pytest.mark.parametrize("transf_mode", SMPL_MODES)
@pytest.mark.parametrize("name", golden_names())
def test_gpu_exact_smpl_golden(session, lz, name, transf_mode):
    """The sample-index path (csrc/smpl.hip): the oracle's lengths on every fixture."""
    g = load_golden(name)
    _, F = run_exact(session, g["text"], transf_mode=transf_mode)
    check_exact(lz, g["text"], F, g["factors_exact"])


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(1, 17))
def test_gpu_exact_c1_seeds(session, orc, lz, seed):
    T = lz.gen_random_repetitive(10000, 200000, seed)
    F_ref = orc.factorize_exact(T)
    _, F = run_exact(session, T, transf_mode=3)
    assert np.array_equal(F, F_ref)
    for tm in SMPL_MODES:
        _, F = run_exact(session, T, transf_mode=tm)
        check_exact(lz, T, F, F_ref)


@pytest.mark.gpu
@pytest.mark.parametrize("transf_mode", SMPL_MODES + [3])
def test_gpu_exact_transform_modes_agree(session, orc, lz, transf_mode):
    T = lz.gen_random_repetitive(50000, 120000, 77)
    _, F = run_exact(session, T, transf_mode=transf_mode)
    check_exact(lz, T, F, orc.factorize_exact(T))


@pytest.mark.gpu
def test_gpu_exact_smpl_structures(session, lz):
    """The sample set of common.cpp:34-88: delta = min(n / z_approx, 256), samples every delta
    characters at most (stats 24..27: samples, delta, phrase tasks, chunks << 32 | doubling levels);
    the chain's phrases are all tasks."""
    T = lz.gen_random_repetitive(200000, 200000, 5)
    s = session(T.size)
    s.load(T)
    za = s.factorize()
    for tm in SMPL_MODES:
        z = s.factorize_exact(transf_mode=tm)
        st = s.stats()
        c, delta = st[24], st[25]
        assert delta == min(T.size // za, 256)
        assert T.size // delta <= c <= T.size // delta + za + 1
        assert z > 0 and st[26] >= z and (st[27] >> 32) >= 1


@pytest.mark.gpu
@pytest.mark.parametrize("period", [1, 3, 170, 171, 600])
def test_gpu_exact_runs(session, orc, lz, period):
    rng = np.random.Generator(np.random.PCG64(period))
    unit = rng.integers(0, 256, period, dtype=np.uint8)
    T = np.concatenate([rng.integers(0, 256, 3000, dtype=np.uint8), np.tile(unit, 40000 // period + 1)[:40000],
                        rng.integers(0, 256, 2000, dtype=np.uint8)])
    F_ref = orc.factorize_exact(T)
    _, F = run_exact(session, T, transf_mode=3)
    assert np.array_equal(F, F_ref)
    for tm in SMPL_MODES:
        _, F = run_exact(session, T, transf_mode=tm)
        check_exact(lz, T, F, F_ref)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,mib", [("genome", 16), ("rr", 16)])
def test_gpu_exact_medium(session, orc, lz, kind, mib):
    n = mib << 20
    T = lz.gen_genome(n, 2 << 20, 0.001, 11) if kind == "genome" else lz.gen_random_repetitive(n, n, 5, 0.5, 0.05)
    F_ref = orc.factorize_exact(T)
    _, F = run_exact(session, T, transf_mode=3)
    assert F.shape == F_ref.shape and np.array_equal(F, F_ref)
    _, F = run_exact(session, T, transf_mode=2)
    check_exact(lz, T, F, F_ref)


@pytest.mark.gpu
@pytest.mark.parametrize("transf_mode", [1, 2])
def test_gpu_exact_smpl_64mib(session, lz, transf_mode):
    """exact-smpl on a 64 MiB repetitive text: the canonical lengths of FULL_SA (which equals the
    oracle bit for bit up to 16 MiB, test_gpu_exact_medium)."""
    n = 64 << 20
    T = lz.gen_random_repetitive(n, n, 9, 0.5, 0.05)
    _, F_ref = run_exact(session, T, transf_mode=3)
    _, F = run_exact(session, T, transf_mode=transf_mode)
    check_exact(lz, T, F, F_ref)


@pytest.mark.gpu
@pytest.mark.slow
def test_gpu_exact_smpl_one_gib(session, lz):
    """configs[4] at full size (1 GiB rr): exact-smpl lengths == FULL_SA lengths, decode == T."""
    n = 1 << 30
    T = lz.gen_random_repetitive(n, n, 42, 0.5, 0.05)
    # its own session: FULL_SA's 44 B x n are released before the next tests
    with lz.Session(n) as s:
        s.load(T)
        z = s.factorize_exact(transf_mode=3)
        F_ref = s.factors(z)
        z2 = s.factorize_exact(transf_mode=2)
        F = s.factors(z2)
        assert z2 == z and np.array_equal(F[:, 1], F_ref[:, 1])
        _, mism = s.decode(out=False)
        assert mism == 0


@pytest.mark.gpu
def test_gpu_exact_one_shot_callback(lz, orc):
    T = lz.gen_random_repetitive(150000, 150000, 8)
    got = []
    EMIT = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p)

    def emit(ptr, count, user):
        got.append(np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ctypes.c_uint32)), (count, 2)).copy())
        return 0

    cb = EMIT(emit)
    p = lz.params()
    for tm, exact_sources in [(lz.WITHOUT_SAMPLES, False), (3, True)]:
        got.clear()
        rc = lz.load_library().lz77sss_factorize_exact_u32(T.ctypes.data_as(ctypes.c_void_p), T.size,
                                                           ctypes.byref(p), tm, cb, None)
        assert rc == 0
        F = np.concatenate(got)
        if exact_sources:
            assert np.array_equal(F, orc.factorize_exact(T))
        else:
            check_exact(lz, T, F, orc.factorize_exact(T))


@pytest.mark.gpu
def test_gpu_exact_invalid_parameters(session, lz):
    T = lz.gen_random_repetitive(20000, 20000, 1)
    s = session(T.size)
    s.load(T)
    with pytest.raises(lz.Lz77SssError):
        s.factorize_exact(transf_mode=7)
    with pytest.raises(lz.Lz77SssError):
        s.factorize_exact(fact_mode=lz.SKIP_PHRASES)


def check_reference_stream(orc, session, T, modes=SMPL_MODES):
    """The device's whole exact-smpl stream, sources included, against the restatement of the
    reference's transform at p = 1 (oracle_exact.hpp): the source pass (k_ref_sources) picks the
    factor the reference's visit order keeps."""
    for tm in modes:
        s, F = run_exact(session, T, transf_mode=tm)
        assert s.stats()[28] == 1  # the source pass ran
        F_ref = orc.factorize_exact_smpl(T, tm, 1)
        assert F.shape == F_ref.shape
        bad = np.nonzero(np.any(F != F_ref, axis=1))[0]
        assert bad.size == 0, (tm, int(bad[0]), F[bad[0]].tolist(), F_ref[bad[0]].tolist(), int(bad.size))


@pytest.mark.gpu
@pytest.mark.parametrize("name", golden_names())
def test_gpu_exact_smpl_reference_sources_golden(session, orc, name):
    check_reference_stream(orc, session, load_golden(name)["text"])


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(1, 17))
def test_gpu_exact_smpl_reference_sources_c1(session, orc, lz, seed):
    check_reference_stream(orc, session, lz.gen_random_repetitive(10000, 200000, seed))


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["genome", "rr", "runs"])
def test_gpu_exact_smpl_reference_sources_medium(session, orc, lz, kind):
    """4 MiB texts: many grid queries (intervals above the 4 096-rank scan threshold)."""
    n = 4 << 20
    if kind == "genome":
        T = lz.gen_genome(n, 1 << 20, 0.001, 3)
    elif kind == "rr":
        T = lz.gen_random_repetitive(n, n, 4, 0.5, 0.05)
    else:
        rng = np.random.Generator(np.random.PCG64(6))
        T = np.tile(rng.integers(0, 4, 777, dtype=np.uint8), n // 777 + 1)[:n]
        T[rng.integers(0, n, 200)] = 9
    check_reference_stream(orc, session, T, modes=[1, 2])


KNOBS = [{"LZ77SSS_SMPL_LSCAN": "0"}, {"LZ77SSS_SMPL_SCAN": "0"}, {"LZ77SSS_SMPL_SCAN": "1000000000"},
         {"LZ77SSS_SMPL_SMALL": "0"}, {"LZ77SSS_SMPL_CHUNK": "1"}, {"LZ77SSS_SMPL_CHUNK": "7"},
         {"LZ77SSS_SMPL_OWN_SOURCES": "1"}]


@pytest.mark.gpu
@pytest.mark.parametrize("knob", KNOBS, ids=lambda k: ",".join(f"{a[13:]}={b}" for a, b in k.items()))
def test_gpu_exact_smpl_knobs(session, orc, lz, monkeypatch, knob):
    """The phrase searches' paths one at a time (lane scans off, every intersect by the grid or by the
    Pi / Psi scan, the per-lane small scans off, one or seven phrases per chunk walk): the same
    stream, sources included (the source pass decides them); with the source pass off, the
    canonical lengths with valid sources."""
    for k, v in knob.items():
        monkeypatch.setenv(k, v)
    texts = [load_golden(nm)["text"] for nm in ("c1_seed1", "genome_small", "binary_30k", "periodic")]
    texts.append(lz.gen_random_repetitive(10000, 200000, 3))
    for T in texts:
        if "LZ77SSS_SMPL_OWN_SOURCES" in knob:
            for tm in SMPL_MODES:
                _, F = run_exact(session, T, transf_mode=tm)
                check_exact(lz, T, F, orc.factorize_exact(T))
        else:
            check_reference_stream(orc, session, T)


@pytest.mark.gpu
@pytest.mark.parametrize("sigma", [2, 256])
def test_gpu_exact_smpl_alphabets(session, orc, lz, sigma):
    """Sort-key packing at 1 bit (two symbols) and 8 bits (all 256 byte values) per character."""
    rng = np.random.Generator(np.random.PCG64(sigma))
    base = rng.integers(0, sigma, 3000, dtype=np.uint8)
    parts = [base]
    for _ in range(60):  # mutated copies: long phrases with sources to choose from
        cp = base[rng.integers(0, 2000):][:rng.integers(200, 1000)].copy()
        cp[rng.integers(0, cp.size, 3)] = rng.integers(0, sigma, 3, dtype=np.uint8)
        parts.append(cp)
    T = np.concatenate(parts)
    if sigma == 256:
        T[:256] = np.arange(256, dtype=np.uint8)
    check_reference_stream(orc, session, T)
