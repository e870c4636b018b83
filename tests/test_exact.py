"""Exact mode (factorize_exact, lz77_sss.hpp:188-200): canonical greedy LZ77.

The reference's own tests check its exact modes only by decode(factorize(T)) == T
(tests/test_lz77_sss.cpp:95-133).  Here the lengths are pinned harder: the
oracle's exact restatement is checked against a brute-force longest-previous-
factor parse, and the device stream (lengths and the PSV/NSV source rule) is
compared bit for bit with the oracle.  Sources are not the reference's (its
sample/range-structure visit order is not restated): "parity unpinned" for
sources, pinned by definition for lengths.
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


def run_exact(session, T, **kw):
    s = session(max(T.size, 1))
    s.load(T)
    z = s.factorize_exact(**kw)
    return s, s.factors(z)


@pytest.mark.gpu
@pytest.mark.parametrize("name", golden_names())
def test_gpu_exact_golden(session, name):
    g = load_golden(name)
    _, F = run_exact(session, g["text"])
    assert np.array_equal(F, g["factors_exact"])


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(1, 17))
def test_gpu_exact_c1_seeds(session, orc, lz, seed):
    T = lz.gen_random_repetitive(10000, 200000, seed)
    _, F = run_exact(session, T)
    assert np.array_equal(F, orc.factorize_exact(T))
    assert np.array_equal(lz.decode(F, T.size), T)


@pytest.mark.gpu
@pytest.mark.parametrize("transf_mode", [0, 2])
def test_gpu_exact_transform_modes_agree(session, orc, lz, transf_mode):
    T = lz.gen_random_repetitive(50000, 120000, 77)
    _, F = run_exact(session, T, transf_mode=transf_mode)
    assert np.array_equal(F, orc.factorize_exact(T))


@pytest.mark.gpu
def test_gpu_exact_with_samples_rejected(session, lz):
    """with_samples needs the reference's sample index (not built on the device): EINVAL, not a silent
    substitute."""
    T = lz.gen_random_repetitive(20000, 20000, 3)
    s = session(T.size)
    s.load(T)
    with pytest.raises(lz.Lz77SssError, match="with_samples"):
        s.factorize_exact(transf_mode=lz.WITH_SAMPLES)


@pytest.mark.gpu
@pytest.mark.parametrize("period", [1, 3, 170, 171, 600])
def test_gpu_exact_runs(session, orc, period):
    rng = np.random.Generator(np.random.PCG64(period))
    unit = rng.integers(0, 256, period, dtype=np.uint8)
    T = np.concatenate([rng.integers(0, 256, 3000, dtype=np.uint8), np.tile(unit, 40000 // period + 1)[:40000],
                        rng.integers(0, 256, 2000, dtype=np.uint8)])
    _, F = run_exact(session, T)
    assert np.array_equal(F, orc.factorize_exact(T))


@pytest.mark.gpu
@pytest.mark.parametrize("kind,mib", [("genome", 16), ("rr", 16)])
def test_gpu_exact_medium(session, orc, lz, kind, mib):
    n = mib << 20
    T = lz.gen_genome(n, 2 << 20, 0.001, 11) if kind == "genome" else lz.gen_random_repetitive(n, n, 5, 0.5, 0.05)
    _, F = run_exact(session, T)
    F_ref = orc.factorize_exact(T)
    assert F.shape == F_ref.shape and np.array_equal(F, F_ref)


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
    rc = lz.load_library().lz77sss_factorize_exact_u32(T.ctypes.data_as(ctypes.c_void_p), T.size, ctypes.byref(p),
                                                       lz.WITHOUT_SAMPLES, cb, None)
    assert rc == 0
    assert np.array_equal(np.concatenate(got), orc.factorize_exact(T))


@pytest.mark.gpu
def test_gpu_exact_invalid_parameters(session, lz):
    T = lz.gen_random_repetitive(20000, 20000, 1)
    s = session(T.size)
    s.load(T)
    with pytest.raises(lz.Lz77SssError):
        s.factorize_exact(transf_mode=7)
    with pytest.raises(lz.Lz77SssError):
        s.factorize_exact(fact_mode=lz.SKIP_PHRASES)
