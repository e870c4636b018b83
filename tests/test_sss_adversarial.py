"""Sync-set parity on hash-adversarial text and through the exact overflow path.

Phi is a polynomial hash mod 2^32.  Thue-Morse windows collide
under any odd base mod 2^32 (the difference of a Thue-Morse block and its
complement is divisible by 2^(k(k+1)/2) for blocks of length 2^k), so ties in
the window minima make S denser than the 2n/tau of random text.  These tests pin
S against the oracle on such texts, report the density, and force the exact
per-stripe fallback (k_sss_fallback) with a lower overflow threshold.
"""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TAU = 512


def thue_morse(n: int) -> np.ndarray:
    i = np.arange(n, dtype=np.uint64)
    bits = np.zeros(n, np.uint8)
    for k in range(64):
        bits ^= ((i >> np.uint64(k)) & np.uint64(1)).astype(np.uint8)
    return (bits + ord("a")).astype(np.uint8)


def fibonacci_word(n: int) -> np.ndarray:
    # f[i] = 'b' iff floor((i+2)/phi) - floor((i+1)/phi) == 0, the standard Sturmian form
    phi = (1 + 5 ** 0.5) / 2
    i = np.arange(n, dtype=np.float64)
    x = np.floor((i + 2) / phi) - np.floor((i + 1) / phi)
    return np.where(x == 1, ord("a"), ord("b")).astype(np.uint8)


def _sss(session, T):
    s = session(max(T.size, 1))
    s.load(T)
    return s, s.sss()


@pytest.mark.slow
@pytest.mark.parametrize("kind", ["thue_morse", "fibonacci"])
def test_adversarial_sync_set_64mib(session, orc, kind):
    n = 64 << 20
    T = thue_morse(n) if kind == "thue_morse" else fibonacci_word(n)
    s, (S, has_runs) = _sss(session, T)
    S_ref, hr_ref = orc.sss(T)
    assert np.array_equal(S, S_ref) and has_runs == hr_ref
    dens = S.size / (2 * n / TAU)
    print(f"{kind}: |S| = {S.size}, |S|/(2n/tau) = {dens:.3f}")
    assert dens < 8.0  # the stripes' capacity (SCAP = 1024 of 32768 decisions) is 8x the random-text density


@pytest.mark.parametrize("kind", ["thue_morse", "fibonacci"])
def test_adversarial_factorization(session, orc, kind):
    n = 3 << 20
    T = thue_morse(n) if kind == "thue_morse" else fibonacci_word(n)
    s = session(n)
    s.load(T)
    z = s.factorize()
    assert np.array_equal(s.factors(z), orc.factorize(T)[0])


def _texts(lz):
    yield "c1", lz.gen_random_repetitive(10000, 200000, 4)
    yield "genome", lz.gen_genome(4 << 20, 1 << 20, 0.001, 5)
    yield "rr", lz.gen_random_repetitive(8 << 20, 8 << 20, 6, 0.5, 0.05)
    yield "thue_morse", thue_morse(1 << 20)
    rng = np.random.Generator(np.random.PCG64(9))
    yield "random", rng.integers(0, 256, (1 << 20) + 12345, dtype=np.uint8)


@pytest.mark.parametrize("scap", [0, 3, 64])
def test_forced_fallback_matches_oracle(session, orc, lz, scap, monkeypatch):
    """LZ77SSS_TEST_SCAP lowers the per-stripe overflow threshold: stripes with more outputs are
    recomputed by the workgroup-parallel exact path; S and the factor stream must not change."""
    monkeypatch.setenv("LZ77SSS_TEST_SCAP", str(scap))
    for name, T in _texts(lz):
        s = session(T.size)
        s.load(T)
        z = s.factorize()
        st = s.stats()
        S, has_runs = s.sss()
        S_ref, hr_ref = orc.sss(T)
        assert np.array_equal(S, S_ref) and has_runs == hr_ref, name
        if S.size > scap * 64:
            assert st[14] > 0, name  # some stripe went through the fallback
        if name in ("c1", "genome"):
            assert np.array_equal(s.factors(z), orc.factorize(T)[0]), name
