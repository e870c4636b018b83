"""Huffman factor container (misc/huffman.hpp:318-436): the device
build (csrc/huffman.hip) against the sequential CPU restatement (oracle/oracle_huffman.cpp),
byte for byte, and the container decoded back to the factors.  The reference header
itself cannot be compiled here (std::byteswap needs GCC >= 12), so the format is pinned
by the restatement plus the decode round trip."""
from __future__ import annotations

import numpy as np
import pytest


@pytest.mark.parametrize("seed", [1, 2, 3, 4, 5, 6])
def test_oracle_container_roundtrip(orc, lz, seed):
    T = lz.gen_random_repetitive(10000, 200000, seed, -1.0, -1.0)
    F, _ = orc.factorize(T)
    buf = orc.huffman(F, T.size)
    assert int.from_bytes(buf[:5], "little") == T.size
    assert np.array_equal(orc.huffman_decode(buf, F.shape[0] + 8), F)


def test_oracle_container_multi_block(orc, lz):
    # > 2^14 factors: several blocks with their own tables, literals and long distances
    rng = np.random.default_rng(9)
    T = np.concatenate([rng.integers(0, 4, 250000).astype(np.uint8) + 65,
                        lz.gen_random_repetitive(100000, 100000, 3, 0.5, 0.05)])
    F, _ = orc.factorize(T)
    assert F.shape[0] > (1 << 14)
    buf = orc.huffman(F, T.size)
    assert np.array_equal(orc.huffman_decode(buf, F.shape[0] + 8), F)


def test_oracle_container_empty(orc):
    assert orc.huffman(np.zeros((0, 2), np.uint32), 0) == bytes(5)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,n", [("rr", 1 << 16), ("rr", 200000), ("genome", 4 << 20), ("rr", 64 << 20),
                                    ("random", 300000)])
def test_device_container_matches_restatement(session, orc, lz, kind, n):
    rng = np.random.default_rng(n)
    if kind == "rr":
        T = lz.gen_random_repetitive(n, n, 17, 0.5, 0.05)
    elif kind == "genome":
        T = lz.gen_genome(n, 1 << 20, 0.001, 5)
    else:
        T = rng.integers(0, 256, n).astype(np.uint8)
    s = session(T.size)
    s.load(T)
    z = s.factorize()
    F = s.factors(z)
    buf = s.huffman()
    assert buf.tobytes() == orc.huffman(F, T.size)
    assert np.array_equal(orc.huffman_decode(buf.tobytes(), z + 8), F)


@pytest.mark.gpu
def test_device_container_exact_mode(session, orc, lz):
    T = lz.gen_genome(1 << 20, 1 << 16, 0.01, 2)
    s = session(T.size)
    s.load(T)
    z = s.factorize_exact()
    F = s.factors(z)
    assert s.huffman().tobytes() == orc.huffman(F, T.size)


@pytest.mark.gpu
def test_device_container_rejects_skip_stream(session, lz):
    T = lz.gen_random_repetitive(100000, 100000, 4, 0.5, 0.05)
    s = session(T.size)
    s.load(T)
    s.factorize(fact_mode=2)
    with pytest.raises(lz.Lz77SssError):
        s.huffman()
