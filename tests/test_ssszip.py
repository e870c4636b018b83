"""ssszip's gapped container: the device build (csrc/ssszip.hip)
against the CPU restatement (oracle/ssszip.py, cli/ssszip.cpp:119-177), and the
container's decode round trip.  CPU: the restatement on the oracle's skip_phrases
streams.  GPU: byte-exact container from the device stream, decode back to the text."""
from __future__ import annotations

import numpy as np
import pytest

import ssszip as SZ

SKIP = 2


def _rr(lz, n, seed):
    return lz.gen_random_repetitive(n, n, seed, 0.5, 0.05)


def test_vbyte_roundtrip():
    for x in [0, 1, 127, 128, 255, 16383, 16384, 2**31 - 1, 2**32 - 1, 2**40 + 5]:
        b = bytearray()
        SZ.encode_vbyte(x, b)
        assert len(b) == max(1, (x.bit_length() + 6) // 7)
        assert SZ.decode_vbyte(b, 0) == (x, len(b))
    b = bytearray()
    SZ.encode_vbyte(300, b)
    assert bytes(b) == bytes([0xAC, 0x02])  # 7-bit groups, least significant first


@pytest.mark.parametrize("seed", [1, 2, 3, 5, 8])
def test_oracle_container_roundtrip(orc, lz, seed):
    T = lz.gen_random_repetitive(10000, 200000, seed, -1.0, -1.0)
    stream = orc.factorize_skip(T)
    buf = SZ.encode_gapped(stream, T)
    assert buf[0] == 0 and int.from_bytes(buf[1:9], "little") == T.size
    assert SZ.decode_gapped(buf) == T.tobytes()


def test_oracle_container_edges(orc):
    rng = np.random.default_rng(3)
    for T in [np.zeros(0, np.uint8), np.frombuffer(b"a", np.uint8), rng.integers(0, 256, 5000).astype(np.uint8),
              np.tile(rng.integers(0, 256, 70).astype(np.uint8), 300)]:
        buf = SZ.encode_gapped(orc.factorize_skip(T), T)
        assert SZ.decode_gapped(buf) == T.tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("kind,n", [("rr", 1 << 16), ("rr", 200000), ("rr", 64 << 20), ("genome", 8 << 20),
                                    ("random", 100000), ("runs", 300000)])
def test_device_container_matches_restatement(session, orc, lz, kind, n):
    rng = np.random.default_rng(n)
    if kind == "rr":
        T = _rr(lz, n, 11)
    elif kind == "genome":
        T = lz.gen_genome(n, 1 << 20, 0.001, 5)
    elif kind == "random":
        T = rng.integers(0, 256, n).astype(np.uint8)
    else:
        T = np.tile(rng.integers(0, 256, 37).astype(np.uint8), n // 37 + 1)[:n]
    s = session(T.size)
    s.load(T)
    z = s.factorize(fact_mode=SKIP)
    stream = s.factors(z)
    if n <= 200000:
        assert np.array_equal(stream, orc.factorize_skip(T))
    buf = s.ssszip_gapped()
    want = SZ.encode_gapped(stream, T)
    assert buf.tobytes() == want
    if n <= (8 << 20):
        assert SZ.decode_gapped(buf) == T.tobytes()


@pytest.mark.gpu
def test_device_container_needs_skip_phrases(session, lz):
    T = _rr(lz, 100000, 4)
    s = session(T.size)
    s.load(T)
    s.factorize()  # greedy
    with pytest.raises(lz.Lz77SssError):
        s.ssszip_gapped()
