"""fact_mode = skip_phrases (factorize_skip_gaps, approximate/factorize/skip_gaps.cpp:31-61): the
gapped stream the reference's ssszip compressor consumes -- {first phrase start, 0}, then every LPF
phrase {src, len}, each followed by {gap length, 0} when the next phrase starts later."""
from __future__ import annotations

import numpy as np
import pytest

from conftest import golden_names, load_golden


def gapped_from_phrases(P, n):
    """The stream restated from the phrase list (p = 1, sentinel {n, n+1, 0}, lz77_sss.hpp:417-419)."""
    P = [tuple(int(x) for x in p) for p in P] + [(n, n + 1, 0)]
    out = [(P[0][0], 0)]
    k = 0
    while P[k][0] < n:
        beg, end, src = P[k]
        k += 1
        out.append((src, end - beg))
        if P[k][0] > end:
            out.append((P[k][0] - end, 0))
    return np.array(out, np.uint32).reshape(-1, 2)


def covered(F):
    pos = int(F[0, 0])
    for src, ln in F[1:]:
        pos += int(ln) if ln else int(src)
    return pos


@pytest.mark.parametrize("name", ["c1_seed1", "c1_seed3", "periodic", "genome_small", "binary_30k", "edge_n100",
                                  "edge_n5000", "zeros_10k"])
def test_oracle_skip_stream_matches_phrase_list(orc, name):
    g = load_golden(name)
    T = g["text"]
    F = orc.factorize_skip(T)
    assert np.array_equal(F, gapped_from_phrases(g["lpf"], T.size))
    assert covered(F) == T.size


@pytest.mark.gpu
@pytest.mark.parametrize("name", golden_names())
@pytest.mark.parametrize("phr", [2, 3])
def test_gpu_skip_golden(session, orc, lz, name, phr):
    g = load_golden(name)
    T = g["text"]
    s = session(max(T.size, 1))
    s.load(T)
    z = s.factorize(fact_mode=lz.SKIP_PHRASES, phr_mode=phr)
    assert np.array_equal(s.factors(z), orc.factorize_skip(T, phr_mode=phr))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(1, 9))
def test_gpu_skip_c1(session, orc, lz, seed):
    T = lz.gen_random_repetitive(10000, 200000, seed)
    s = session(T.size)
    s.load(T)
    z = s.factorize(fact_mode=lz.SKIP_PHRASES)
    F = s.factors(z)
    assert np.array_equal(F, orc.factorize_skip(T))
    assert covered(F) == T.size


@pytest.mark.gpu
def test_verify_refuses_skip_stream(session, lz):
    """lz77sss_session_verify checks a factorization against the text in HBM: after a skip_phrases call
    it refuses (LZ77SSS_EINVAL) instead of reporting bad positions; a later factorization is checked
    again; another loaded text is checked against the kept factors (it differs)."""
    T = lz.gen_random_repetitive(10000, 200000, 4)
    s = session(T.size)
    s.load(T)
    s.factorize()
    assert s.verify() == 0
    s.factorize(fact_mode=lz.SKIP_PHRASES)
    with pytest.raises(lz.Lz77SssError):
        s.verify()
    s.factorize()
    assert s.verify() == 0
    s.load(T[::-1].copy())
    assert s.verify() > 0
