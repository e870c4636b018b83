"""GPU parity: the HIP path through the C-ABI against the oracle and the golden fixtures.

Bit-exact on every intermediate the reference exposes (S, SA_S, LCP, LPF_opt
phrases) and on the factor stream.  Full-size (1 GiB) inputs are checked by
size-independent properties (decode round trip, factor validity) and, for the
repetitive text, against the oracle stream itself.
"""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

from conftest import golden_names, load_golden

pytestmark = pytest.mark.gpu


def run(session, T, **kw):
    s = session(max(T.size, 1))
    s.load(T)
    z = s.factorize(**kw)
    return s, s.factors(z)


@pytest.mark.parametrize("name", golden_names())
def test_golden_factor_stream(session, name):
    g = load_golden(name)
    s, F = run(session, g["text"])
    assert np.array_equal(F, g["factors"])
    st = s.stats()
    assert st[:12] == [int(x) for x in g["stats"][:12]]


@pytest.mark.parametrize("name", golden_names())
def test_golden_intermediates(session, name):
    g = load_golden(name)
    s, _ = run(session, g["text"])
    S, has_runs = s.sss()
    assert np.array_equal(S, g["sss"]) and has_runs == bool(g["has_runs"][0])
    if S.size:
        SA, LCP = s.sa_s(S.size)
        assert np.array_equal(SA, g["sa_s"]) and np.array_equal(LCP, g["lcp"])
    assert np.array_equal(s.lpf(), g["lpf"])


@pytest.mark.parametrize("name", golden_names())
def test_verify_factors_in_hbm(session, name):
    """lz77sss_session_verify (decode.hip k_verify_blocks): 0 bad positions for the golden stream;
    after the text in HBM is changed at one position (the factors kept) the check reports it."""
    g = load_golden(name)
    T = g["text"]
    s, F = run(session, T)
    assert s.verify() == 0
    if T.size:
        for p in {0, T.size // 2, T.size - 1}:
            T2 = T.copy()
            T2[p] ^= 0x5A
            s.load(T2)
            assert s.verify() >= 1, p
        s.load(T)
        assert s.verify() == 0


@pytest.mark.parametrize("seed", range(1, 17))
def test_c1_seeds_vs_oracle(session, orc, lz, seed):
    """Config C1: random_repetitive_string(10^4, 2·10^5), p = 1 stream."""
    T = lz.gen_random_repetitive(10000, 200000, seed)
    _, F = run(session, T)
    F_ref, _ = orc.factorize(T)
    assert np.array_equal(F, F_ref)
    assert np.array_equal(lz.decode(F, T.size), T)


@pytest.mark.parametrize("rk_seed", [0, 1, 7, 123456789])
def test_gap_index_seeds(session, orc, lz, rk_seed):
    T = lz.gen_random_repetitive(50000, 150000, 99)
    _, F = run(session, T, rk_seed=rk_seed)
    F_ref, _ = orc.factorize(T, rk_seed=rk_seed)
    assert np.array_equal(F, F_ref)


@pytest.mark.parametrize("n", [0, 1, 2, 3, 511, 512, 513, 1023, 1024, 1025, 1535, 1536, 1537, 2048, 4097, 65536,
                               65537, 262144 + 3])
def test_edge_sizes(session, orc, n):
    rng = np.random.Generator(np.random.PCG64(n))
    T = rng.integers(0, 3, n, dtype=np.uint8)
    if n > 3000:
        T[1000:2500] = T[100:1600]  # a long repeat -> LPF phrases
    s, F = run(session, T)
    F_ref, _ = orc.factorize(T)
    assert np.array_equal(F, F_ref)


@pytest.mark.parametrize("period", [1, 2, 5, 170, 171, 300])
def test_runs(session, orc, period):
    rng = np.random.Generator(np.random.PCG64(period))
    unit = rng.integers(0, 256, period, dtype=np.uint8)
    T = np.concatenate([rng.integers(0, 256, 3000, dtype=np.uint8), np.tile(unit, 200000 // period),
                        rng.integers(0, 256, 5000, dtype=np.uint8), np.tile(unit, 3000 // period + 1)])
    s, F = run(session, T)
    F_ref, _ = orc.factorize(T)
    assert np.array_equal(F, F_ref)
    S, has_runs = s.sss()
    S_ref, hr_ref = orc.sss(T)
    assert np.array_equal(S, S_ref) and has_runs == hr_ref


@pytest.mark.parametrize("kind,mib", [("genome", 16), ("rr", 64)])
def test_medium_vs_oracle(session, orc, lz, kind, mib):
    n = mib << 20
    T = lz.gen_genome(n, 2 << 20, 0.001, 11) if kind == "genome" else lz.gen_random_repetitive(n, n, 5, 0.5, 0.05)
    _, F = run(session, T)
    F_ref, _ = orc.factorize(T)
    assert F.shape == F_ref.shape and np.array_equal(F, F_ref)


def test_one_shot_callback_api(lz, orc):
    """lz77sss_factorize_approx_u32: factors arrive in order, batched, through the emit callback."""
    T = lz.gen_random_repetitive(150000, 150000, 8)
    got = []
    EMIT = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p)

    def emit(ptr, count, user):
        got.append(np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ctypes.c_uint32)), (count, 2)).copy())
        return 0

    cb = EMIT(emit)
    p = lz.params()
    rc = lz.load_library().lz77sss_factorize_approx_u32(T.ctypes.data_as(ctypes.c_void_p), T.size,
                                                        ctypes.byref(p), cb, None)
    assert rc == 0
    F = np.concatenate(got)
    assert np.array_equal(F, orc.factorize(T)[0])


def test_invalid_parameters_fail_loudly(session, lz):
    T = lz.gen_random_repetitive(20000, 20000, 1)
    s = session(T.size)
    s.load(T)
    with pytest.raises(lz.Lz77SssError):
        s.factorize(tau=256)
    with pytest.raises(lz.Lz77SssError):
        s.factorize(fact_mode=lz.GREEDY_NAIVE)
    with pytest.raises(lz.Lz77SssError):
        s.factorize(phr_mode=7)
    small = lz.Session(1 << 10)
    with pytest.raises(lz.Lz77SssError):
        small.load(T)
    small.close()


def _check_valid(T, F):
    """Vectorised factor validity: literals match, references point backwards, lengths sum to n."""
    ln = F[:, 1].astype(np.int64)
    pos = np.concatenate([[0], np.cumsum(np.maximum(ln, 1))[:-1]])
    assert pos[-1] + max(ln[-1], 1) == T.size
    lit = ln == 0
    assert np.array_equal(F[lit, 0].astype(np.uint8), T[pos[lit]])
    assert np.all(F[~lit, 0].astype(np.int64) < pos[~lit])


@pytest.mark.slow
@pytest.mark.parametrize("kind", ["rr", "genome"])
def test_one_gib_properties(session, orc, lz, kind):
    n = 1 << 30
    T = lz.gen_random_repetitive(n, n, 42, 0.5, 0.05) if kind == "rr" else lz.gen_genome(n, 64 << 20, 0.001, 7)
    s, F = run(session, T)
    _check_valid(T, F)
    assert np.array_equal(lz.decode(F, n), T)
    _, mism = s.decode(out=False)  # device decode compared in HBM with the loaded text
    assert mism == 0
    st = s.stats()
    assert st[0] <= 2 * n // 512 + 1024
    if kind == "rr":  # the oracle finishes this one in seconds
        F_ref, _ = orc.factorize(T)
        assert np.array_equal(F, F_ref)


def test_cpp_mirror_roundtrip(tmp_path):
    """The reference's own test shape through the C++ template mirror on the GPU."""
    import subprocess

    from test_capi import build_cpp_client

    exe = build_cpp_client(tmp_path)
    r = subprocess.run([str(exe), "8"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count(" ok") == 16  # 8 seeds x pos_t in {uint32_t, uint64_t}


@pytest.mark.parametrize("name", golden_names())
def test_golden_lpf_lnf_stream(session, name):
    """Config 3: factorize_approximate<greedy, lpf_lnf_opt> (reversed-text LNF phrases + selection)."""
    g = load_golden(name)
    s, F = run(session, g["text"], phr_mode=3)
    assert np.array_equal(F, g["factors_lnf"])
    assert s.stats()[:12] == [int(x) for x in g["stats_lnf"][:12]]


@pytest.mark.parametrize("seed", range(1, 9))
@pytest.mark.parametrize("mode", [3, 1])
def test_c1_lpf_lnf_vs_oracle(session, orc, lz, seed, mode):
    T = lz.gen_random_repetitive(10000, 200000, seed)
    _, F = run(session, T, phr_mode=mode)
    F_ref, _ = orc.factorize(T, phr_mode=mode)
    assert np.array_equal(F, F_ref)
    assert np.array_equal(lz.decode(F, T.size), T)


@pytest.mark.parametrize("kind,mib", [("genome", 8), ("rr", 32)])
def test_medium_lpf_lnf_vs_oracle(session, orc, lz, kind, mib):
    n = mib << 20
    T = lz.gen_genome(n, 1 << 20, 0.001, 3) if kind == "genome" else lz.gen_random_repetitive(n, n, 9, 0.5, 0.05)
    _, F = run(session, T, phr_mode=3)
    F_ref, _ = orc.factorize(T, phr_mode=3)
    assert F.shape == F_ref.shape and np.array_equal(F, F_ref)


# ---- device decode (csrc/decode.hip) vs the reference's sequential decode (algorithms/common.cpp:31-54)

@pytest.mark.parametrize("name", golden_names())
def test_device_decode_golden(lz, name):
    g = load_golden(name)
    T, F = g["text"], g["factors"]
    assert np.array_equal(lz.decode_device(F, T.size), T)


def _deep_chain_stream(n):
    """'a' then one self-overlapping copy (src 0): every position's chain has depth p."""
    return np.array([[ord("a"), 0], [0, n - 1]], np.uint32)


@pytest.mark.parametrize("n", [1, 2, 3, 1000, 1 << 20, (1 << 24) + 7])
def test_device_decode_deep_chains(lz, n):
    F = _deep_chain_stream(n) if n > 1 else np.array([[ord("a"), 0]], np.uint32)
    assert np.array_equal(lz.decode_device(F, n), np.full(n, ord("a"), np.uint8))
    # period-3 run: literals x y z then a copy of distance 3
    if n > 3:
        F3 = np.array([[120, 0], [121, 0], [122, 0], [0, n - 3]], np.uint32)
        assert np.array_equal(lz.decode_device(F3, n), np.resize(np.array([120, 121, 122], np.uint8), n))


@pytest.mark.parametrize("seed", range(1, 9))
def test_device_decode_session_roundtrip(session, lz, seed):
    T = lz.gen_random_repetitive(50000, 400000, seed)
    s, F = run(session, T)
    D, mism = s.decode()
    assert mism == 0 and np.array_equal(D, T)
    assert np.array_equal(lz.decode_device(F, T.size), lz.decode(F, T.size))


def test_device_decode_random_streams(lz):
    """Arbitrary valid streams (not LZ77-greedy): random sources and lengths."""
    rng = np.random.default_rng(3)
    for n in [10, 1000, 100000]:
        F, pos = [], 0
        while pos < n:
            if pos == 0 or rng.random() < 0.3:
                F.append((int(rng.integers(0, 256)), 0)); pos += 1
            else:
                ln = int(min(n - pos, rng.integers(1, 2 * pos + 2)))
                F.append((int(rng.integers(0, pos)), ln)); pos += ln
        F = np.array(F, np.uint32)
        assert np.array_equal(lz.decode_device(F, n), lz.decode(F, n))


def test_device_decode_rejects_invalid(lz):
    with pytest.raises(lz.Lz77SssError):  # forward reference
        lz.decode_device(np.array([[97, 0], [1, 2]], np.uint32), 3)
    with pytest.raises(lz.Lz77SssError):  # lengths do not sum to n
        lz.decode_device(np.array([[97, 0], [0, 2]], np.uint32), 5)
    with pytest.raises(lz.Lz77SssError):
        lz.decode_device(np.array([[97, 0]], np.uint32), 0)
    with pytest.raises(lz.Lz77SssError):  # lengths sum to n + 2^32: a 32-bit running sum would wrap to n
        lz.decode_device(np.array([[97, 0], [0, 4], [0, 0xFFFFFFFF], [0, 1]], np.uint32), 5)
    assert lz.decode_device(np.zeros((0, 2), np.uint32), 0).size == 0


@pytest.mark.slow
def test_device_decode_past_2g(lz):
    """n just above 2^31: every device scan of the decode runs on 64-bit item counts."""
    n = (1 << 31) + 7
    F = np.array([[ord("x"), 0], [ord("y"), 0], [0, n - 2]], np.uint32)
    out = lz.decode_device(F, n)
    assert out.size == n and out[0] == ord("x") and out[1] == ord("y")
    assert out[-1] == (ord("x") if (n - 1) % 2 == 0 else ord("y"))
    assert np.array_equal(out[:1 << 20], np.resize(np.array([ord("x"), ord("y")], np.uint8), 1 << 20))


@pytest.mark.parametrize("name", golden_names())
def test_golden_lpf_naive_vs_oracle(session, orc, name):
    """phr_mode = lpf_naive (lpf_lnf/lpf_naive.cpp:33-110) with the greedy emitter."""
    g = load_golden(name)
    _, F = run(session, g["text"], phr_mode=0)
    F_ref, _ = orc.factorize(g["text"], phr_mode=0)
    assert np.array_equal(F, F_ref)


@pytest.mark.parametrize("seed", range(1, 9))
def test_c1_lpf_naive_vs_oracle(session, orc, lz, seed):
    T = lz.gen_random_repetitive(10000, 200000, seed)
    _, F = run(session, T, phr_mode=lz.LPF_NAIVE)
    F_ref, _ = orc.factorize(T, phr_mode=0)
    assert np.array_equal(F, F_ref)
    assert np.array_equal(lz.decode(F, T.size), T)


@pytest.mark.parametrize("kind,mib", [("rr", 128), ("rr", 1), ("genome", 8)])
def test_dense_slot_ids_match_slot_sort(session, lz, kind, mib, monkeypatch):
    """Greedy base set sorted on dense slot ids (few distinct slots) == sorted on the slots."""
    n = mib << 20
    T = lz.gen_genome(n, 1 << 20, 0.001, 13) if kind == "genome" else lz.gen_random_repetitive(n, n, 7, 0.5, 0.05)
    _, F1 = run(session, T)
    monkeypatch.setenv("LZ77SSS_NO_DENSE", "1")
    _, F0 = run(session, T)
    assert F1.shape == F0.shape and np.array_equal(F1, F0)


@pytest.mark.parametrize("mib,seed", [(1, 7), (32, 5), (64, 9)])
def test_lsd_base_sort_vs_oracle(session, orc, lz, mib, seed, monkeypatch):
    """Bucket-search lookups on dense slot ids: the base set sorted by the LSD sort (reduce-then-scan,
    dense-id map fused, csrc/greedy.hip) equals rocprim's radix sort (LZ77SSS_NO_LSD) and the oracle."""
    n = mib << 20
    T = lz.gen_random_repetitive(n, n, seed, 0.5, 0.05)
    F_ref, _ = orc.factorize(T)
    monkeypatch.setenv("LZ77SSS_NO_PRED", "1")
    _, F1 = run(session, T)
    assert F1.shape == F_ref.shape and np.array_equal(F1, F_ref)
    for knob in ("LZ77SSS_LS_RANK", "LZ77SSS_LS_BLOCKSORT"):  # every pass by ballot ranking / by block sort
        monkeypatch.setenv(knob, "1")
        _, F2 = run(session, T)
        assert np.array_equal(F2, F_ref), knob
        monkeypatch.delenv(knob)
    monkeypatch.setenv("LZ77SSS_NO_LSD", "1")
    _, F0 = run(session, T)
    assert np.array_equal(F0, F_ref)


@pytest.mark.parametrize("log2", [6, 10, 14, 18])
def test_lsd_base_sort_table_sizes(session, lz, log2, monkeypatch):
    """Gap-index tables of 2^6 .. 2^18 slots: one to three LSD passes of 7 bits; the stream equals the
    rocprim-sorted one and decodes to the text."""
    n = 16 << 20
    T = lz.gen_random_repetitive(n, n, 3, 0.5, 0.05)
    monkeypatch.setenv("LZ77SSS_NO_PRED", "1")
    _, F1 = run(session, T, index_log2_size=log2)
    monkeypatch.setenv("LZ77SSS_NO_LSD", "1")
    _, F0 = run(session, T, index_log2_size=log2)
    assert F1.shape == F0.shape and np.array_equal(F1, F0)
    assert np.array_equal(lz.decode(F1, n), T)


@pytest.mark.parametrize("kind,mib", [("genome", 16), ("rr", 32)])
def test_sorted_predecessor_paths_vs_oracle(session, orc, lz, kind, mib, monkeypatch):
    """Base sets above LZ77SSS_PRED_SORTED_MIN move their predecessors back by bucket scatter
    (default) or by a radix sort (LZ77SSS_PRED_RADIX): both equal the oracle stream."""
    n = mib << 20
    T = lz.gen_genome(n, 2 << 20, 0.001, 11) if kind == "genome" else lz.gen_random_repetitive(n, n, 5, 0.5, 0.05)
    F_ref, _ = orc.factorize(T)
    monkeypatch.setenv("LZ77SSS_PRED_SORTED_MIN", "1")
    _, F1 = run(session, T)
    assert F1.shape == F_ref.shape and np.array_equal(F1, F_ref)
    monkeypatch.setenv("LZ77SSS_PRED_RADIX", "1")
    _, F2 = run(session, T)
    assert np.array_equal(F2, F_ref)


@pytest.mark.parametrize("kind,mib", [("genome", 16), ("rr", 32)])
def test_pred_and_bucket_search_paths_vs_oracle(session, orc, lz, kind, mib, monkeypatch):
    """Base lookups through the same-slot predecessors (LZ77SSS_PRED) and through bucket
    searches (LZ77SSS_NO_PRED; chosen by default for texts with few long gaps) both equal
    the oracle stream."""
    n = mib << 20
    T = lz.gen_genome(n, 2 << 20, 0.001, 17) if kind == "genome" else lz.gen_random_repetitive(n, n, 9, 0.5, 0.05)
    F_ref, _ = orc.factorize(T)
    monkeypatch.setenv("LZ77SSS_PRED", "1")
    _, F1 = run(session, T)
    assert F1.shape == F_ref.shape and np.array_equal(F1, F_ref)
    monkeypatch.setenv("LZ77SSS_NO_IPOSR", "1")  # removed flags in their own array, not in the positions
    _, F3 = run(session, T)
    assert np.array_equal(F3, F_ref)
    monkeypatch.delenv("LZ77SSS_NO_IPOSR")
    monkeypatch.delenv("LZ77SSS_PRED")
    monkeypatch.setenv("LZ77SSS_NO_PRED", "1")
    _, F2 = run(session, T)
    assert np.array_equal(F2, F_ref)


@pytest.mark.parametrize("kind,mib", [("rr", 32), ("genome", 16)])
def test_fast_convergence_check_vs_full_check(session, orc, lz, kind, mib, monkeypatch):
    """The fast I' == I decision (insert counts outside I + the subset check, csrc/greedy.hip) and the
    full xor/count path (LZ77SSS_NO_FAST_CHECK) give the same stream, equal to the oracle's."""
    n = mib << 20
    T = lz.gen_genome(n, 2 << 20, 0.001, 19) if kind == "genome" else lz.gen_random_repetitive(n, n, 13, 0.5, 0.05)
    F_ref, _ = orc.factorize(T)
    _, F1 = run(session, T)
    assert F1.shape == F_ref.shape and np.array_equal(F1, F_ref)
    monkeypatch.setenv("LZ77SSS_NO_FAST_CHECK", "1")
    _, F0 = run(session, T)
    assert np.array_equal(F0, F_ref)


@pytest.mark.parametrize("cap", ["0", "1", "3"])
def test_long_range_list_overflow(session, orc, lz, cap, monkeypatch):
    """k_chain_inserts hands ranges longer than LZ77SSS_TEST_LONG_WORDS words to the whole grid through
    a list of LZ77SSS_TEST_LNG_CAP entries; a wave whose range did not fit inserts it itself (decided
    from its own atomic's result).  With tiny caps most ranges overflow: the stream stays the oracle's,
    with the fast check and with the full one."""
    n = 8 << 20
    T = lz.gen_random_repetitive(n, n, 21, 0.5, 0.05)
    F_ref, _ = orc.factorize(T)
    monkeypatch.setenv("LZ77SSS_TEST_LONG_WORDS", "4")
    monkeypatch.setenv("LZ77SSS_TEST_LNG_CAP", cap)
    _, F1 = run(session, T)
    assert F1.shape == F_ref.shape and np.array_equal(F1, F_ref)
    monkeypatch.setenv("LZ77SSS_NO_FAST_CHECK", "1")
    _, F0 = run(session, T)
    assert np.array_equal(F0, F_ref)


CHUNKS_PROBE = ["16", "64", "128", "256", "512", "1024", "100000"]


@pytest.mark.parametrize("chunk", CHUNKS_PROBE)
@pytest.mark.parametrize("name", golden_names())
def test_gap_chunk_lengths_golden(session, name, chunk, monkeypatch):
    """Every chunk length must give the fixture's stream.  (Round-2 defect, fixed in round 3,
    DESIGN.md 4.5: a chunk walk stopped at its boundary on a factor start inside the tail region,
    so the tail walk started past positions whose conditional inserts it never modelled; chunks
    <= 128 changed factor 618's source on c1_seed2.)"""
    g = load_golden(name)
    monkeypatch.setenv("LZ77SSS_GAP_CHUNK", chunk)
    _, F = run(session, g["text"])
    assert np.array_equal(F, g["factors"])


@pytest.mark.parametrize("chunk", CHUNKS_PROBE)
@pytest.mark.parametrize("kind,mib", [("genome", 8), ("rr", 16)])
def test_gap_chunk_lengths_vs_oracle(session, orc, lz, kind, mib, chunk, monkeypatch):
    """Long gaps are cut into chunks of LZ77SSS_GAP_CHUNK positions whose walks converge onto
    the chain at a shared factor start: every chunk length gives the oracle stream."""
    n = mib << 20
    T = lz.gen_genome(n, 1 << 20, 0.001, 19) if kind == "genome" else lz.gen_random_repetitive(n, n, 21, 0.5, 0.05)
    F_ref, _ = orc.factorize(T)
    monkeypatch.setenv("LZ77SSS_GAP_CHUNK", chunk)
    _, F = run(session, T)
    assert F.shape == F_ref.shape and np.array_equal(F, F_ref)


# ---- bounded greedy completion (k_seq_walk): the exact sequential walk from the confirmed chain prefix

@pytest.mark.parametrize("max_outer", [0, 1, 2])
@pytest.mark.parametrize("seed", [1, 2, 3, 5, 8, 13])
def test_greedy_bounded_completion_c1(session, orc, lz, seed, max_outer, monkeypatch):
    """LZ77SSS_GREEDY_MAX_OUTER caps the speculation rounds; past the cap the chain prefix that is exact
    (up to the first position where the speculated and the actual insert sets differ) is kept and the
    rest is walked sequentially (0: the whole text).  Either way the stream is the p = 1 oracle's."""
    T = lz.gen_random_repetitive(10000, 200000, seed)
    monkeypatch.setenv("LZ77SSS_GREEDY_MAX_OUTER", str(max_outer))
    s, F = run(session, T)
    assert np.array_equal(F, orc.factorize(T)[0])
    st = s.stats()
    if max_outer == 0:
        assert st[19] == 1 and st[20] == 0
    else:
        assert st[12] <= max_outer


@pytest.mark.parametrize("n", [1, 2, 511, 1024, 1537, 4097, 65537])
def test_greedy_sequential_edges(session, orc, n, monkeypatch):
    """The sequential walk's tail semantics (stale / zeroed fingerprints, conditional inserts) at edge sizes."""
    rng = np.random.Generator(np.random.PCG64(n))
    T = rng.integers(0, 3, n, dtype=np.uint8)
    if n > 3000:
        T[1000:2500] = T[100:1600]
    monkeypatch.setenv("LZ77SSS_GREEDY_MAX_OUTER", "0")
    _, F = run(session, T)
    assert np.array_equal(F, orc.factorize(T)[0])


@pytest.mark.parametrize("max_outer", [1, 2, 3])
def test_greedy_bounded_completion_genome(session, orc, lz, max_outer, monkeypatch):
    """A genome-like text needs several speculation rounds; cutting them short must not change the stream."""
    n = 4 << 20
    T = lz.gen_genome(n, 1 << 20, 0.001, 21)
    F_ref, _ = orc.factorize(T)
    s0, F0 = run(session, T)
    rounds = s0.stats()[12]
    assert np.array_equal(F0, F_ref)
    monkeypatch.setenv("LZ77SSS_GREEDY_MAX_OUTER", str(max_outer))
    s, F = run(session, T)
    assert F.shape == F_ref.shape and np.array_equal(F, F_ref)
    st = s.stats()
    assert st[19] == (1 if rounds > max_outer else 0)


# ---- greedy windows: the chain walked window by window with the exact state and the
# last-insert-per-slot table handed over; any window size gives the same stream

@pytest.mark.parametrize("window", [4096, 20000, 65536])
@pytest.mark.parametrize("seed", [1, 4, 9])
def test_greedy_windows_c1(session, orc, lz, seed, window, monkeypatch):
    T = lz.gen_random_repetitive(10000, 200000, seed)
    monkeypatch.setenv("LZ77SSS_GREEDY_WINDOW", str(window))
    s, F = run(session, T)
    assert np.array_equal(F, orc.factorize(T)[0])
    assert s.stats()[21] >= (1 if T.size < 2 * window else 2)


@pytest.mark.parametrize("window,max_outer", [(1 << 20, 256), (3 << 20, 256), (1 << 20, 1), (1 << 20, 0)])
def test_greedy_windows_genome(session, orc, lz, window, max_outer, monkeypatch):
    """Windows on a gap-heavy text, also with the sequential completion inside windows."""
    n = 8 << 20
    T = lz.gen_genome(n, 1 << 20, 0.001, 17)
    monkeypatch.setenv("LZ77SSS_GREEDY_WINDOW", str(window))
    monkeypatch.setenv("LZ77SSS_GREEDY_MAX_OUTER", str(max_outer))
    s, F = run(session, T)
    F_ref, _ = orc.factorize(T)
    assert F.shape == F_ref.shape and np.array_equal(F, F_ref)
    assert s.stats()[21] >= 2


@pytest.mark.parametrize("chunk", ["16", "64", "128"])
@pytest.mark.parametrize("seed", range(1, 17))
def test_gap_chunk_short_c1_seeds(session, orc, lz, seed, chunk, monkeypatch):
    """Short chunks put a chunk boundary right below the tail region on most C1 texts (the
    round-2 divergence); every one of them gives the p = 1 oracle stream."""
    T = lz.gen_random_repetitive(10000, 200000, seed)
    monkeypatch.setenv("LZ77SSS_GAP_CHUNK", chunk)
    _, F = run(session, T)
    assert np.array_equal(F, orc.factorize(T)[0])


def _run_into_tail_text(n_rand=20000, run_len=19960, n_end=40, seed=5):
    """A gap factor that starts far below the text end and ends inside the tail region (the last
    64 positions): a random prefix, a run of one byte (no sync positions, so no LPF phrase covers
    it), then a few random bytes."""
    rng = np.random.default_rng(seed)
    return np.concatenate([rng.integers(0, 256, n_rand, dtype=np.uint8), np.full(run_len, 97, np.uint8),
                           rng.integers(0, 256, n_end, dtype=np.uint8)])


@pytest.mark.parametrize("max_outer", [256, 0])
@pytest.mark.parametrize("window", [4096, 8192])
@pytest.mark.parametrize("run_len", [19960, 19995])
@pytest.mark.parametrize("n_end", [1, 2, 5, 20])
def test_greedy_window_chain_reaches_tail(session, orc, window, max_outer, run_len, n_end, monkeypatch):
    """A non-last window whose chain reaches the tail region is walked again as the last window;
    the stream equals the oracle's.  With 1-2 trailing bytes the run has no sync position near
    its end, so the gap factor from 20 001 runs through every window end into the last 64
    positions (checked on the oracle stream); with more, an LPF phrase truncates it first."""
    T = _run_into_tail_text(run_len=run_len, n_end=n_end)
    n = T.size
    F_ref = orc.factorize(T)[0]
    L = np.maximum(F_ref[:, 1].astype(np.int64), 1)
    ends = np.cumsum(L)
    crosses = bool(np.any((L > 4096) & (ends >= n - 64) & (ends < n)))
    assert crosses == (n_end <= 2)
    monkeypatch.setenv("LZ77SSS_GREEDY_WINDOW", str(window))
    monkeypatch.setenv("LZ77SSS_GREEDY_MAX_OUTER", str(max_outer))
    s, F = run(session, T)
    assert np.array_equal(F, F_ref)
    # stats[23]: windows walked again as the last one (the sequential completion also re-walks
    # a window whose hand-over point an LPF factor carried past n - 64)
    assert s.stats()[23] >= 1 if crosses else (max_outer == 0 or s.stats()[23] == 0)


@pytest.mark.parametrize("kind,mib", [("rr", 64), ("rr", 3), ("periods", 8)])
def test_block_run_records_vs_scan_form(session, orc, lz, kind, mib, monkeypatch):
    """The per-block run records' segment ends / starts (k_blk_seg_tiles + k_blk_seg_info, ballot masks
    per 64-block group) equal the marker + min/max-scan formulation entry by entry (LZ77SSS_BLK_CHECK
    raises on any difference), and the stream equals the oracle's with and without the records and
    with every stopped stripe sent through the Q-anchor path (LZ77SSS_NO_RUNS_KERNEL)."""
    n = mib << 20
    if kind == "periods":
        rng = np.random.default_rng(5)
        parts, tot = [], 0
        while tot < n:  # runs of random periods 1..200 and lengths up to 2 MiB, random glue between
            p = int(rng.integers(1, 201))
            unit = rng.integers(97, 101, p, dtype=np.uint8)
            ln = int(rng.integers(1, 2 << 20))
            parts += [np.resize(unit, ln), rng.integers(0, 256, int(rng.integers(0, 3000)), dtype=np.uint8)]
            tot += ln
        T = np.concatenate(parts)[:n]
    else:
        T = lz.gen_random_repetitive(n, n, 31 + mib, 0.5, 0.05)
    F_ref, _ = orc.factorize(T)
    monkeypatch.setenv("LZ77SSS_BLK_CHECK", "1")
    _, F1 = run(session, T)
    assert F1.shape == F_ref.shape and np.array_equal(F1, F_ref)
    monkeypatch.delenv("LZ77SSS_BLK_CHECK")
    for knob in ("LZ77SSS_NO_BLKREC", "LZ77SSS_NO_RUNS_KERNEL"):
        monkeypatch.setenv(knob, "1")
        _, F2 = run(session, T)
        assert np.array_equal(F2, F_ref), knob
        monkeypatch.delenv(knob)


@pytest.mark.parametrize("kind,mib", [("rr", 32), ("genome", 16)])
def test_lean_release_of_phase_scratch(session, orc, lz, kind, mib, monkeypatch):
    """Large texts release the phases' own scratch before the emitter (engine::release_phase_scratch;
    LZ77SSS_LEAN=1 forces it at any size): the stream equals the oracle's, repeated calls on the same
    session (buffers grown again) stay equal, and the per-phase device memory shows the drop."""
    n = mib << 20
    T = lz.gen_genome(n, 2 << 20, 0.001, 23) if kind == "genome" else lz.gen_random_repetitive(n, n, 29, 0.5, 0.05)
    F_ref, _ = orc.factorize(T)
    s, F0 = run(session, T)
    held_full = s.phase_mem()["greedy"]["held"]
    monkeypatch.setenv("LZ77SSS_LEAN", "1")
    for _ in range(2):
        z = s.factorize()
        F = s.factors(z)
        assert F.shape == F_ref.shape and np.array_equal(F, F_ref)
    pm = s.phase_mem()
    assert set(pm) >= {"sss", "sa_s", "lcp_rmq", "lpf", "greedy"}
    assert pm["greedy"]["held"] < held_full  # (the release follows the "lpf" mark)
    assert all(m["peak"] >= m["held"] for m in pm.values())


@pytest.mark.parametrize("seed", range(1, 13))
def test_rr_4mib_seeds_vs_oracle(session, orc, lz, seed):
    """Run-heavy 4 MiB texts (runs of period 1 next to runs of other periods): the LPF phrases and
    the stream equal the oracle's.  Seed 4 once ended a period-1 run at the first break of the next
    run's period (the record written after k_sss_runs gave the stripe to the Q-anchor path), and the
    LCE's run skip stopped 343 bytes early."""
    n = 4 << 20
    T = lz.gen_random_repetitive(n, n, seed, 0.5, 0.05)
    F_ref, _ = orc.factorize(T)
    s, F = run(session, T)
    assert np.array_equal(s.lpf(), orc.lpf_opt(T))
    assert F.shape == F_ref.shape and np.array_equal(F, F_ref)
