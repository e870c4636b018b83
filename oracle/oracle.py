"""ctypes wrapper of the CPU oracle (oracle/_build/liboracle.so).

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module; the product path
(``lz77-sss_amd/``) never does.  The oracle is a CPU restatement of the
reference algorithm (see ``oracle.hpp``); parity is *unpinned* against the
reference binary because the reference cannot be built here.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "_build" / "liboracle.so"
_P = ctypes.c_void_p
_U64 = ctypes.c_uint64
_lib = None

LPF_OPT, LPF_LNF_OPT = 2, 3


def build(force: bool = False) -> Path:
    src_newer = any(p.stat().st_mtime > LIB.stat().st_mtime for p in HERE.glob("oracle*.?pp")) if LIB.exists() else True
    if force or src_newer:
        subprocess.run(["make", "-s", "-C", str(HERE), f"-j{min(8, os.cpu_count() or 1)}"], check=True)
    return LIB


def lib():
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        L = ctypes.CDLL(str(LIB))
        L.oracle_factorize_approx.restype = ctypes.c_int64
        L.oracle_factorize_approx.argtypes = [_P, _U64, ctypes.c_int, ctypes.c_uint32, _P, _U64, _P]
        L.oracle_factorize_timed.restype = ctypes.c_int64
        L.oracle_factorize_timed.argtypes = [_P, _U64, ctypes.c_int, ctypes.c_uint32, ctypes.POINTER(ctypes.c_double),
                                             ctypes.POINTER(_U64)]
        L.oracle_factorize_timed_p.restype = ctypes.c_int64
        L.oracle_factorize_timed_p.argtypes = [_P, _U64, ctypes.c_int, ctypes.c_uint32, ctypes.c_int,
                                               ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_U64),
                                               ctypes.POINTER(ctypes.c_int)]
        L.oracle_factorize_timed_p64.restype = ctypes.c_int64
        L.oracle_factorize_timed_p64.argtypes = L.oracle_factorize_timed_p.argtypes
        L.oracle_factorize_p.restype = ctypes.c_int64
        L.oracle_factorize_p.argtypes = [_P, _U64, ctypes.c_int, ctypes.c_uint32, _P, _U64,
                                         ctypes.POINTER(ctypes.c_int)]
        L.oracle_sss.restype = ctypes.c_int64
        L.oracle_sss.argtypes = [_P, _U64, _P, _U64, ctypes.POINTER(ctypes.c_int)]
        L.oracle_q_bruteforce.restype = None
        L.oracle_q_bruteforce.argtypes = [_P, _U64, _P]
        L.oracle_phi.restype = None
        L.oracle_phi.argtypes = [_P, _U64, _P]
        L.oracle_sa_s.restype = ctypes.c_int64
        L.oracle_sa_s.argtypes = [_P, _U64, _P, _P, _P, _U64]
        L.oracle_lce.restype = None
        L.oracle_lce.argtypes = [_P, _U64, _P, _P, _U64, _P]
        L.oracle_lpf_opt.restype = ctypes.c_int64
        L.oracle_lpf_opt.argtypes = [_P, _U64, _P, _U64]
        L.oracle_decode.restype = None
        L.oracle_decode.argtypes = [_P, _U64, _P, _U64]
        L.oracle_gap_bases.restype = None
        L.oracle_gap_bases.argtypes = [ctypes.c_uint32, _P]
        L.oracle_factorize_skip.restype = ctypes.c_int64
        L.oracle_factorize_skip.argtypes = [_P, _U64, ctypes.c_int, _P, _U64]
        L.oracle_factorize_exact.restype = ctypes.c_int64
        L.oracle_factorize_exact.argtypes = [_P, _U64, _P, _U64]
        L.oracle_factorize_exact_timed.restype = ctypes.c_int64
        L.oracle_factorize_exact_timed.argtypes = [_P, _U64, ctypes.POINTER(ctypes.c_double)]
        L.oracle_factorize_exact_smpl.restype = ctypes.c_int64
        L.oracle_factorize_exact_smpl.argtypes = [_P, _U64, ctypes.c_int, ctypes.c_int, _P, _U64]
        L.oracle_factorize_exact_smpl_timed.restype = ctypes.c_int64
        L.oracle_factorize_exact_smpl_timed.argtypes = [_P, _U64, ctypes.c_int, ctypes.c_int,
                                                        ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
        L.oracle_factorize_approx64.restype = ctypes.c_int64
        L.oracle_factorize_approx64.argtypes = [_P, _U64, ctypes.c_int, ctypes.c_uint32, ctypes.c_int, _P, _U64, _P]
        L.oracle_sss64.restype = ctypes.c_int64
        L.oracle_sss64.argtypes = [_P, _U64, _P, _U64, ctypes.POINTER(ctypes.c_int)]
        L.oracle_lpf_opt64.restype = ctypes.c_int64
        L.oracle_lpf_opt64.argtypes = [_P, _U64, _P, _U64]
        L.oracle_greedy_block.restype = ctypes.c_int64
        L.oracle_greedy_block.argtypes = [_P, _U64, ctypes.c_int, ctypes.c_uint32, ctypes.c_int, _P, _P,
                                          ctypes.POINTER(_U64), _P, _U64]
        L.oracle_num_threads.restype = ctypes.c_int
        L.oracle_num_threads.argtypes = []
        _lib = L
    return _lib


def _u8(T) -> np.ndarray:
    if isinstance(T, (bytes, bytearray)):
        T = np.frombuffer(bytes(T), np.uint8)
    return np.ascontiguousarray(T, dtype=np.uint8)


def _padded(T) -> np.ndarray:
    """Copy with zero padding (the oracle may read a few words past n, like the reference callers' padding)."""
    T = _u8(T)
    buf = np.zeros(T.size + 4096, np.uint8)
    buf[:T.size] = T
    return buf


def factorize(T, phr_mode: int = LPF_OPT, rk_seed: int = 42):
    """lz77_sss<u32>::factorize_approximate<greedy, phr_mode, 512> at p=1 -> ((z,2) u32 factors, stats[16])."""
    buf = _padded(T)
    n = _u8(T).size
    out = np.zeros((n + 2, 2), np.uint32)
    st = np.zeros(16, np.uint32)
    z = lib().oracle_factorize_approx(buf.ctypes.data_as(_P), n, phr_mode, rk_seed, out.ctypes.data_as(_P), n + 2,
                                      st.ctypes.data_as(_P))
    if z < 0:
        raise RuntimeError("oracle factorization failed")
    return out[:z].copy(), st


def factorize64(T, phr_mode: int = LPF_OPT, rk_seed: int = 42, fact_mode: int = 1, buf=None):
    """lz77_sss<u64>::factorize_approximate<fact_mode, phr_mode, 512> at p=1 -> ((z,2) u64 factors, stats[12]).
    The gap index has the reference's pos_t = uint64_t size (8-byte entries), so the stream differs from the
    uint32_t one in general.  `buf` may be a pre-padded copy (text + >= 4096 zero bytes) to skip the copy."""
    n = _u8(T).size
    if buf is None:
        buf = _padded(T)
    cap = n // 32 + 65536
    st = np.zeros(12, np.uint64)
    while True:
        out = np.zeros((cap, 2), np.uint64)
        z = lib().oracle_factorize_approx64(buf.ctypes.data_as(_P), n, phr_mode, rk_seed, fact_mode,
                                            out.ctypes.data_as(_P), cap, st.ctypes.data_as(_P))
        if z >= 0:
            return out[:z].copy(), st
        if cap >= n + 4:
            raise RuntimeError("oracle factorization failed")
        cap = n + 4


def sss64(T):
    buf = _padded(T)
    n = _u8(T).size
    out = np.zeros(2 * n // 512 * 4 + 1024, np.uint64)
    hr = ctypes.c_int()
    k = lib().oracle_sss64(buf.ctypes.data_as(_P), n, out.ctypes.data_as(_P), out.size, ctypes.byref(hr))
    if k < 0:
        out = np.zeros(n + 1, np.uint64)
        k = lib().oracle_sss64(buf.ctypes.data_as(_P), n, out.ctypes.data_as(_P), out.size, ctypes.byref(hr))
    return out[:k].copy(), bool(hr.value)


def lpf_opt64(T):
    buf = _padded(T)
    n = _u8(T).size
    out = np.zeros((n // 64 + 1024, 3), np.uint64)
    k = lib().oracle_lpf_opt64(buf.ctypes.data_as(_P), n, out.ctypes.data_as(_P), out.shape[0])
    if k < 0:
        raise RuntimeError("oracle lpf failed")
    return out[:k].copy()


def greedy_block(T, start: int, idxpos: int, end: int, table=None, wide: bool = False, phr_mode: int = LPF_OPT,
                 rk_seed: int = 42):
    """One block of the sharded greedy (oracle.hpp greedy_block) -> (factors (z,2) uint64, (exit_start,
    exit_idxpos), carried table (uint32 / uint64 array, pos + 1))."""
    buf = _padded(T)
    n = _u8(T).size
    dt = np.uint64 if wide else np.uint32
    tab = np.zeros(0, dt) if table is None else np.ascontiguousarray(table, dtype=dt).copy()
    cap = n + 4
    out = np.zeros((cap, 2), np.uint64)
    for _ in range(2):
        state = np.array([start, idxpos, end, 0, 0], np.uint64)
        ent = _U64(tab.size)
        z = lib().oracle_greedy_block(buf.ctypes.data_as(_P), n, phr_mode, rk_seed, int(wide), state.ctypes.data_as(_P),
                                      tab.ctypes.data_as(_P) if tab.size else None, ctypes.byref(ent),
                                      out.ctypes.data_as(_P), cap)
        if z == -2:  # the carried table was empty: size it (zeros) and run again
            tab = np.zeros(ent.value, dt)
            continue
        if z < 0:
            raise RuntimeError("oracle greedy block failed")
        return out[:z].copy(), (int(state[3]), int(state[4])), tab
    raise RuntimeError("oracle greedy block: table size")


def factorize_timed(T, phr_mode: int = LPF_OPT, rk_seed: int = 42):
    """Times the oracle factorization (output discarded into a running FNV-1a hash) -> (z, seconds, hash)."""
    buf = _padded(T)
    n = _u8(T).size
    sec, h = ctypes.c_double(), _U64()
    z = lib().oracle_factorize_timed(buf.ctypes.data_as(_P), n, phr_mode, rk_seed, ctypes.byref(sec), ctypes.byref(h))
    return int(z), sec.value, h.value


def factorize_timed_p(T, threads: int, phr_mode: int = LPF_OPT, rk_seed: int = 42):
    """CPU baseline at `threads` threads (every OpenMP stage; LPF in per-thread partitions as
    lpf_opt.cpp:46-56 when threads > 1, the reference's racy parallel greedy where
    lz77_sss.hpp:467-474 selects it) -> (z, seconds, hash, parallel_greedy_ran).  Timing only: at
    threads > 1 the phrases (and so the stream) may differ from the p = 1 parity stream."""
    buf = _padded(T)
    n = _u8(T).size
    sec, h, par = ctypes.c_double(), _U64(), ctypes.c_int()
    z = lib().oracle_factorize_timed_p(buf.ctypes.data_as(_P), n, phr_mode, rk_seed, threads, ctypes.byref(sec),
                                       ctypes.byref(h), ctypes.byref(par))
    return int(z), sec.value, h.value, bool(par.value)


def factorize_timed_p64(T, threads: int, phr_mode: int = LPF_OPT, rk_seed: int = 42, buf=None):
    """factorize_timed_p with pos_t = uint64_t (texts past 4 GiB, configs[3]); `buf` may be a pre-padded
    copy -> (z, seconds, hash, parallel_greedy_ran)."""
    n = _u8(T).size
    if buf is None:
        buf = _padded(T)
    sec, h, par = ctypes.c_double(), _U64(), ctypes.c_int()
    z = lib().oracle_factorize_timed_p64(buf.ctypes.data_as(_P), n, phr_mode, rk_seed, threads, ctypes.byref(sec),
                                         ctypes.byref(h), ctypes.byref(par))
    if z < 0:
        raise RuntimeError("oracle factorization failed")
    return int(z), sec.value, h.value, bool(par.value)


def factorize_p(T, threads: int, rk_seed: int = 42):
    """The CPU baseline's p-thread stream (LPF in `threads` partitions; the reference's racy parallel
    greedy where lz77_sss.hpp:467-474 selects it) -> (factors (z,2) uint32, parallel_greedy_ran).
    Validity tests of the timing leg only: it is not a parity stream."""
    buf = _padded(T)
    n = _u8(T).size
    cap = n + 4
    out = np.zeros((cap, 2), np.uint32)
    par = ctypes.c_int()
    z = lib().oracle_factorize_p(buf.ctypes.data_as(_P), n, threads, rk_seed, out.ctypes.data_as(_P), cap,
                                 ctypes.byref(par))
    if z < 0:
        raise RuntimeError("oracle factorize_p failed")
    return out[:z].copy(), bool(par.value)


def factorize_skip(T, phr_mode: int = LPF_OPT):
    """factorize_approximate<skip_phrases, phr_mode>: the gapped stream ((k,2) u32: {src,len} phrases, {gap,0})."""
    buf = _padded(T)
    n = _u8(T).size
    out = np.zeros((2 * n + 4, 2), np.uint32)
    z = lib().oracle_factorize_skip(buf.ctypes.data_as(_P), n, phr_mode, out.ctypes.data_as(_P), 2 * n + 4)
    if z < 0:
        raise RuntimeError("oracle skip_phrases factorization failed")
    return out[:z].copy()


def factorize_exact(T):
    """Exact greedy LZ77 restatement (factorize_exact lengths; PSV/NSV source rule) -> (z,2) u32 factors."""
    buf = _padded(T)
    n = _u8(T).size
    cap = n // 64 + 65536
    while True:
        out = np.zeros((cap, 2), np.uint32)
        z = lib().oracle_factorize_exact(buf.ctypes.data_as(_P), n, out.ctypes.data_as(_P), cap)
        if z >= 0:
            return out[:z].copy()
        if cap >= n + 1:
            raise RuntimeError("oracle exact factorization failed")
        cap = n + 1


NAIVE, WITH_SAMPLES, WITHOUT_SAMPLES = 0, 1, 2


def factorize_exact_smpl(T, mode=WITH_SAMPLES, p=1):
    """The reference's exact transform restated (oracle_exact.hpp): factorize_exact<greedy, lpf_opt,
    with_samples | without_samples> -> (z,2) u32 factors; p = 1 is the deterministic stream."""
    buf = _padded(T)
    n = _u8(T).size
    cap = n // 64 + 65536
    while True:
        out = np.zeros((cap, 2), np.uint32)
        z = lib().oracle_factorize_exact_smpl(buf.ctypes.data_as(_P), n, mode, p, out.ctypes.data_as(_P), cap)
        if z >= 0:
            return out[:z].copy()
        if cap >= n + 1:
            raise RuntimeError("oracle exact-smpl factorization failed")
        cap = n + 1


def factorize_exact_smpl_timed(T, mode=WITH_SAMPLES, p=1):
    """Times the exact transform restatement -> (z, seconds, seconds of its approximation stage)."""
    buf = _padded(T)
    n = _u8(T).size
    sec, sa = ctypes.c_double(), ctypes.c_double()
    z = lib().oracle_factorize_exact_smpl_timed(buf.ctypes.data_as(_P), n, mode, p, ctypes.byref(sec), ctypes.byref(sa))
    return int(z), sec.value, sa.value


def factorize_exact_timed(T):
    """Times the exact restatement -> (z, seconds)."""
    buf = _padded(T)
    n = _u8(T).size
    sec = ctypes.c_double()
    z = lib().oracle_factorize_exact_timed(buf.ctypes.data_as(_P), n, ctypes.byref(sec))
    return int(z), sec.value


def sss(T):
    buf = _padded(T)
    n = _u8(T).size
    out = np.zeros(n + 1, np.uint32)
    hr = ctypes.c_int()
    k = lib().oracle_sss(buf.ctypes.data_as(_P), n, out.ctypes.data_as(_P), n + 1, ctypes.byref(hr))
    return out[:k].copy(), bool(hr.value)


def q_bruteforce(T) -> np.ndarray:
    buf = _padded(T)
    n = _u8(T).size
    q = np.zeros(n + 1, np.uint8)
    lib().oracle_q_bruteforce(buf.ctypes.data_as(_P), n, q.ctypes.data_as(_P))
    return q[:max(n - 511, 0)]


def phi(T) -> np.ndarray:
    buf = _padded(T)
    n = _u8(T).size
    out = np.zeros(n + 1, np.uint64)
    lib().oracle_phi(buf.ctypes.data_as(_P), n, out.ctypes.data_as(_P))
    return out[:max(n - 511, 0)]


def sa_s(T):
    """(S, SA_S, LCP) of the oracle's LCE structure."""
    buf = _padded(T)
    n = _u8(T).size
    S, SA, LCP = (np.zeros(n + 1, np.uint32) for _ in range(3))
    k = lib().oracle_sa_s(buf.ctypes.data_as(_P), n, S.ctypes.data_as(_P), SA.ctypes.data_as(_P),
                          LCP.ctypes.data_as(_P), n + 1)
    return S[:k].copy(), SA[:k].copy(), LCP[:k].copy()


def lce(T, qi, qj) -> np.ndarray:
    buf = _padded(T)
    n = _u8(T).size
    qi = np.ascontiguousarray(qi, np.uint32)
    qj = np.ascontiguousarray(qj, np.uint32)
    out = np.zeros(qi.size, np.uint32)
    lib().oracle_lce(buf.ctypes.data_as(_P), n, qi.ctypes.data_as(_P), qj.ctypes.data_as(_P), qi.size,
                     out.ctypes.data_as(_P))
    return out


def lpf_opt(T) -> np.ndarray:
    """(beg, end, src) triples of build_LPF_opt at p=1."""
    buf = _padded(T)
    n = _u8(T).size
    out = np.zeros((n + 1, 3), np.uint32)
    k = lib().oracle_lpf_opt(buf.ctypes.data_as(_P), n, out.ctypes.data_as(_P), n + 1)
    return out[:k].copy()


def decode(F, n: int) -> np.ndarray:
    F = np.ascontiguousarray(F, np.uint32)
    out = np.zeros(max(n, 1), np.uint8)
    lib().oracle_decode(F.ctypes.data_as(_P), F.shape[0], out.ctypes.data_as(_P), n)
    return out[:n]


def gap_bases(rk_seed: int) -> list[int]:
    out = np.zeros(5, np.uint64)
    lib().oracle_gap_bases(rk_seed, out.ctypes.data_as(_P))
    return [int(x) for x in out]


def num_threads() -> int:
    return int(lib().oracle_num_threads())


def huffman(F, n: int) -> bytes:
    """The Huffman factor container (misc/huffman.hpp huff_writer) of a factor stream (oracle_huffman.cpp)."""
    f = np.ascontiguousarray(np.asarray(F, dtype=np.uint32).reshape(-1, 2))
    L = lib()
    L.oracle_huffman.restype = ctypes.c_int64
    L.oracle_huffman.argtypes = [_P, _U64, _U64, _P, _U64]
    size = L.oracle_huffman(f.ctypes.data_as(_P), f.shape[0], n, None, 0)
    out = np.zeros(max(size, 1), np.uint8)
    L.oracle_huffman(f.ctypes.data_as(_P), f.shape[0], n, out.ctypes.data_as(_P), size)
    return out[:size].tobytes()


def huffman_decode(buf, cap: int) -> np.ndarray:
    """Factors back from a Huffman container (huff_factor_iterator restated)."""
    b = np.frombuffer(bytes(buf), np.uint8)
    out = np.zeros((max(cap, 1), 2), np.uint32)
    L = lib()
    L.oracle_huffman_decode.restype = ctypes.c_int64
    L.oracle_huffman_decode.argtypes = [_P, _U64, _P, _U64]
    z = L.oracle_huffman_decode(b.ctypes.data_as(_P), b.size, out.ctypes.data_as(_P), cap)
    if z < 0:
        raise RuntimeError("invalid Huffman container")
    return out[:z].copy()
