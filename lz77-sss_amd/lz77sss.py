"""Python mirror of the reference API over the C-ABI of liblz77sss_hip.so.

Mirrors ``lz77_sss<pos_t>`` for pos_t in {uint32_t, uint64_t} (include/lz77_sss/lz77_sss.hpp:72-203
of LukasNalbach/lz77-sss; ``pos64=True`` selects uint64_t, which texts past 2^32 - 16 bytes need):

* ``factorize_approximate(text, fact_mode=GREEDY, phr_mode=LPF_OPT, ...)``
  <- ``lz77_sss<>::factorize_approximate<fact_mode, phr_mode, tau>`` (:176-186)
* ``decode(factors, n)`` <- ``lz77_sss<>::decode`` (:202-203, algorithms/common.cpp:31-54)
* factors are an ``(z, 2)`` uint32 (uint64 for pos64) array of ``(src, len)`` =
  ``lz77_sss<>::factor`` (:129-147); a literal has ``len == 0`` and ``src`` = the byte.

There is no CPU fallback: if the HIP library or a gfx950 device is missing,
every compute call raises ``Lz77SssError``.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import numpy as np

LPF_NAIVE, LPF_LNF_NAIVE, LPF_OPT, LPF_LNF_OPT = 0, 1, 2, 3   # enum phrase_mode, lz77_sss.hpp:48-53
GREEDY_NAIVE, GREEDY, SKIP_PHRASES = 0, 1, 2                 # enum factorize_mode, lz77_sss.hpp:55-59
NAIVE, WITH_SAMPLES, WITHOUT_SAMPLES = 0, 1, 2               # enum transform_mode, lz77_sss.hpp:60-64
FULL_SA = 3                                                    # device extension: LPF over the full suffix array
DEFAULT_TAU = 512
OK, EINVAL, ENODEV, EHIP, ENOMEM, ECALLBACK, EINTERNAL = 0, -1, -2, -3, -4, -5, -6  # include/lz77sss.h

_HERE = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("LZ77SSS_LIB", _HERE / "lib" / "liblz77sss_hip.so"))


class Lz77SssError(RuntimeError):
    def __init__(self, msg: str, code: int = 0):
        super().__init__(msg)
        self.code = code


class Params(ctypes.Structure):
    _fields_ = [("phr_mode", ctypes.c_int32), ("fact_mode", ctypes.c_int32), ("tau", ctypes.c_uint32),
                ("rk_seed", ctypes.c_uint32), ("index_log2_size", ctypes.c_int32), ("device", ctypes.c_int32),
                ("log", ctypes.c_int32), ("num_threads", ctypes.c_uint16)]


_P = ctypes.c_void_p
_U64 = ctypes.c_uint64
_SYMBOLS = {
    # name: (restype, argtypes)
    "lz77sss_default_params": (None, [ctypes.POINTER(Params)]),
    "lz77sss_factorize_approx_u32": (ctypes.c_int, [_P, _U64, ctypes.POINTER(Params), _P, _P]),
    "lz77sss_factorize_exact_u32": (ctypes.c_int, [_P, _U64, ctypes.POINTER(Params), ctypes.c_int, _P, _P]),
    "lz77sss_factorize_approx_u64": (ctypes.c_int, [_P, _U64, ctypes.POINTER(Params), _P, _P]),
    "lz77sss_factorize_exact_u64": (ctypes.c_int, [_P, _U64, ctypes.POINTER(Params), ctypes.c_int, _P, _P]),
    "lz77sss_decode_u64": (ctypes.c_int, [_P, _U64, _P, _U64]),
    "lz77sss_decode_u64_device": (ctypes.c_int, [_P, _U64, _P, _U64, ctypes.c_int]),
    "lz77sss_serialize_factors64": (ctypes.c_int, [_P, _U64, _P]),
    "lz77sss_deserialize_factors64": (ctypes.c_int, [_P, _U64, _P]),
    "lz77sss_session_create64": (ctypes.c_int, [ctypes.c_int, _U64, ctypes.POINTER(_P)]),
    "lz77sss_session_is64": (ctypes.c_int, [_P]),
    "lz77sss_session_get_factors64": (ctypes.c_int, [_P, _P, _U64]),
    "lz77sss_session_get_lpf64": (ctypes.c_int, [_P, _P, _U64, ctypes.POINTER(_U64)]),
    "lz77sss_session_set_sss": (ctypes.c_int, [_P, _P, _U64, ctypes.c_int]),
    "lz77sss_session_prepare": (ctypes.c_int, [_P, ctypes.POINTER(Params), ctypes.c_int, ctypes.POINTER(_U64)]),
    "lz77sss_session_carried_copy": (ctypes.c_int, [_P, _P, _U64, ctypes.c_int]),
    "lz77sss_session_greedy_block": (ctypes.c_int, [_P, ctypes.POINTER(Params), _P, ctypes.POINTER(_U64)]),
    "lz77sss_session_spec_begin": (ctypes.c_int, [_P, ctypes.c_int, _U64]),
    "lz77sss_session_spec_resolve": (ctypes.c_int, [_P, _P, _U64, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]),
    "lz77sss_session_factorize_exact": (ctypes.c_int, [_P, ctypes.POINTER(Params), ctypes.c_int,
                                                       ctypes.POINTER(_U64)]),
    "lz77sss_decode_u32": (ctypes.c_int, [_P, _U64, _P, _U64]),
    "lz77sss_decode_u32_device": (ctypes.c_int, [_P, _U64, _P, _U64, ctypes.c_int]),
    "lz77sss_session_decode": (ctypes.c_int, [_P, _P, _U64, ctypes.POINTER(_U64)]),
    "lz77sss_session_verify": (ctypes.c_int, [_P, ctypes.POINTER(_U64), ctypes.POINTER(_U64)]),
    "lz77sss_session_create": (ctypes.c_int, [ctypes.c_int, _U64, ctypes.POINTER(_P)]),
    "lz77sss_session_load": (ctypes.c_int, [_P, _P, _U64]),
    "lz77sss_session_factorize": (ctypes.c_int, [_P, ctypes.POINTER(Params), ctypes.POINTER(_U64)]),
    "lz77sss_session_get_factors": (ctypes.c_int, [_P, _P, _U64]),
    "lz77sss_session_sss": (ctypes.c_int, [_P, ctypes.POINTER(_U64), ctypes.POINTER(ctypes.c_int)]),
    "lz77sss_session_get_sss": (ctypes.c_int, [_P, _P, _U64]),
    "lz77sss_session_sss_range": (ctypes.c_int, [_P, _U64, _U64, _U64, _U64, ctypes.POINTER(_U64),
                                                 ctypes.POINTER(ctypes.c_int)]),
    "lz77sss_session_get_sss64": (ctypes.c_int, [_P, _P, _U64]),
    "lz77sss_session_copy_sss64_device": (ctypes.c_int, [_P, _P, _U64]),
    "lz77sss_session_copy_factors_device": (ctypes.c_int, [_P, _P, _U64, ctypes.POINTER(_U64)]),
    "lz77sss_session_huffman": (ctypes.c_int, [_P, _P, _U64, ctypes.POINTER(_U64)]),
    "lz77sss_session_ssszip_gapped": (ctypes.c_int, [_P, _P, _U64, ctypes.POINTER(_U64)]),
    "lz77sss_session_gen_genome": (ctypes.c_int, [_P, _U64, _U64, ctypes.c_double, ctypes.c_uint32, _U64]),
    "lz77sss_session_get_sa_s": (ctypes.c_int, [_P, _P, _P, _U64]),
    "lz77sss_session_get_lpf": (ctypes.c_int, [_P, _P, _U64, ctypes.POINTER(_U64)]),
    "lz77sss_session_phase_times": (ctypes.c_int, [_P, _P, _P, ctypes.c_int]),
    "lz77sss_session_phase_mem": (ctypes.c_int, [_P, _P, _P, _P, ctypes.c_int]),
    "lz77sss_session_stats": (ctypes.c_int, [_P, _P, ctypes.c_int]),
    "lz77sss_session_sss_kernel_time": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_U64)]),
    "lz77sss_session_destroy": (None, [_P]),
    "lz77sss_gen_random_repetitive": (ctypes.c_int64, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                                       ctypes.c_double, ctypes.c_double, _P, _U64]),
    "lz77sss_gen_genome": (ctypes.c_int64, [_U64, _U64, ctypes.c_double, ctypes.c_uint32, _P]),
    "lz77sss_gen_genome_pos": (ctypes.c_int, [_U64, _U64, ctypes.c_double, ctypes.c_uint32, _U64, _P]),
    "lz77sss_last_error": (ctypes.c_char_p, []),
    "lz77sss_device_count": (ctypes.c_int, []),
}

_lib = None


def load_library(path: Path | str | None = None):
    """Loads liblz77sss_hip.so (raises Lz77SssError if it is missing)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = Path(path) if path else Path(os.environ.get("LZ77SSS_LIB", LIB_PATH))  # LZ77SSS_LIB: build variants (tools)
    if not p.exists():
        raise Lz77SssError(f"HIP library not built: {p} (run `make -C lz77-sss_amd`)")
    lib = ctypes.CDLL(str(p))
    for name, (res, args) in _SYMBOLS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def _check(rc: int):
    if rc != 0:
        msg = load_library().lz77sss_last_error()
        raise Lz77SssError(f"lz77sss error {rc}: {msg.decode() if msg else ''}", rc)


def _as_u8(text) -> np.ndarray:
    if isinstance(text, (bytes, bytearray, memoryview)):
        return np.frombuffer(bytes(text), dtype=np.uint8)
    a = np.ascontiguousarray(text)
    if a.dtype != np.uint8:
        a = a.view(np.uint8)
    return a


def params(phr_mode=LPF_OPT, fact_mode=GREEDY, tau=DEFAULT_TAU, rk_seed=42, index_log2_size=0, device=0,
           log=False, num_threads=0) -> Params:
    p = Params()
    load_library().lz77sss_default_params(ctypes.byref(p))
    p.phr_mode, p.fact_mode, p.tau, p.rk_seed = phr_mode, fact_mode, tau, rk_seed
    p.index_log2_size, p.device, p.log, p.num_threads = index_log2_size, device, int(log), num_threads
    return p


class Block(ctypes.Structure):
    """lz77sss_block: one block of a sharded factorization (include/lz77sss.h)."""
    _fields_ = [("start", ctypes.c_uint64), ("idxpos", ctypes.c_uint64), ("zmask", ctypes.c_uint32),
                ("carried", ctypes.c_int32), ("end", ctypes.c_uint64), ("exit_start", ctypes.c_uint64),
                ("exit_idxpos", ctypes.c_uint64), ("exit_zmask", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


class Session:
    """Device-resident session: the text stays in HBM across calls."""

    def __init__(self, max_n: int, device: int = 0, pos64: bool = False):
        lib = load_library()
        h = _P()
        create = lib.lz77sss_session_create64 if pos64 else lib.lz77sss_session_create
        _check(create(device, max_n, ctypes.byref(h)))
        self._h = h
        self.n = 0
        self.pos64 = pos64

    def close(self):
        if self._h:
            load_library().lz77sss_session_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def load(self, text):
        a = _as_u8(text)
        _check(load_library().lz77sss_session_load(self._h, a.ctypes.data_as(_P), a.size))
        self.n = a.size

    def factorize(self, **kw) -> int:
        p = params(**kw)
        z = _U64()
        _check(load_library().lz77sss_session_factorize(self._h, ctypes.byref(p), ctypes.byref(z)))
        return z.value

    def factorize_exact(self, transf_mode=WITHOUT_SAMPLES, **kw) -> int:
        """factorize_exact<greedy, lpf_opt, transf_mode>: canonical greedy LZ77 lengths.  naive /
        with_samples / without_samples: the sample-index path (csrc/smpl.hip); FULL_SA: LPF over
        the full suffix array (csrc/exact.hip)."""
        p = params(**kw)
        z = _U64()
        _check(load_library().lz77sss_session_factorize_exact(self._h, ctypes.byref(p), transf_mode, ctypes.byref(z)))
        return z.value

    # ---- sharded factorization (include/lz77sss.h; lz77-sss_amd/sharded.py drives it)
    def set_sss(self, S, has_runs: bool, device_ptr: int | None = None):
        """Loads an externally built sync set (uint64 host array, or a device pointer + len(S))."""
        if device_ptr is not None:
            _check(load_library().lz77sss_session_set_sss(self._h, _P(device_ptr), int(S), int(has_runs)))
            return
        a = np.ascontiguousarray(S, dtype=np.uint64)
        _check(load_library().lz77sss_session_set_sss(self._h, a.ctypes.data_as(_P), a.size, int(has_runs)))

    def prepare(self, external_sss: bool = True, **kw) -> int:
        """Phases before the greedy emitter; returns the carried table's size in bytes."""
        p = params(**kw)
        b = _U64()
        _check(load_library().lz77sss_session_prepare(self._h, ctypes.byref(p), int(external_sss), ctypes.byref(b)))
        return b.value

    def carried_get(self, nbytes: int, device_ptr: int | None = None) -> np.ndarray | None:
        if device_ptr is not None:
            _check(load_library().lz77sss_session_carried_copy(self._h, _P(device_ptr), nbytes, 0))
            return None
        out = np.empty(max(nbytes, 1), np.uint8)
        _check(load_library().lz77sss_session_carried_copy(self._h, out.ctypes.data_as(_P), nbytes, 0))
        return out[:nbytes]

    def carried_set(self, table=None, nbytes: int = 0, device_ptr: int | None = None):
        if device_ptr is not None:
            _check(load_library().lz77sss_session_carried_copy(self._h, _P(device_ptr), nbytes, 1))
            return
        a = np.ascontiguousarray(table, dtype=np.uint8)
        _check(load_library().lz77sss_session_carried_copy(self._h, a.ctypes.data_as(_P), a.size, 1))

    def greedy_block(self, start: int, idxpos: int, zmask: int, carried: bool, end: int, seed: bool = False, **kw):
        """The greedy chain of [start, end) -> (factor count, (exit_start, exit_idxpos, exit_zmask)).
        seed (not carried): the table starts as the gap positions before start (a speculative lead-in)."""
        p = params(**kw)
        b = Block(start, idxpos, zmask, int(carried), end, 0, 0, 0, 1 if (seed and not carried) else 0)
        z = _U64()
        _check(load_library().lz77sss_session_greedy_block(self._h, ctypes.byref(p), ctypes.byref(b), ctypes.byref(z)))
        return z.value, (b.exit_start, b.exit_idxpos, b.exit_zmask)

    def spec_begin(self, part: int = 0, block_start: int = 0):
        """The next greedy_block is part `part` of a speculative block starting at `block_start`
        (part 0: from the speculated carried table now in the session)."""
        _check(load_library().lz77sss_session_spec_begin(self._h, part, block_start))

    def spec_resolve(self, table=None, nbytes: int = 0, parts: int = 1, device_ptr: int | None = None) -> int:
        """Checks the speculative block's parts against the true entry table (host array or device
        pointer) and returns how many leading parts stand (their factors / exit states are the
        true ones).  The carried table becomes their writes over the true entry table: the exit
        table when all stand, else the table to re-walk the rest with (parts=0: the true table)."""
        acc = ctypes.c_int()
        if device_ptr is not None:
            _check(load_library().lz77sss_session_spec_resolve(self._h, _P(device_ptr), nbytes, parts,
                                                                ctypes.byref(acc)))
        else:
            a = np.ascontiguousarray(table, dtype=np.uint8)
            _check(load_library().lz77sss_session_spec_resolve(self._h, a.ctypes.data_as(_P), a.size, parts,
                                                                ctypes.byref(acc)))
        return acc.value

    def factors(self, z: int) -> np.ndarray:
        if self.pos64:
            out = np.empty((max(z, 1), 2), np.uint64)
            _check(load_library().lz77sss_session_get_factors64(self._h, out.ctypes.data_as(_P), z))
            return out[:z]
        out = np.empty((max(z, 1), 2), np.uint32)
        _check(load_library().lz77sss_session_get_factors(self._h, out.ctypes.data_as(_P), z))
        return out[:z]

    def decode(self, out: bool = True, verify: bool = True):
        """Decodes the last factorization on the device (csrc/decode.hip).
        Returns (text or None, mismatches vs the loaded text or None)."""
        buf = np.empty(max(self.n, 1), np.uint8) if out else None
        m = _U64()
        _check(load_library().lz77sss_session_decode(self._h, buf.ctypes.data_as(_P) if out else None,
                                                     self.n if out else 0, ctypes.byref(m) if verify else None))
        return (buf[:self.n] if out else None), (m.value if verify else None)

    def verify(self, first: bool = False):
        """Positions of the loaded text that the last factorization does not reproduce, checked in
        HBM without decoding (lz77sss_session_verify; 0 <=> decode(F) == T; any size).  With
        first=True: (count, smallest bad position or None)."""
        b, f = _U64(), _U64()
        _check(load_library().lz77sss_session_verify(self._h, ctypes.byref(b), ctypes.byref(f)))
        if first:
            return b.value, (None if f.value == (1 << 64) - 1 else f.value)
        return b.value

    def sss(self):
        s, r = _U64(), ctypes.c_int()
        _check(load_library().lz77sss_session_sss(self._h, ctypes.byref(s), ctypes.byref(r)))
        if self.pos64:
            return self.sync_set64(s.value), bool(r.value)
        out = np.empty(max(s.value, 1), np.uint32)
        _check(load_library().lz77sss_session_get_sss(self._h, out.ctypes.data_as(_P), s.value))
        return out[:s.value], bool(r.value)

    def sss_range(self, first: int = 0, end: int = 2**64 - 1, base: int = 0, window: int = 0):
        """pos_t = uint64_t sync set S n [first, end) of the loaded text, + base (csrc/sss.hip
        build_sss_range).  Returns (count, has_runs); the positions stay in HBM."""
        s, r = _U64(), ctypes.c_int()
        _check(load_library().lz77sss_session_sss_range(self._h, first, end, base, window, ctypes.byref(s),
                                                        ctypes.byref(r)))
        return s.value, bool(r.value)

    def sync_set64(self, s: int) -> np.ndarray:
        out = np.empty(max(s, 1), np.uint64)
        _check(load_library().lz77sss_session_get_sss64(self._h, out.ctypes.data_as(_P), s))
        return out[:s]

    def copy_sync_set64(self, dst_ptr: int, cap: int):
        """Device-to-device copy of the sss_range result to a device address (same device)."""
        _check(load_library().lz77sss_session_copy_sss64_device(self._h, _P(dst_ptr), cap))

    def factor_bytes(self) -> int:
        """Size of the last factorization in the session's layout (8 or 16 bytes per factor)."""
        b = _U64()
        _check(load_library().lz77sss_session_copy_factors_device(self._h, None, 0, ctypes.byref(b)))
        return b.value

    def copy_factors(self, dst_ptr: int, cap_bytes: int) -> int:
        """Copies the last factorization's raw pairs to a device (or host) address; returns the bytes."""
        b = _U64()
        _check(load_library().lz77sss_session_copy_factors_device(self._h, _P(dst_ptr), cap_bytes, ctypes.byref(b)))
        return b.value

    def huffman(self) -> np.ndarray:
        """Huffman factor container (bytes) of the last factorization (csrc/huffman.hip)."""
        sz = _U64()
        _check(load_library().lz77sss_session_huffman(self._h, None, 0, ctypes.byref(sz)))
        out = np.empty(max(sz.value, 1), np.uint8)
        _check(load_library().lz77sss_session_huffman(self._h, out.ctypes.data_as(_P), sz.value, ctypes.byref(sz)))
        return out[:sz.value]

    def ssszip_gapped(self) -> np.ndarray:
        """ssszip's gapped container (bytes) of the last skip_phrases factorization (csrc/ssszip.hip)."""
        sz = _U64()
        _check(load_library().lz77sss_session_ssszip_gapped(self._h, None, 0, ctypes.byref(sz)))
        out = np.empty(max(sz.value, 1), np.uint8)
        _check(load_library().lz77sss_session_ssszip_gapped(self._h, out.ctypes.data_as(_P), sz.value,
                                                           ctypes.byref(sz)))
        return out[:sz.value]

    def gen_genome(self, n: int, base_len: int, mut_rate: float, seed: int, offset: int = 0):
        """Generates bytes [offset, offset + n) of a chr19-style text directly in HBM."""
        _check(load_library().lz77sss_session_gen_genome(self._h, n, base_len, mut_rate, seed, offset))
        self.n = n

    def sync_set(self, s: int) -> np.ndarray:
        out = np.empty(max(s, 1), np.uint32)
        _check(load_library().lz77sss_session_get_sss(self._h, out.ctypes.data_as(_P), s))
        return out[:s]

    def sa_s(self, s: int):
        sa, lcp = np.empty(max(s, 1), np.uint32), np.empty(max(s, 1), np.uint32)
        _check(load_library().lz77sss_session_get_sa_s(self._h, sa.ctypes.data_as(_P), lcp.ctypes.data_as(_P), s))
        return sa[:s], lcp[:s]

    def lpf(self) -> np.ndarray:
        c = _U64()
        if self.pos64:
            _check(load_library().lz77sss_session_get_lpf64(self._h, None, 0, ctypes.byref(c)))
            out = np.empty((max(c.value, 1), 3), np.uint64)
            _check(load_library().lz77sss_session_get_lpf64(self._h, out.ctypes.data_as(_P), c.value, ctypes.byref(c)))
            return out[:c.value]
        _check(load_library().lz77sss_session_get_lpf(self._h, None, 0, ctypes.byref(c)))
        out = np.empty((max(c.value, 1), 3), np.uint32)
        _check(load_library().lz77sss_session_get_lpf(self._h, out.ctypes.data_as(_P), c.value, ctypes.byref(c)))
        return out[:c.value]

    def stats(self) -> list[int]:
        out = np.zeros(32, np.uint64)
        k = load_library().lz77sss_session_stats(self._h, out.ctypes.data_as(_P), 32)
        return [int(x) for x in out[:max(k, 0)]]

    def _phase_list(self) -> list[tuple[str, float]]:
        """(name, ms) per phase of the last call, in order; a repeated name (a phase run again, e.g.
        a retried task table) is kept as name#2, name#3, ..."""
        ms = (ctypes.c_double * 32)()
        names = (ctypes.c_char_p * 32)()
        k = load_library().lz77sss_session_phase_times(self._h, ms, names, 32)
        if k < 0:
            _check(k)
        out, seen = [], {}
        for i in range(k):
            nm = names[i].decode()
            seen[nm] = seen.get(nm, 0) + 1
            out.append((nm if seen[nm] == 1 else f"{nm}#{seen[nm]}", ms[i]))
        return out

    def phase_times(self) -> dict[str, float]:
        return dict(self._phase_list())

    def phase_mem(self) -> dict[str, dict[str, int]]:
        """Per phase of the last call (lz77sss_session_phase_mem): device bytes the process's buffers
        held when the phase was enqueued, their peak during it, and the GPU's free memory then (all
        process-wide: every session of the process counts).  Names pair with the C API's entries by
        position, duplicates kept as name#k."""
        names = [nm for nm, _ in self._phase_list()]
        h, p, f = (np.zeros(32, np.uint64) for _ in range(3))
        k = load_library().lz77sss_session_phase_mem(self._h, h.ctypes.data_as(_P), p.ctypes.data_as(_P),
                                                      f.ctypes.data_as(_P), 32)
        if k < 0:
            _check(k)
        return {names[i]: {"held": int(h[i]), "peak": int(p[i]), "hbm_free": int(f[i])}
                for i in range(min(k, len(names)))}

    def sss_kernel_time(self):
        ms, b = ctypes.c_double(), _U64()
        _check(load_library().lz77sss_session_sss_kernel_time(self._h, ctypes.byref(ms), ctypes.byref(b)))
        return ms.value, b.value


def factorize_approximate(text, fact_mode=GREEDY, phr_mode=LPF_OPT, tau=DEFAULT_TAU, rk_seed=42, device=0,
                          log=False, pos64=False) -> np.ndarray:
    """lz77_sss<pos_t>::factorize_approximate: returns the (z, 2) uint32 (pos64: uint64) factor array."""
    a = _as_u8(text)
    with Session(max(a.size, 1), device, pos64=pos64) as s:
        s.load(a)
        z = s.factorize(phr_mode=phr_mode, fact_mode=fact_mode, tau=tau, rk_seed=rk_seed, device=device, log=log)
        return s.factors(z)


def factorize_exact(text, transf_mode=None, fact_mode=GREEDY, phr_mode=LPF_OPT, tau=DEFAULT_TAU, device=0,
                    log=False) -> np.ndarray:
    """lz77_sss<>::factorize_exact: returns the (z, 2) uint32 factor array (exact greedy LZ77)."""
    a = _as_u8(text)
    with Session(max(a.size, 1), device) as s:
        s.load(a)
        z = s.factorize_exact(WITHOUT_SAMPLES if transf_mode is None else transf_mode, phr_mode=phr_mode,
                              fact_mode=fact_mode, tau=tau, device=device, log=log)
        return s.factors(z)


def decode(factors: np.ndarray, n: int) -> np.ndarray:
    """lz77_sss<>::decode (host, sequential as in the reference); uint64 factors use pos_t = uint64_t."""
    wide = np.asarray(factors).dtype == np.uint64
    f = np.ascontiguousarray(factors, dtype=np.uint64 if wide else np.uint32).reshape(-1, 2)
    out = np.empty(max(n, 1), np.uint8)
    fn = load_library().lz77sss_decode_u64 if wide else load_library().lz77sss_decode_u32
    _check(fn(f.ctypes.data_as(_P), f.shape[0], out.ctypes.data_as(_P), n))
    return out[:n]


def decode_device(factors: np.ndarray, n: int, device: int = 0) -> np.ndarray:
    """Same as decode, on the device (pointer jumping, csrc/decode.hip)."""
    wide = np.asarray(factors).dtype == np.uint64
    f = np.ascontiguousarray(factors, dtype=np.uint64 if wide else np.uint32).reshape(-1, 2)
    out = np.empty(max(n, 1), np.uint8)
    fn = load_library().lz77sss_decode_u64_device if wide else load_library().lz77sss_decode_u32_device
    _check(fn(f.ctypes.data_as(_P), f.shape[0], out.ctypes.data_as(_P), n, device))
    return out[:n]


def serialize_factors64(factors: np.ndarray) -> bytes:
    """The reference's pos_t = uint64_t factor stream: 5 + 5 bytes per factor (lz77_sss.hpp:149-173)."""
    f = np.ascontiguousarray(factors, dtype=np.uint64).reshape(-1, 2)
    out = np.empty(max(10 * f.shape[0], 1), np.uint8)
    _check(load_library().lz77sss_serialize_factors64(f.ctypes.data_as(_P), f.shape[0], out.ctypes.data_as(_P)))
    return out[:10 * f.shape[0]].tobytes()


def deserialize_factors64(data: bytes) -> np.ndarray:
    b = np.frombuffer(data, np.uint8)
    nf = b.size // 10
    out = np.empty((max(nf, 1), 2), np.uint64)
    _check(load_library().lz77sss_deserialize_factors64(b.ctypes.data_as(_P), nf, out.ctypes.data_as(_P)))
    return out[:nf]


def gen_random_repetitive(min_size: int, max_size: int, seed: int, rep: float = -1.0, run: float = -1.0) -> np.ndarray:
    """random_repetitive_string (utils.hpp:579-640) with a seed instead of std::random_device."""
    buf = np.empty(max_size + 16, np.uint8)
    n = load_library().lz77sss_gen_random_repetitive(min_size, max_size, seed, rep, run, buf.ctypes.data_as(_P),
                                                     max_size)
    if n < 0:
        raise Lz77SssError("generator failed")
    return buf[:n].copy()


def gen_genome(n: int, base_len: int, mut_rate: float, seed: int) -> np.ndarray:
    buf = np.empty(max(n, 1), np.uint8)
    load_library().lz77sss_gen_genome(n, base_len, mut_rate, seed, buf.ctypes.data_as(_P))
    return buf[:n]


def gen_genome_pos(n: int, base_len: int, mut_rate: float, seed: int, offset: int = 0, pad: int = 0) -> np.ndarray:
    """The chr19-style text of Session.gen_genome (position-hashed), on the host; `pad` zero bytes follow."""
    buf = np.zeros(max(n + pad, 1), np.uint8)
    _check(load_library().lz77sss_gen_genome_pos(n, base_len, mut_rate, seed, offset, buf.ctypes.data_as(_P)))
    return buf[:n + pad]
