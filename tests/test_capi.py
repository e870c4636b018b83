"""CPU tests of the C-ABI library: it loads, exports every symbol of include/lz77sss.h, host-side entry
points behave, and compute calls fail loudly (no CPU fallback) when no device is present."""
from __future__ import annotations

import ctypes
import re

import numpy as np
import pytest

from conftest import ROOT, load_golden


def header_symbols():
    text = (ROOT / "include" / "lz77sss.h").read_text()
    return sorted(set(re.findall(r"\b(lz77sss_\w+)\s*\(", text)))


def test_header_declares_the_api():
    syms = header_symbols()
    for must in ("lz77sss_factorize_approx_u32", "lz77sss_decode_u32", "lz77sss_session_create",
                 "lz77sss_session_factorize", "lz77sss_default_params"):
        assert must in syms


def test_library_exports_every_header_symbol(lz):
    lib = ctypes.CDLL(str(lz.LIB_PATH))
    missing = [s for s in header_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    assert set(lz._SYMBOLS) >= set(header_symbols())


def test_default_params(lz):
    p = lz.Params()
    lz.load_library().lz77sss_default_params(ctypes.byref(p))
    assert (p.phr_mode, p.fact_mode, p.tau, p.index_log2_size, p.device) == (lz.LPF_OPT, lz.GREEDY, 512, 0, 0)


@pytest.mark.parametrize("name", ["c1_seed1", "periodic", "zeros_10k", "edge_n1"])
def test_decode_host(lz, name):
    g = load_golden(name)
    assert np.array_equal(lz.decode(g["factors"], g["text"].size), g["text"])


def test_decode_rejects_invalid_stream(lz):
    F = np.array([[65, 0], [5, 3]], np.uint32)  # source 5 >= position 1
    with pytest.raises(lz.Lz77SssError):
        lz.decode(F, 4)
    with pytest.raises(lz.Lz77SssError):
        lz.decode(np.array([[65, 0]], np.uint32), 3)  # stream shorter than n


def test_generators_deterministic(lz):
    a = lz.gen_random_repetitive(10000, 200000, 5)
    b = lz.gen_random_repetitive(10000, 200000, 5)
    c = lz.gen_random_repetitive(10000, 200000, 6)
    assert np.array_equal(a, b) and not np.array_equal(a[:1000], c[:1000])
    assert 10000 <= a.size <= 200000
    g = load_golden("c1_seed1")
    assert np.array_equal(lz.gen_random_repetitive(10000, 200000, 1), g["text"])
    x = lz.gen_genome(1 << 16, 1 << 12, 0.001, 7)
    assert set(np.unique(x)) <= set(b"ACGT")


def test_no_cpu_fallback_without_device(lz):
    if lz.load_library().lz77sss_device_count() > 0:
        pytest.skip("a device is present")
    T = lz.gen_random_repetitive(10000, 20000, 1)
    with pytest.raises(lz.Lz77SssError):
        lz.factorize_approximate(T)
    with pytest.raises(lz.Lz77SssError):
        lz.Session(1 << 20)


def build_cpp_client(tmp_path):
    import subprocess

    exe = tmp_path / "api_roundtrip"
    src = ROOT / "tests" / "cpp" / "api_roundtrip.cpp"
    libdir = ROOT / "lz77-sss_amd" / "lib"
    subprocess.run(["g++", "-O1", "-std=c++20", str(src), "-o", str(exe), f"-L{libdir}", "-llz77sss_hip",
                    f"-Wl,-rpath,{libdir}"], check=True)
    return exe


def test_cpp_mirror_compiles_and_fails_loudly_without_device(lz, tmp_path):
    """The C++ template mirror (lz77-sss_amd/host/lz77_sss.hpp) builds against the C-ABI; without a
    device the factorization raises lz77_sss_error(ENODEV) instead of falling back to the CPU."""
    import subprocess

    exe = build_cpp_client(tmp_path)
    if lz.load_library().lz77sss_device_count() > 0:
        pytest.skip("a device is present (the GPU test runs the binary)")
    r = subprocess.run([str(exe), "1"], capture_output=True, text=True)
    assert r.returncode == 2, r.stdout + r.stderr
