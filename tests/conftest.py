"""Shared fixtures.  `-m gpu` tests need a gfx950 device; everything else runs on CPU."""
from __future__ import annotations

import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / "lz77-sss_amd"
GOLDEN = Path(__file__).resolve().parent / "golden"
sys.path.insert(0, str(PKG))
sys.path.insert(0, str(ROOT / "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device; parity through the C-ABI")
    config.addinivalue_line("markers", "slow: large inputs (seconds to a minute)")


def _ensure_built():
    lib = PKG / "lib" / "liblz77sss_hip.so"
    if not lib.exists():
        subprocess.run(["make", "-s", "-C", str(PKG), "-j8"], check=True)
    orc = ROOT / "oracle" / "_build" / "liboracle.so"
    if not orc.exists():
        subprocess.run(["make", "-s", "-C", str(ROOT / "oracle"), "-j8"], check=True)


@pytest.fixture(scope="session")
def lz():
    _ensure_built()
    import lz77sss

    lz77sss.load_library()
    return lz77sss


@pytest.fixture(scope="session")
def orc():
    _ensure_built()
    import oracle

    oracle.lib()
    return oracle


def golden_names():
    return sorted(p.stem for p in GOLDEN.glob("*.npz"))


def load_golden(name):
    with np.load(GOLDEN / f"{name}.npz", allow_pickle=False) as d:
        return {k: d[k] for k in d.files}


@pytest.fixture(scope="session")
def session(lz):
    """One device session reused by the GPU tests (grows on demand)."""
    s = {"sess": None, "cap": 0}

    def get(n):
        if s["sess"] is None or n > s["cap"]:
            if s["sess"] is not None:
                s["sess"].close()
            cap = max(n, 1 << 22)
            s["sess"], s["cap"] = lz.Session(cap), cap
        return s["sess"]

    yield get
    if s["sess"] is not None:
        s["sess"].close()
