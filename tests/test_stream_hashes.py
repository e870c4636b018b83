"""Full-size streams pinned by the oracle's SHA-256 (tests/golden/stream_hashes.json, written in the
container by tests/golden/make_stream_hashes.py): the device regenerates each text from its seeded
generator, factorizes it and hashes the factor stream.  Bit-exact parity at sizes where re-running the
oracle on the GPU box would cost minutes (the 1 GiB headline and genome texts, a 4 GiB + 3 MiB
chr19-style text at 0.1 % mutations with pos_t = uint64_t)."""
from __future__ import annotations

import hashlib
import json
from pathlib import Path

import numpy as np
import pytest

from conftest import GOLDEN

DB = json.loads((GOLDEN / "stream_hashes.json").read_text()) if (GOLDEN / "stream_hashes.json").exists() else {}


def _sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).view(np.uint8)).hexdigest()


def test_hash_db_complete():
    assert {"rr_1gib", "genome_1gib", "rr_1gib_lpf_lnf", "rr_1gib_exact_lengths"} <= set(DB), \
        "run tests/golden/make_stream_hashes.py"
    for e in DB.values():
        assert len(e["stream_sha256"]) == 64 and e["z"] > 0


@pytest.mark.gpu
@pytest.mark.slow
@pytest.mark.parametrize("name", sorted(DB))
def test_full_size_stream_hash(lz, name):
    e = DB[name]
    a, n = e["args"], e["n"]
    pos64 = e["pos_bits"] == 64
    with lz.Session(n, pos64=pos64) as s:
        if e["kind"] == "random_repetitive":
            T = lz.gen_random_repetitive(n, n, a["seed"], a["rep"], a["run"])
            assert _sha(T) == e["text_sha256"]
            s.load(T)
            del T
        elif e["kind"] == "genome":
            T = lz.gen_genome(n, a["base_len"], a["mut"], a["seed"])
            assert _sha(T) == e["text_sha256"]
            s.load(T)
            del T
        else:  # generated in HBM (the host generator of make_stream_hashes.py makes the same bytes)
            s.gen_genome(n, a["base_len"], a["mut"], a["seed"])
        mode = e.get("mode", "lpf_opt")
        if mode == "exact_lengths":  # configs[4]: the sample-index path (transf_mode with_samples)
            z = s.factorize_exact(transf_mode=lz.WITH_SAMPLES)
            F = s.factors(z)
            assert s.verify() == 0
            assert z == e["z"]
            assert _sha(F[:, 1].astype("<u4")) == e["stream_sha256"]
            return
        z = s.factorize(phr_mode=lz.LPF_LNF_OPT if mode == "lpf_lnf_opt" else lz.LPF_OPT)
        st = s.stats()
        F = s.factors(z)
    assert z == e["z"]
    assert st[:12] == e["stats"]
    assert _sha(F.astype("<u8" if pos64 else "<u4")) == e["stream_sha256"]
