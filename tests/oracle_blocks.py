"""The block interface of lz77-sss_amd/sharded.py (HipBlocks) on the CPU oracle: the
gloo world-size-N tests drive sharded.factorize_sharded with it (test infrastructure only;
oracle.hpp greedy_block)."""
from __future__ import annotations

import numpy as np


class OracleBlocks:
    """The same interface on the CPU oracle (tests; oracle.hpp greedy_block)."""

    def __init__(self, text, n: int, pos64: bool = False, **params):
        import oracle

        self.o = oracle
        self.T = np.ascontiguousarray(text)
        self.wide = pos64
        self.params = params

    def prepare(self, S, runs: bool) -> int:
        want, _ = self.o.sss(self.T)
        assert np.array_equal(np.asarray(S, np.uint64), want.astype(np.uint64)), "gathered sync set differs"
        return 0

    def run(self, state, end: int, table):
        start, idxpos, _ = state
        dt = np.uint64 if self.wide else np.uint32
        tab = None if table is None else np.frombuffer(np.ascontiguousarray(table).tobytes(), dt)
        F, (es, ei), tab = self.o.greedy_block(self.T, start, idxpos, end, tab, wide=self.wide, **self.params)
        return F, (es, ei, 0), tab.view(np.uint8)

    def close(self):
        pass
