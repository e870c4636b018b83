#!/bin/bash
# tail entry state of the c1_seed2 fixture at chunk 128 vs 512 (LZ77SSS_DEBUG lines)
mkdir -p gpurun_out
for ch in 128 512; do
  LZ77SSS_DEBUG=1 LZ77SSS_GAP_CHUNK=$ch timeout -k 10 100 python3 -c "
import sys, numpy as np; sys.path.insert(0, 'lz77-sss_amd'); import lz77sss as lz
g = np.load('tests/golden/c1_seed2.npz'); T = g['text']
with lz.Session(T.size) as s:
    s.load(T); z = s.factorize(); F = s.factors(z); print('match', np.array_equal(F, g['factors']))
" > gpurun_out/diag2_$ch.log 2>&1 || exit 1
  echo "== CH=$ch"; grep -E "tail entry|match|greedy \|I\||delta" gpurun_out/diag2_$ch.log | head -12
done
