#!/bin/bash
# greedy chunk length sweep (LZ77SSS_GAP_CHUNK): phase times of prof_step steps on rr and genome
set -o pipefail
mkdir -p gpurun_out
for wl in rr genome; do
  for ch in 128 256 512 1024; do
    LZ77SSS_GAP_CHUNK=$ch timeout -k 10 200 python3 tools/prof_step.py $wl 3 > gpurun_out/chunk_${wl}_$ch.log 2>&1 || exit 1
    echo "$wl CH=$ch: $(grep '^step' gpurun_out/chunk_${wl}_$ch.log | tail -3 | sed -e 's/.*ms  phases=//' -e 's/stats.*//' | tr '\n' ' ' | cut -c1-400)"
  done
done
