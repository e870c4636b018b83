#!/bin/bash
# greedy chunk length sweep on genome only (LZ77SSS_GAP_CHUNK)
set -o pipefail
mkdir -p gpurun_out
for ch in 32 64 128; do
  LZ77SSS_GAP_CHUNK=$ch timeout -k 10 200 python3 tools/prof_step.py genome 3 > gpurun_out/chunk2_genome_$ch.log 2>&1 || exit 1
  echo "genome CH=$ch: $(grep '^step' gpurun_out/chunk2_genome_$ch.log | tail -3 | sed -e 's/.*ms  phases=//' -e 's/stats.*//' -e "s/'sss.*'greedy'/greedy/" | tr '\n' ' ')"
done
