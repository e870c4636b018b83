#!/bin/bash
# k_segmerge output-run cap A/B (sa_s phase) on rr and genome.
set -o pipefail
mkdir -p gpurun_out
for wl in rr genome; do
  for o in 16 8 4 2; do
    LZ77SSS_SEGMERGE_OPW=$o timeout -k 10 150 python -u tools/phase_time.py $wl 5 >> gpurun_out/phase_r03q.log 2>&1 || exit 1
  done
done
cat gpurun_out/phase_r03q.log
