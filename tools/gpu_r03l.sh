#!/bin/bash
# Greedy walk occupancy A/B (product = 8 waves/SIMD, lib_var walk5 / walk6) on genome and rr.
set -o pipefail
mkdir -p gpurun_out
for wl in genome rr; do
  for v in product lz77-sss_amd/lib_var/walk5.so lz77-sss_amd/lib_var/walk6.so product; do
    if [ "$v" = product ]; then timeout -k 10 200 python -u tools/greedy_time.py $wl 4 >> gpurun_out/greedy_ab.log 2>&1 || exit 1
    else LZ77SSS_LIB=$v timeout -k 10 200 python -u tools/greedy_time.py $wl 4 >> gpurun_out/greedy_ab.log 2>&1 || exit 1; fi
  done
done
cat gpurun_out/greedy_ab.log
