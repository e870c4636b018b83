#!/bin/bash
set -eo pipefail
bash tools/gpu_quick.sh r04d "pred_and_bucket or lsd_base or medium or (stream_hash and rr) or c1_seeds or window"
LZ77SSS_DEBUG=1 timeout -k 10 120 python3 tools/rle_probe.py 1024 42 > gpurun_out/sa_s_debug.log 2>&1
grep -a "sa_s\|fast check\|greedy base" gpurun_out/sa_s_debug.log | head -60
