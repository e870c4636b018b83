#!/bin/bash
# Combined: greedy A/B (k_pb_apply XCD remap in all builds; walk occupancy 8 / 5 / 6),
# then the speculative-block checks (lead=1 rejection, 4 GiB acceptance report).
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_r03l.sh || exit 1
bash tools/gpu_r03k.sh
