#!/bin/bash
# kernel trace of tools/prof_step.py <wl> 2 into gpurun_out/tr_<tag>_<wl>, then the parity tests of the greedy/SA_S paths
set -eo pipefail
TAG=$1; WL=${2:-rr}
REPO=$(pwd); OUT=$REPO/gpurun_out; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d "$OUT/tr_${TAG}_$WL" -o run -- python3 "$REPO/tools/prof_step.py" "$WL" 2 > "$OUT/tr_${TAG}_$WL.log" 2>&1
tail -3 "$OUT/tr_${TAG}_$WL.log"
