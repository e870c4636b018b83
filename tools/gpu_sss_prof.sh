#!/bin/bash
# SSS-phase kernel trace of one workload (from the repo root via gpurun): tools/gpu_sss_prof.sh <tag> <rr|genome>
set -eo pipefail
TAG=$1; WL=$2
REPO=$(pwd); OUT=$REPO/gpurun_out; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_${TAG}_${WL}" -o run -- \
    python3 "$REPO/tools/prof_step.py" "$WL" 2 > "$OUT/prof_${TAG}_${WL}.log" 2>&1
python3 "$REPO/tools/kstats.py" "$OUT/prof_${TAG}_${WL}/run_kernel_stats.csv" 3 22
grep "^step 2" "$OUT/prof_${TAG}_${WL}.log" | cut -c1-400
