#!/bin/bash
# Round-5 GPU check (from the repo root via gpurun): tools/gpu_r05.sh <tag> "<pytest -k expr or ->" [workloads...]
#   1. a -m gpu pytest subset ("-": none)
#   2. per workload (rr, genome): kernel trace of 3 factorization steps (tools/prof_step.py), the SSS
#      phase of the last step (tools/trace_sss.py) and the top kernels (tools/kstats.py)
set -eo pipefail
TAG=$1; K=$2; shift 2 || true
REPO=$(pwd); OUT=$REPO/gpurun_out; mkdir -p "$OUT"
if [ "$K" != "-" ]; then
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread -k "$K" \
        > "$OUT/pytest_${TAG}.log" 2>&1 || { tail -40 "$OUT/pytest_${TAG}.log"; exit 1; }
    tail -3 "$OUT/pytest_${TAG}.log"
fi
cd /tmp && export TMPDIR=/tmp
for WL in "$@"; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_${TAG}_${WL}" -o run -- \
        python3 "$REPO/tools/prof_step.py" "$WL" 3 > "$OUT/prof_${TAG}_${WL}.log" 2>&1
    grep "^step" "$OUT/prof_${TAG}_${WL}.log" | cut -c1-300
    python3 "$REPO/tools/trace_sss.py" "$OUT/prof_${TAG}_${WL}/run_kernel_trace.csv" 26 > "$OUT/sss_${TAG}_${WL}.txt"
    cat "$OUT/sss_${TAG}_${WL}.txt"
    python3 "$REPO/tools/kstats.py" "$OUT/prof_${TAG}_${WL}/run_kernel_stats.csv" 4 16
done
echo "r05 $TAG done"
