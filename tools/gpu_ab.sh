#!/bin/bash
# A/B of library builds (run from the repo root via gpurun):
#   tools/gpu_ab.sh <tag> "<workloads>" <lib.so>...
# per library and workload: kernel trace of 3 factorization steps (tools/prof_step.py), the SSS
# phase of the last step (tools/trace_sss.py) and the top kernels (tools/kstats.py)
set -eo pipefail
TAG=$1; WLS=$2; shift 2
REPO=$(pwd); OUT=$REPO/gpurun_out; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for LIB in "$@"; do
    V=$(basename "$LIB" .so)
    for WL in $WLS; do
        D="$OUT/ab_${TAG}_${V}_${WL}"
        LZ77SSS_LIB="$REPO/$LIB" timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d "$D" -o run -- \
            python3 "$REPO/tools/prof_step.py" "$WL" 3 > "$D.log" 2>&1
        echo "== $V $WL"
        grep "^step 3" "$D.log" | cut -c1-200
        python3 "$REPO/tools/trace_sss.py" "$D/run_kernel_trace.csv" > "$D.sss.txt"
        cat "$D.sss.txt"
        python3 "$REPO/tools/kstats.py" "$D/run_kernel_stats.csv" 4 12 > "$D.top.txt" || true
    done
done
echo "ab $TAG done"
