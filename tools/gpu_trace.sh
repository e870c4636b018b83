# kernel trace of factorization steps: tools/gpu_trace.sh <tag> <wl> [steps]
set -eo pipefail
TAG=$1; WL=$2; ST=${3:-3}
REPO=$(pwd); OUT=$REPO/gpurun_out; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace_${TAG}_${WL}" -o run -- \
    python3 "$REPO/tools/prof_step.py" "$WL" "$ST" > "$OUT/trace_${TAG}_${WL}.log" 2>&1
tail -2 "$OUT/trace_${TAG}_${WL}.log"
