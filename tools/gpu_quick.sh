#!/bin/bash
# Quick GPU check (from the repo root via gpurun): tools/gpu_quick.sh <tag> <pytest -k expr> [bench args...]
# pytest subset, then one rr bench line (no CPU leg) + a kernel trace of 3 factorize calls.
set -eo pipefail
TAG=$1; K=$2; shift 2 || true
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread -k "$K" > gpurun_out/pytest_${TAG}.log 2>&1 || { tail -30 gpurun_out/pytest_${TAG}.log; exit 1; }
tail -3 gpurun_out/pytest_${TAG}.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err
cat gpurun_out/bench_${TAG}.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}" -o run -- \
    python3 "$GRAFT_REPO_ROOT/tools/prof_step.py" rr 3 > "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}.log" 2>&1
echo "quick $TAG done"
