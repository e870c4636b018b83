#!/bin/bash
# Round profile on one MI355X (run from the repo root via gpurun):
#   1. rocprofv3 kernel trace + stats of a short bench run (per-kernel durations)
#   2. two PMC passes (FETCH_SIZE, WRITE_SIZE) restricted to the SSS kernel
# Outputs land in gpurun_out/prof_<tag>*/; tools/summarize_profile.py turns them into profiles/.
set -eo pipefail
TAG=${1:-r01}
WL=${2:-rr}
REPO=$(pwd)
OUT=$REPO/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_${TAG}_${WL}" -o run -- \
    python3 "$REPO/bench.py" --steps 3 --warmup 1 --workload "$WL" --no-cpu-baseline > "$OUT/prof_${TAG}_${WL}.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_sss_stream -f csv -d "$OUT/pmc_${TAG}_${WL}_fetch" -o run -- \
    python3 "$REPO/bench.py" --steps 2 --warmup 0 --workload "$WL" --no-cpu-baseline > "$OUT/pmc_${TAG}_${WL}_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_sss_stream -f csv -d "$OUT/pmc_${TAG}_${WL}_write" -o run -- \
    python3 "$REPO/bench.py" --steps 2 --warmup 0 --workload "$WL" --no-cpu-baseline > "$OUT/pmc_${TAG}_${WL}_write.log" 2>&1
