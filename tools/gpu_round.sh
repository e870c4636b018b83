#!/bin/bash
# Round measurement (from the repo root via gpurun): tools/gpu_round.sh <tag> [workloads...]
#   bench lines (rr headline + listed extra modes), then kernel trace + SSS-phase PMC per workload.
# Every GPU step has its own time limit; the first failure ends the script.
set -eo pipefail
TAG=${1:-r03}
shift || true
WLS=${*:-rr genome}
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench_${TAG}_rr.json 2> gpurun_out/bench_${TAG}_rr.err
cat gpurun_out/bench_${TAG}_rr.json
for WL in $WLS; do
  if [ "$WL" != rr ]; then
    timeout -k 10 400 python -u bench.py --workload "$WL" --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_${TAG}_${WL}.json 2> gpurun_out/bench_${TAG}_${WL}.err
    cat gpurun_out/bench_${TAG}_${WL}.json
  fi
  bash tools/gpu_profile_round.sh "$TAG" "$WL"
done
echo "round measurement $TAG done"
