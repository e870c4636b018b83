#!/bin/bash
# exact-smpl check (from the repo root via gpurun): the exact tests, then configs[4] bench lines (rr, genome)
set -eo pipefail
TAG=${1:-r04}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -k "exact or smoke" > gpurun_out/pytest_${TAG}_exact.log 2>&1 || { tail -20 gpurun_out/pytest_${TAG}_exact.log; exit 1; }
tail -2 gpurun_out/pytest_${TAG}_exact.log
for WL in rr genome; do
  timeout -k 10 300 python -u bench.py --mode exact --workload $WL --steps 2 --warmup 1 > gpurun_out/bench_${TAG}_${WL}_exact.json 2> gpurun_out/bench_${TAG}_${WL}_exact.err
  tail -1 gpurun_out/bench_${TAG}_${WL}_exact.json | cut -c1-300
done
