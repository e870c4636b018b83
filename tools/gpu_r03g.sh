#!/bin/bash
# Full GPU suite, then the rr and genome bench lines with their CPU baselines (full 1 GiB texts).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r03g.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_r03g.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench_r03g_rr.json 2> gpurun_out/bench_r03g_rr.err || exit 1
cat gpurun_out/bench_r03g_rr.json
timeout -k 10 600 python -u bench.py --workload genome --steps 5 --warmup 1 > gpurun_out/bench_r03g_genome.json 2> gpurun_out/bench_r03g_genome.err || exit 1
cat gpurun_out/bench_r03g_genome.json
