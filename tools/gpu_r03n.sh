#!/bin/bash
# Validation of the latest changes: full GPU suite, exact-smpl scaling, rr + genome + exact bench lines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r03n.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_r03n.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/exact_scale.py genome 16,64,256 > gpurun_out/exact_scale_r03n.log 2>&1 || exit 1
cat gpurun_out/exact_scale_r03n.log
timeout -k 10 300 python -u bench.py --mode exact --workload genome --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_r03n_genome_exact.json 2> gpurun_out/bench_r03n_genome_exact.err || exit 1
cat gpurun_out/bench_r03n_genome_exact.json
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench_r03n_rr.json 2> gpurun_out/bench_r03n_rr.err || exit 1
cat gpurun_out/bench_r03n_rr.json
timeout -k 10 300 python -u bench.py --workload genome --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_r03n_genome.json 2> gpurun_out/bench_r03n_genome.err || exit 1
cat gpurun_out/bench_r03n_genome.json
