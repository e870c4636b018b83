#!/bin/bash
# Round-3 closing evidence for the final code: full GPU suite, bench lines (rr with its CPU
# baseline, genome), kernel trace + SSS PMC (rr, genome).  First failure ends it.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r03s.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_r03s.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench_r03s_rr.json 2> gpurun_out/bench_r03s_rr.err || exit 1
cat gpurun_out/bench_r03s_rr.json
timeout -k 10 300 python -u bench.py --workload genome --steps 5 --warmup 1 > gpurun_out/bench_r03s_genome.json 2> gpurun_out/bench_r03s_genome.err || exit 1
cat gpurun_out/bench_r03s_genome.json
bash tools/gpu_profile_round.sh r03s rr || exit 1
bash tools/gpu_profile_round.sh r03s genome || exit 1
echo done
