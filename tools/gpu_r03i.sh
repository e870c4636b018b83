#!/bin/bash
# SSS change check: full GPU suite, then SSS kernel times (rr, genome) and the rr bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r03i.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_r03i.log
[ $rc -eq 0 ] || exit $rc
for wl in rr genome; do timeout -k 10 120 python -u tools/sss_time.py $wl 8 >> gpurun_out/sss_r03i.log 2>&1 || exit 1; done
cat gpurun_out/sss_r03i.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_r03i_rr.json 2> gpurun_out/bench_r03i_rr.err || exit 1
cat gpurun_out/bench_r03i_rr.json
