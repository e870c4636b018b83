#!/bin/bash
# smoke() after the exact-check fix, then one short bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r03v.log 2>&1; rc=$?
tail -3 gpurun_out/smoke_r03v.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_r03v_rr.json 2> gpurun_out/bench_r03v_rr.err || exit 1
cat gpurun_out/bench_r03v_rr.json
