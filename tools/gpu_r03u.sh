#!/bin/bash
# Final-tree check: full GPU suite, smoke(), one short bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r03u.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_r03u.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r03u.log 2>&1 || exit 1
tail -2 gpurun_out/smoke_r03u.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_r03u_rr.json 2> gpurun_out/bench_r03u_rr.err || exit 1
cat gpurun_out/bench_r03u_rr.json
