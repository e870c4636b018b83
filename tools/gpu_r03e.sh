#!/bin/bash
# Round 3e (from the repo root via gpurun): full GPU suite, exact bench lines (rr, genome),
# configs[3] 3-aprx of a 50 GiB chr19-style text on one GPU.  First failure ends it.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r03e.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_r03e.log
[ $rc -eq 0 ] || exit $rc
for WL in rr genome; do
  timeout -k 10 300 python -u bench.py --mode exact --workload $WL --steps 2 --warmup 1 \
      > gpurun_out/bench_r03e_${WL}_exact.json 2> gpurun_out/bench_r03e_${WL}_exact.err || exit 1
  cat gpurun_out/bench_r03e_${WL}_exact.json
done
timeout -k 10 900 python -u bench.py --shard --workload chr19 --size-gib ${1:-50} --steps 1 --warmup 0 \
    > gpurun_out/bench_r03e_c4.json 2> gpurun_out/bench_r03e_c4.err; rc=$?
tail -5 gpurun_out/bench_r03e_c4.err
cat gpurun_out/bench_r03e_c4.json
exit $rc
