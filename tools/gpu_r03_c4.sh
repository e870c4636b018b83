#!/bin/bash
# C4 checks (from the repo root via gpurun): tools/gpu_r03_c4.sh <size-gib>
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_sharded_sss.py -m gpu -x -q -rs --timeout 800 --timeout-method thread -k resident > gpurun_out/pytest_c4.log 2>&1 || { tail -30 gpurun_out/pytest_c4.log; exit 1; }
tail -3 gpurun_out/pytest_c4.log
timeout -k 10 900 python -u bench.py --shard --workload chr19 --size-gib ${1:-8} --steps 1 --warmup 1 > gpurun_out/bench_c4_${1:-8}.json 2> gpurun_out/bench_c4_${1:-8}.err || { tail -20 gpurun_out/bench_c4_${1:-8}.err; exit 1; }
cat gpurun_out/bench_c4_${1:-8}.json
