#!/bin/bash
# GPU test run on one MI355X (from the repo root via gpurun): tools/gpu_tests.sh [pytest -k expression]
# Output: gpurun_out/pytest_gpu.log (tail printed).  Every step has its own time limit.
set -o pipefail
mkdir -p gpurun_out
K=${1:-}
if [ -n "$K" ]; then
  timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread -k "$K" > gpurun_out/pytest_gpu.log 2>&1
else
  timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
fi
rc=$?
tail -15 gpurun_out/pytest_gpu.log
exit $rc
