#!/bin/bash
# smoke() through pytest (tests/test_smoke.py).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_smoke.py -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/pytest_r03w.log 2>&1; rc=$?
grep -E "PASSED|FAILED|Error" gpurun_out/pytest_r03w.log | tail -5
exit $rc
