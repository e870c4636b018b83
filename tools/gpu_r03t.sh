#!/bin/bash
# plain factorize after the sharded path on one session (the r03e 50 GiB open item), small sizes.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_sharded_sss.py -m gpu -x -v -k plain_factorize_after --timeout 200 --timeout-method thread > gpurun_out/pytest_r03t.log 2>&1; rc=$?
grep -E "PASSED|FAILED|Error|error" gpurun_out/pytest_r03t.log | tail -20
exit $rc
