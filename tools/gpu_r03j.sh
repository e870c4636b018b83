#!/bin/bash
# Speculative sharded chain blocks: the resident sharded GPU tests (2-3 gloo ranks sharing the GPU).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_sharded_sss.py -m gpu -x -v --timeout 600 --timeout-method thread -k "resident" > gpurun_out/pytest_r03j.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_r03j.log | tail -20
exit $rc
