#!/bin/bash
# Speculative blocks in parts: the sharded GPU tests, then the 4 GiB two-rank run with the
# per-part acceptance printed.
set -o pipefail
mkdir -p gpurun_out
export LZ77SSS_SPEC_DEBUG=1
timeout -k 10 900 python -u -m pytest tests/test_sharded_sss.py -m gpu -x -v -s --timeout 600 --timeout-method thread > gpurun_out/pytest_r03o.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|speculative|rank [01]:" gpurun_out/pytest_r03o.log | tail -40
exit $rc
