#!/bin/bash
# Speculative blocks: the lead=1 rejection check and the 4 GiB acceptance report (printed).
set -o pipefail
mkdir -p gpurun_out
LZ77SSS_SPEC_DEBUG=1 timeout -k 10 900 python -u -m pytest tests/test_sharded_sss.py -m gpu -x -v -s --timeout 600 --timeout-method thread -k "past_4gib" > gpurun_out/pytest_r03k.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed|accepted=|speculative block at" gpurun_out/pytest_r03k.log | tail -20
exit $rc
