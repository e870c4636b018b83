#!/bin/bash
# greedy phase breakdown on rr (debug laps), after the segmerge cap change: SA_S parity tests.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r03r.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_r03r.log
[ $rc -eq 0 ] || exit $rc
LZ77SSS_DEBUG=1 timeout -k 10 150 python -u tools/phase_time.py rr 1 > gpurun_out/debug_rr_r03r.log 2>&1 || exit 1
grep -v "^\[sa_s\]" gpurun_out/debug_rr_r03r.log | tail -80
