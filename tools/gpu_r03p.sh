#!/bin/bash
# k_sss_runs with the LDS-DMA ring: SSS parity tests, then A/B against the register ring.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_sss_adversarial.py tests/test_gpu_parity.py -m gpu -x -q -k "sss or sync or run or lce" --timeout 200 --timeout-method thread > gpurun_out/pytest_r03p.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_r03p.log
[ $rc -eq 0 ] || exit $rc
for wl in rr genome; do
  timeout -k 10 120 python -u tools/sss_time.py $wl 10 >> gpurun_out/sss_r03p.log 2>&1 || exit 1
  LZ77SSS_SSS_REGRING=1 timeout -k 10 120 python -u tools/sss_time.py $wl 10 >> gpurun_out/sss_r03p.log 2>&1 || exit 1
  timeout -k 10 120 python -u tools/sss_time.py $wl 10 >> gpurun_out/sss_r03p.log 2>&1 || exit 1
done
cat gpurun_out/sss_r03p.log
