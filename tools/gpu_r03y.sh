#!/bin/bash
# k_sss_runs period search from the LDS ring: SSS/parity tests, then SSS timing and rr debug counters.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_sss_adversarial.py tests/test_gpu_parity.py tests/test_stream_hashes.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r03y.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_r03y.log
[ $rc -eq 0 ] || exit $rc
for wl in rr genome; do
  timeout -k 10 120 python -u tools/sss_time.py $wl 10 >> gpurun_out/sss_r03y.log 2>&1 || exit 1
done
timeout -k 10 200 python -u tools/phase_time.py rr 5 >> gpurun_out/sss_r03y.log 2>&1 || exit 1
cat gpurun_out/sss_r03y.log
