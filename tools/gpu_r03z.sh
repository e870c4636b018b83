#!/bin/bash
# Rebuilt library after the A/B revert: parity + smoke.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_smoke.py tests/test_sss_adversarial.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r03z.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_r03z.log
exit $rc
