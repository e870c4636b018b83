#!/bin/bash
set -eo pipefail
timeout -k 10 900 python -u -m pytest tests/test_sharded_sss.py -m gpu -x -q -s --timeout 600 --timeout-method thread -k "ring or speculative or tail_repeat or ranks_on_gpu" > gpurun_out/pytest_r04p.log 2>&1 || { tail -30 gpurun_out/pytest_r04p.log; exit 1; }
tail -2 gpurun_out/pytest_r04p.log
timeout -k 10 900 python -u -m pytest tests/test_sharded_sss.py -m gpu -x -q -s --timeout 900 --timeout-method thread -k "past_4gib_hash and ring" > gpurun_out/pytest_r04p_4g.log 2>&1 || { tail -30 gpurun_out/pytest_r04p_4g.log; exit 1; }
grep -a "speculation\|passed\|failed" gpurun_out/pytest_r04p_4g.log | cut -c1-600
