#!/bin/bash
set -eo pipefail
LZ77SSS_SPEC_DEBUG=1 timeout -k 10 900 python -u -m pytest tests/test_sharded_sss.py -m gpu -x -q -s --timeout 900 --timeout-method thread -k "past_4gib_hash and ring" > gpurun_out/pytest_r04q_4g.log 2>&1 || { tail -30 gpurun_out/pytest_r04q_4g.log; exit 1; }
grep -a "speculat\|slot\|passed\|failed" gpurun_out/pytest_r04q_4g.log | cut -c1-300
