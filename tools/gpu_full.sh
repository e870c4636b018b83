#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q -rs --timeout 600 --timeout-method thread > gpurun_out/pytest_gpu_r04full.log 2>&1
rc=$?
tail -6 gpurun_out/pytest_gpu_r04full.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r04full.log 2>&1
rc=$?
tail -3 gpurun_out/smoke_r04full.log
exit $rc
