#!/bin/bash
# exact-smpl checks (from the repo root via gpurun): GPU exact tests, then sizes x grid-cell variants.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_exact.py tests/test_gpu_u64.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r03d.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_r03d.log
[ $rc -eq 0 ] || exit $rc
for v in product; do
  for wl in genome rr; do
    if [ "$v" = product ]; then L=""; else L="LZ77SSS_LIB=$v"; fi
    env $L timeout -k 10 200 python -u tools/exact_scale.py $wl 16,64,256 >> gpurun_out/exact_scale_r03d.log 2>&1; rc=$?
    echo "[$v $wl rc=$rc]" >> gpurun_out/exact_scale_r03d.log
    [ $rc -eq 0 ] || { cat gpurun_out/exact_scale_r03d.log; exit $rc; }
  done
done
cat gpurun_out/exact_scale_r03d.log
