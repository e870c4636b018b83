#!/bin/bash
# Round 3b (from the repo root via gpurun): GPU tests with the run-record cross-check, SSS A/B of
# lib_var builds, SQ counters of k_sss_runs on rr, exact-smpl scaling.  First failure ends it.
set -o pipefail
mkdir -p gpurun_out
LZ77SSS_BLK_CHECK=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r03b.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_r03b.log
[ $rc -eq 0 ] || exit $rc
for wl in rr genome; do
  for v in product lz77-sss_amd/lib_var/*.so; do
    if [ "$v" = product ]; then timeout -k 10 120 python -u tools/sss_time.py $wl 8 >> gpurun_out/sss_ab.log 2>&1 || exit 1
    else LZ77SSS_LIB=$v timeout -k 10 120 python -u tools/sss_time.py $wl 8 >> gpurun_out/sss_ab.log 2>&1 || exit 1; fi
  done
done
cat gpurun_out/sss_ab.log
bash tools/gpu_pmc_q.sh r03b rr k_sss_runs || exit 1
timeout -k 10 240 python -u tools/exact_scale.py rr 16,64,256 > gpurun_out/exact_scale_rr.log 2>&1; rc=$?
cat gpurun_out/exact_scale_rr.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u tools/exact_scale.py genome 16,64,256 > gpurun_out/exact_scale_genome.log 2>&1; rc=$?
cat gpurun_out/exact_scale_genome.log
exit $rc
