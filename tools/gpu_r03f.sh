#!/bin/bash
# k_slots / k_walk counters on rr + genome, then the configs[3] one-GPU factorize diagnostic.
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_pmc_k.sh r03f rr 'k_slots|k_dense_keys|k_walk' || exit 1
bash tools/gpu_pmc_k.sh r03f genome 'k_slots|k_pb_move|k_pb_apply' || exit 1
LZ77SSS_DEBUG=1 timeout -k 10 600 python -u tools/c4_plain.py ${1:-50} > gpurun_out/c4_plain.log 2>&1; rc=$?
grep -v "amdgpu.ids" gpurun_out/c4_plain.log | tail -25
exit $rc
