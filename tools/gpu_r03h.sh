#!/bin/bash
# Round-3 final profiles (kernel trace + SSS PMC, rr and genome), then configs[3] at 50 GiB
# (sharded path at world 1, compared with the one-GPU stream of a fresh session).
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_profile_round.sh r03h rr || exit 1
bash tools/gpu_profile_round.sh r03h genome || exit 1
timeout -k 10 900 python -u bench.py --shard --workload chr19 --size-gib ${1:-50} --steps 1 --warmup 0 \
    > gpurun_out/bench_r03h_c4.json 2> gpurun_out/bench_r03h_c4.err; rc=$?
grep -v amdgpu.ids gpurun_out/bench_r03h_c4.err | tail -5
cat gpurun_out/bench_r03h_c4.json
exit $rc
