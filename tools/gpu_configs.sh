#!/bin/bash
# configs[3] / configs[4] bench lines (from the repo root via gpurun): tools/gpu_configs.sh <tag> [c4-size-gib]
# exact-smpl on rr + genome (1 GiB), then the chr19-style 3-aprx on one GPU (pos_t = uint64_t).
set -eo pipefail
TAG=${1:-r03}
GIB=${2:-50}
mkdir -p gpurun_out
for WL in rr genome; do
  timeout -k 10 300 python -u bench.py --mode exact --workload $WL --steps 2 --warmup 1 \
      > gpurun_out/bench_${TAG}_${WL}_exact.json 2> gpurun_out/bench_${TAG}_${WL}_exact.err
  cat gpurun_out/bench_${TAG}_${WL}_exact.json
done
timeout -k 10 900 python -u bench.py --shard --workload chr19 --size-gib $GIB --steps 1 --warmup 0 \
    > gpurun_out/bench_${TAG}_c4_${GIB}.json 2> gpurun_out/bench_${TAG}_c4_${GIB}.err
cat gpurun_out/bench_${TAG}_c4_${GIB}.json
