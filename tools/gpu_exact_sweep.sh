#!/bin/bash
# exact-smpl genome: the own-lane intersect threshold (LZ77SSS_SMPL_SMALL) swept (from the repo root via gpurun)
set -eo pipefail
TAG=${1:-r04}
for S in 32 256 1024; do
  LZ77SSS_SMPL_SMALL=$S timeout -k 10 200 python -u bench.py --mode exact --workload genome --steps 1 --warmup 1 > gpurun_out/sweep_${TAG}_${S}.json 2> gpurun_out/sweep_${TAG}_${S}.err
  echo "small=$S $(tail -1 gpurun_out/sweep_${TAG}_${S}.json | cut -c1-240)"
done
