#!/bin/bash
# kernel traces of the configs[4] exact-smpl (with_samples) bench lines (from the repo root via gpurun);
# keeps only the kernel stats summaries (the full traces exceed what gpurun copies back)
set -eo pipefail
TAG=${1:-r04}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for WL in rr genome; do
  D=gpurun_out/prof_${TAG}_${WL}_exact
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_${WL} -o run -- python3 -u bench.py --mode exact --workload $WL --steps 1 --warmup 1 > gpurun_out/prof_${TAG}_${WL}_exact.log 2>&1
  mkdir -p $D && find /tmp/prof_${WL} -name '*kernel_stats.csv' -exec cp {} $D/ \;
  echo "$WL done"
done
