#!/bin/bash
# Round measurement (from the repo root via gpurun): tools/gpu_measure.sh <tag>
#   rr headline (CPU leg included) + genome + LPF/LNF bench lines, kernel traces and SSS PMC for rr
#   and genome (tools/gpu_round.sh); then tools/summarize_profile2.py <tag> rr|genome on the CPU side.
set -eo pipefail
TAG=${1:-r04}
bash tools/gpu_round.sh "$TAG" rr genome
timeout -k 10 400 python -u bench.py --phr-mode lpf_lnf_opt --steps 10 --warmup 2 > gpurun_out/bench_${TAG}_rr_lnf.json 2> gpurun_out/bench_${TAG}_rr_lnf.err
tail -1 gpurun_out/bench_${TAG}_rr_lnf.json | cut -c1-400
echo "$TAG done"
