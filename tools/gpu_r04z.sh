#!/bin/bash
# Round-4 measurement: rr headline (CPU leg included) + genome + LPF/LNF bench lines, kernel traces and
# SSS PMC for rr and genome (tools/gpu_round.sh), every step with its own time limit.
set -eo pipefail
bash tools/gpu_round.sh r04z rr genome
timeout -k 10 400 python -u bench.py --phr-mode lpf_lnf_opt --steps 10 --warmup 2 > gpurun_out/bench_r04z_rr_lnf.json 2> gpurun_out/bench_r04z_rr_lnf.err
tail -1 gpurun_out/bench_r04z_rr_lnf.json | cut -c1-400
echo "r04z done"
