#!/bin/bash
# Kernel trace of exact-smpl on the genome-like text (256 MiB) for the round-4 plan.
set -o pipefail
REPO=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$REPO/gpurun_out/prof_r03x_exact_genome" -o run -- \
    python3 "$REPO/tools/exact_scale.py" genome 256 > "$REPO/gpurun_out/prof_r03x_exact_genome.log" 2>&1; rc=$?
tail -3 "$REPO/gpurun_out/prof_r03x_exact_genome.log"
exit $rc
