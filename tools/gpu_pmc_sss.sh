#!/bin/bash
# HBM traffic of the SSS phase kernels (from the repo root via gpurun): tools/gpu_pmc_sss.sh <tag> <rr|genome>
# two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE: they do not fit in one) over tools/prof_step.py
# (2 factorizations), summarized by tools/pmc_sss.py into gpurun_out/<tag>_<wl>_pmc_sss.json
set -eo pipefail
TAG=$1; WL=$2
REPO=$(pwd); OUT=$REPO/gpurun_out; mkdir -p "$OUT"
KR='k_sss_stream|k_sss_runs|k_blk_seg|k_sss_compact|k_q_anchors|k_sss_fallback|k_sss_marks'
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KR" -f csv -d "$OUT/pmcf_${TAG}_${WL}" -o run -- \
    python3 "$REPO/tools/prof_step.py" "$WL" 1 > "$OUT/pmcf_${TAG}_${WL}.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KR" -f csv -d "$OUT/pmcw_${TAG}_${WL}" -o run -- \
    python3 "$REPO/tools/prof_step.py" "$WL" 1 > "$OUT/pmcw_${TAG}_${WL}.log" 2>&1
python3 "$REPO/tools/pmc_sss.py" "$WL" "$OUT/pmcf_${TAG}_${WL}/run_counter_collection.csv" \
    "$OUT/pmcw_${TAG}_${WL}/run_counter_collection.csv" > "$OUT/${TAG}_${WL}_pmc_sss.json"
cat "$OUT/${TAG}_${WL}_pmc_sss.json"
