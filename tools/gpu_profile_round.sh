#!/bin/bash
# Round profile (run from the repo root via gpurun):
#   1. rocprofv3 kernel trace + stats of factorization steps (tools/prof_step.py, no decode)
#   2. PMC passes FETCH_SIZE, WRITE_SIZE over the SSS-phase kernels (separate runs)
# tools/summarize_profile2.py turns gpurun_out/ into profiles/<tag>_<wl>_*.
set -eo pipefail
TAG=${1:-r03}
WL=${2:-rr}
REPO=$(pwd)
OUT=$REPO/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
KR='k_sss_stream|k_sss_runs|k_sss_marks|k_flag_count|k_flag_list|k_q_anchors|k_run_keys|k_run_apply|k_blk_seg_tiles|k_blk_seg_info|k_blk_marks|k_blk_runinfo|k_sss_compact|k_count_scan'
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_${TAG}_${WL}" -o run -- \
    python3 "$REPO/tools/prof_step.py" "$WL" 3 > "$OUT/prof_${TAG}_${WL}.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KR" -f csv -d "$OUT/pmc_${TAG}_${WL}_fetch" -o run -- \
    python3 "$REPO/tools/prof_step.py" "$WL" 2 > "$OUT/pmc_${TAG}_${WL}_fetch.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KR" -f csv -d "$OUT/pmc_${TAG}_${WL}_write" -o run -- \
    python3 "$REPO/tools/prof_step.py" "$WL" 2 > "$OUT/pmc_${TAG}_${WL}_write.log" 2>&1
echo "profile $TAG $WL done"
