#!/bin/bash
# Counters of the kernels matching a regex over tools/prof_step.py (one factorization):
# tools/gpu_pmc_k.sh <tag> <rr|genome> <kernel-regex>.  Three passes (SQ, FETCH_SIZE, WRITE_SIZE).
set -eo pipefail
TAG=$1; WL=$2; KR=$3
REPO=$(pwd); OUT=$REPO/gpurun_out; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES --kernel-include-regex "$KR" -f csv -d "$OUT/pmc_${TAG}_${WL}_sq" -o run -- python3 "$REPO/tools/prof_step.py" "$WL" 1 > "$OUT/pmc_${TAG}_${WL}_sq.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KR" -f csv -d "$OUT/pmc_${TAG}_${WL}_fs" -o run -- python3 "$REPO/tools/prof_step.py" "$WL" 1 > "$OUT/pmc_${TAG}_${WL}_fs.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KR" -f csv -d "$OUT/pmc_${TAG}_${WL}_ws" -o run -- python3 "$REPO/tools/prof_step.py" "$WL" 1 > "$OUT/pmc_${TAG}_${WL}_ws.log" 2>&1
echo "pmc $TAG $WL done"
