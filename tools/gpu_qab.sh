#!/bin/bash
# A/B of SSS-phase variants on rr (kernel traces of the last step's SSS phase).  The knobs
# (LZ77SSS_QT_GRID, LZ77SSS_SSS_NOSKIPLOAD) belonged to the reverted round-2c experiment.
set -eo pipefail
REPO=$(pwd); OUT=$REPO/gpurun_out; mkdir -p "$OUT"
WL=${1:-rr}
cd /tmp && export TMPDIR=/tmp
run() {
  timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d "$OUT/qab_$1_$WL" -o run -- python3 "$REPO/tools/prof_step.py" "$WL" 2 > "$OUT/qab_$1_$WL.log" 2>&1
  echo "== $1"; python3 "$REPO/tools/trace_sss.py" "$(find "$OUT/qab_$1_$WL" -name '*kernel_trace.csv' | head -1)" 22
}
run base
LZ77SSS_QT_GRID=0 run g0
LZ77SSS_QT_GRID=2048 run g2k
LZ77SSS_SSS_NOSKIPLOAD=1 run nsl
