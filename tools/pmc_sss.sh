#!/bin/bash
# Instruction-mix counters for the SSS kernels (two PMC passes, kernel trace only).
set -eo pipefail
WL=${1:-rr}
REPO=$(pwd)
OUT=$REPO/gpurun_out/pmcx_$WL
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    --kernel-include-regex "k_sss_stream|k_q_anchors" -f csv -d "$OUT/p1" -o run -- python3 "$REPO/tools/sss_probe.py" "$WL" 2 > "$OUT/p1.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    --kernel-include-regex "k_sss_stream|k_q_anchors" -f csv -d "$OUT/p2" -o run -- python3 "$REPO/tools/sss_probe.py" "$WL" 2 > "$OUT/p2.log" 2>&1
