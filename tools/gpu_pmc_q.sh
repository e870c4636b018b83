# SQ counters of one kernel over tools/prof_step.py: tools/gpu_pmc_q.sh <tag> <wl> <kernel-regex>
set -eo pipefail
TAG=$1; WL=$2; KR=$3
REPO=$(pwd); OUT=$REPO/gpurun_out; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex "$KR" -f csv -d "$OUT/pmc_${TAG}_${WL}_a" -o run -- python3 "$REPO/tools/prof_step.py" "$WL" 1 > "$OUT/pmc_${TAG}_${WL}_a.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH --kernel-include-regex "$KR" -f csv -d "$OUT/pmc_${TAG}_${WL}_b" -o run -- python3 "$REPO/tools/prof_step.py" "$WL" 1 > "$OUT/pmc_${TAG}_${WL}_b.log" 2>&1
echo pmc done
