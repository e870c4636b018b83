#!/bin/bash
# k_q_anchors workgroup size (LZ_QT_THREADS build variants in lz77-sss_amd/lib/variants): SSS parity
# tests, then the SSS phase of the last rr step per variant (kernel traces)
set -eo pipefail
REPO=$(pwd); OUT=$REPO/gpurun_out; mkdir -p "$OUT"
for v in q64 q128; do
  LZ77SSS_LIB=$REPO/lz77-sss_amd/lib/variants/liblz77sss_$v.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "sss or adversarial or fallback or golden or run" > "$OUT/qvar2_$v.log" 2>&1 || { echo "$v FAIL"; tail -30 "$OUT/qvar2_$v.log"; exit 1; }
  echo "$v: $(tail -1 "$OUT/qvar2_$v.log")"
done
cd /tmp && export TMPDIR=/tmp
for v in base q64 q128; do
  if [ $v = base ]; then unset LZ77SSS_LIB; else export LZ77SSS_LIB=$REPO/lz77-sss_amd/lib/variants/liblz77sss_$v.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d "$OUT/qv2_$v" -o run -- python3 "$REPO/tools/prof_step.py" rr 2 > "$OUT/qv2_$v.log" 2>&1
  echo "== $v"; python3 "$REPO/tools/trace_sss.py" "$(find "$OUT/qv2_$v" -name '*kernel_trace.csv' | head -1)" 22 | grep -E "q_anchors|k_sss_stream|k_run"
done
