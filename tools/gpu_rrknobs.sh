# rr step time under the greedy tuning knobs (timing experiments)
mkdir -p gpurun_out
run() { echo "== $1"; env $1 timeout -k 10 200 python3 tools/prof_step.py rr 3 > gpurun_out/knob.log 2>&1 || { tail -5 gpurun_out/knob.log; exit 1; }; grep "^step [23]" gpurun_out/knob.log | cut -c1-150; }
run X=0 && run LZ77SSS_PRED_SORTED_MIN=0 && run LZ77SSS_NO_DENSE=1 && run LZ77SSS_NO_PRED=1 && run "LZ77SSS_NO_DENSE=1 LZ77SSS_PRED_SORTED_MIN=0"
