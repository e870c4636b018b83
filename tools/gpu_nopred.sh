# greedy phase with and without pred5 (LZ77SSS_NO_PRED) on rr and genome
mkdir -p gpurun_out
for wl in rr genome; do
  timeout -k 10 200 python3 tools/prof_step.py $wl 2 > gpurun_out/np_${wl}_pred.log 2>&1 || exit 1
  LZ77SSS_NO_PRED=1 timeout -k 10 200 python3 tools/prof_step.py $wl 2 > gpurun_out/np_${wl}_nopred.log 2>&1 || exit 1
done
grep -h "^step 2" gpurun_out/np_*.log | cut -c1-140
