# k_walk occupancy variants (lib/variants) + the default library: genome and rr step times
mkdir -p gpurun_out
for v in default w6 w7 w8; do
  if [ $v = default ]; then L=lz77-sss_amd/lib/liblz77sss_hip.so; else L=lz77-sss_amd/lib/variants/liblz77sss_$v.so; fi
  LZ77SSS_LIB=$PWD/$L timeout -k 10 200 python3 tools/prof_step.py genome 2 > gpurun_out/wv_$v.log 2>&1 || exit 1
  echo "$v $(grep '^step 2' gpurun_out/wv_$v.log | cut -c1-130)"
done
timeout -k 10 200 python3 tools/prof_step.py rr 3 > gpurun_out/wv_rr.log 2>&1 || exit 1
grep '^step' gpurun_out/wv_rr.log | cut -c1-130
