# genome step times: product build and lib/variants builds
mkdir -p gpurun_out
for v in product lz77-sss_amd/lib/variants/*.so; do
  for wl in genome; do
    if [ "$v" = product ]; then timeout -k 10 100 python3 -u tools/prof_step.py $wl 2 > gpurun_out/qv.log 2>&1 || { tail -3 gpurun_out/qv.log; exit 1; }
    else LZ77SSS_LIB=$PWD/$v timeout -k 10 100 python3 -u tools/prof_step.py $wl 2 > gpurun_out/qv.log 2>&1 || { tail -3 gpurun_out/qv.log; exit 1; }; fi
    echo "$(basename $v) $wl $(grep '^step 2' gpurun_out/qv.log | cut -c1-120)"
  done
done
