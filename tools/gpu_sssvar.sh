# SSS phase timing of the product build and the timing variants (lib/variants)
mkdir -p gpurun_out
for wl in genome rr; do
  timeout -k 10 200 python3 tools/sss_time.py $wl || exit 1
  for v in lz77-sss_amd/lib/variants/liblz_sss*.so; do
    LZ77SSS_LIB=$PWD/$v timeout -k 10 200 python3 tools/sss_time.py $wl || exit 1
  done
done
