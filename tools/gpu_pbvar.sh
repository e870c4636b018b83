# genome phase timings: product (PB_SH 18) and PB_SH variants
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/phase_stats.py genome 4 || exit 1
for v in lz77-sss_amd/lib/variants/*.so; do LZ77SSS_LIB=$PWD/$v timeout -k 10 200 python3 tools/phase_stats.py genome 4 || exit 1; done
