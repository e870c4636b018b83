# A/B: the no-stash variant vs the current library on the C1 seeds
mkdir -p gpurun_out
LZ77SSS_LIB=$PWD/lz77-sss_amd/lib/variants/liblz77sss_ns.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "c1_seeds" --timeout 120 --timeout-method thread > gpurun_out/ab_ns.log 2>&1; echo "nostash rc=$?"; tail -1 gpurun_out/ab_ns.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "c1_seeds" --timeout 120 --timeout-method thread > gpurun_out/ab_cur.log 2>&1; echo "current rc=$?"; tail -1 gpurun_out/ab_cur.log
