set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for wl in rr genome; do timeout -k 10 200 python3 tools/prof_step.py $wl 2 > gpurun_out/st_$wl.log 2>&1 || exit 1; grep "^step 2" gpurun_out/st_$wl.log | cut -c1-140; done
