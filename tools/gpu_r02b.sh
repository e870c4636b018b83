set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread -k "sss or golden or adversarial or fallback or run or sync" > gpurun_out/pytest_sel.log 2>&1 || { tail -60 gpurun_out/pytest_sel.log; exit 1; }
tail -3 gpurun_out/pytest_sel.log
bash tools/gpu_trace.sh r02b rr 3 && bash tools/gpu_trace.sh r02b genome 2
