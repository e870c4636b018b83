# GPU check: the whole -m gpu suite, then verbose runs of selected tests (args: pytest -k expression)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
if [ -n "$1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread -k "$1" > gpurun_out/pytest_sel.log 2>&1 || { echo SEL_FAIL; tail -40 gpurun_out/pytest_sel.log; exit 1; }
  grep -E "\|S\||passed|failed" gpurun_out/pytest_sel.log | tail -20
fi
