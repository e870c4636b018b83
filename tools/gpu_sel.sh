# GPU run of a selection of tests (arg: pytest -k expression), verbose, stops at the first failure
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -rs --timeout 600 --timeout-method thread -k "$1" > gpurun_out/pytest_sel.log 2>&1
rc=$?
tail -40 gpurun_out/pytest_sel.log
exit $rc
