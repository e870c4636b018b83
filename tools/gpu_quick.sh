# quick GPU check: parity tests, rr bench, one debug-instrumented rr run (phase laps on stderr)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
WL=${1:-rr}
timeout -k 10 300 python bench.py --workload $WL --no-cpu-baseline > gpurun_out/bench_$WL.json 2> gpurun_out/bench_$WL.err || { tail -20 gpurun_out/bench_$WL.err; exit 1; }
cat gpurun_out/bench_$WL.json
LZ77SSS_DEBUG=1 timeout -k 10 300 python bench.py --workload $WL --no-cpu-baseline --steps 1 --warmup 1 > /dev/null 2> gpurun_out/debug_$WL.err || exit 1
grep -v "^\[sa_s\] [a-z ]*ok$" gpurun_out/debug_$WL.err | tail -60
