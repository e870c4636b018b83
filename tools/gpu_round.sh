set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py > gpurun_out/bench_rr.json 2> gpurun_out/bench_rr.err && cat gpurun_out/bench_rr.json
timeout -k 10 300 python bench.py --workload genome --no-cpu-baseline > gpurun_out/bench_genome.json 2> gpurun_out/bench_genome.err && cat gpurun_out/bench_genome.json
