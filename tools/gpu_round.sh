# Round-end GPU evidence: parity tests, profiles (kernel stats + PMC HBM bytes of the SSS kernel), bench lines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
bash tools/gpu_profile.sh r01 rr && bash tools/gpu_profile.sh r01 genome || exit 1
# (profiles/ summaries are made locally from the merged gpurun_out/: tools/summarize_profile.py)
timeout -k 10 600 python bench.py > gpurun_out/bench_rr.json 2> gpurun_out/bench_rr.err || { tail -20 gpurun_out/bench_rr.err; exit 1; }
timeout -k 10 300 python bench.py --workload genome --cpu-sample-mib 128 > gpurun_out/bench_genome.json 2> gpurun_out/bench_genome.err || exit 1
timeout -k 10 300 python bench.py --phr-mode lpf_lnf_opt > gpurun_out/bench_rr_lnf.json 2> gpurun_out/bench_rr_lnf.err || exit 1
timeout -k 10 300 python bench.py --mode exact --steps 3 --warmup 1 > gpurun_out/bench_rr_exact.json 2> gpurun_out/bench_rr_exact.err || exit 1
timeout -k 10 300 python bench.py --mode exact --workload genome --steps 3 --warmup 1 > gpurun_out/bench_genome_exact.json 2> gpurun_out/bench_genome_exact.err || exit 1
timeout -k 10 300 python bench.py --mode sss --size-gib 50 --steps 3 --warmup 1 > gpurun_out/bench_sss50.json 2> gpurun_out/bench_sss50.err || exit 1
cat gpurun_out/bench_*.json
