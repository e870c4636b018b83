set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_sharded_sss.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pt_sharded.log 2>&1 || { tail -40 gpurun_out/pt_sharded.log; exit 1; }
tail -8 gpurun_out/pt_sharded.log
timeout -k 10 300 python bench.py --mode sss --size-gib 50 --steps 3 --warmup 1 > gpurun_out/bench_sss50.json 2> gpurun_out/bench_sss50.err || { tail -20 gpurun_out/bench_sss50.err; exit 1; }
cat gpurun_out/bench_sss50.json
