# resident sharded test + bench lines (no CPU baseline) for a quick look
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread -k "resident" > gpurun_out/pytest_sel.log 2>&1 || { tail -40 gpurun_out/pytest_sel.log; exit 1; }
tail -3 gpurun_out/pytest_sel.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b_rr.json 2> gpurun_out/b_rr.err || { tail -20 gpurun_out/b_rr.err; exit 1; }
timeout -k 10 300 python bench.py --workload genome --no-cpu-baseline > gpurun_out/b_genome.json 2> gpurun_out/b_genome.err || { tail -20 gpurun_out/b_genome.err; exit 1; }
timeout -k 10 300 python bench.py --shard --steps 3 --warmup 1 > gpurun_out/b_shard.json 2> gpurun_out/b_shard.err || { tail -20 gpurun_out/b_shard.err; exit 1; }
cat gpurun_out/b_rr.json gpurun_out/b_genome.json gpurun_out/b_shard.json
