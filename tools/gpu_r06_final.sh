#!/bin/bash
# Round-6 final GPU evidence (from the repo root via gpurun): tools/gpu_r06_final.sh <tests|bench>
#   tests: the whole -m gpu suite
#   bench: bench.py lines (rr approx headline, genome / rr exact) and rocprofv3 kernel stats of each
set -o pipefail
REPO=$(pwd); OUT=$REPO/gpurun_out/r06f; mkdir -p "$OUT"
if [ "$1" = tests ]; then
    timeout -k 10 1080 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread \
        > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
    tail -3 "$OUT/pytest_gpu.log"
    exit 0
fi
timeout -k 10 300 python -u bench.py > "$OUT/bench_rr.json" 2> "$OUT/bench_rr.err" || exit 1
timeout -k 10 300 python -u bench.py --workload genome > "$OUT/bench_genome.json" 2> "$OUT/bench_genome.err" || exit 1
timeout -k 10 400 python -u bench.py --mode exact --workload genome --steps 2 --warmup 1 --cpu-sample-mib 64 \
    > "$OUT/bench_genome_exact.json" 2> "$OUT/bench_genome_exact.err" || exit 1
timeout -k 10 400 python -u bench.py --mode exact --workload rr --steps 3 --warmup 1 \
    > "$OUT/bench_rr_exact.json" 2> "$OUT/bench_rr_exact.err" || exit 1
cat "$OUT"/bench_*.json | cut -c1-400
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_rr" -o run -- \
    python3 "$REPO/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/prof_rr.json" 2> "$OUT/prof_rr.err" || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_genome_exact" -o run -- \
    python3 "$REPO/bench.py" --mode exact --workload genome --steps 2 --warmup 1 --no-cpu-baseline \
    > "$OUT/prof_genome_exact.json" 2> "$OUT/prof_genome_exact.err" || exit 1
echo "r06 final bench done"
