# round evidence: profiles + bench lines (outputs under gpurun_out/)
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r02}
bash tools/gpu_profile2.sh $TAG rr && bash tools/gpu_profile2.sh $TAG genome || exit 1
timeout -k 10 600 python bench.py > gpurun_out/bench_${TAG}_rr.json 2> gpurun_out/bench_${TAG}_rr.err || { tail -20 gpurun_out/bench_${TAG}_rr.err; exit 1; }
timeout -k 10 900 python bench.py --workload genome > gpurun_out/bench_${TAG}_genome.json 2> gpurun_out/bench_${TAG}_genome.err || { tail -20 gpurun_out/bench_${TAG}_genome.err; exit 1; }
cat gpurun_out/bench_${TAG}_*.json
