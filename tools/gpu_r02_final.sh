# round-2 evidence: profiles (rr, genome) + bench lines (outputs under gpurun_out/, progress on stdout)
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r02b}
bash tools/gpu_profile2.sh $TAG rr && bash tools/gpu_profile2.sh $TAG genome || exit 1
b() { local name=$1; shift; timeout -k 10 900 python bench.py "$@" > gpurun_out/bench_${TAG}_$name.json 2> gpurun_out/bench_${TAG}_$name.err || { tail -20 gpurun_out/bench_${TAG}_$name.err; exit 1; }; echo "bench $name done"; }
b rr && b genome --workload genome && b rr_lnf --phr-mode lpf_lnf_opt --no-cpu-baseline && b rr_exact --mode exact --no-cpu-baseline && b genome_exact --workload genome --mode exact --no-cpu-baseline && b sss50 --mode sss --no-cpu-baseline
cat gpurun_out/bench_${TAG}_*.json | cut -c1-300
