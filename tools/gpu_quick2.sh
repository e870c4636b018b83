# parity subset + rr/genome bench with phase laps
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "dense or medium or c1_seeds or edge or runs or golden or lpf_lnf" > gpurun_out/pt_q2.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pt_q2.log; exit 1; }
tail -2 gpurun_out/pt_q2.log
for WL in rr genome; do
timeout -k 10 300 python bench.py --workload $WL --no-cpu-baseline > gpurun_out/bench_$WL.json 2> gpurun_out/bench_$WL.err || { tail -20 gpurun_out/bench_$WL.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_$WL.json'));print('$WL',d['value'],d['ms_per_step'],d['config']['phase_ms'],d['roofline']['avg_launch_ms'])"
done
LZ77SSS_DEBUG=1 timeout -k 10 300 python bench.py --workload rr --no-cpu-baseline --steps 1 --warmup 1 > /dev/null 2> gpurun_out/debug_rr.err || exit 1
grep -E "greedy base|lap|slot" gpurun_out/debug_rr.err | tail -30
