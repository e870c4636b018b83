#!/bin/bash
set -eo pipefail
bash tools/gpu_quick.sh r04e "test_gpu_parity or stream_hash or sharded or exact or decode"
LZ77SSS_NO_SPIN=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_r04e_nospin.json 2>&1
python3 -c "import json; d=json.load(open('gpurun_out/bench_r04e_nospin.json')); print('nospin', d['ms_per_step'], d['config']['phase_ms'])"
