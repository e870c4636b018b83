#!/bin/bash
set -eo pipefail
timeout -k 10 300 bash tools/lsdcheck.sh
bash tools/gpu_quick.sh r04j "lsd_base or medium or (stream_hash and rr) or c1_seeds or window or golden_factor or gap_index or edge or dense"
for ch in 128 256 1024 2048; do
  LZ77SSS_GAP_CHUNK=$ch timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_r04j_ch$ch.json 2> /dev/null
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_r04j_ch$ch.json').read().strip().splitlines()[-1]); print('chunk', $ch, d['ms_per_step'], d['config']['phase_ms'], d['config']['greedy'])"
done
