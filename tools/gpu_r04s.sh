#!/bin/bash
set -eo pipefail
for c in 32 16 24 48 64; do
  LZ77SSS_SLOT_CHUNK=$c timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_r04s_c$c.json 2> /dev/null
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_r04s_c$c.json').read().strip().splitlines()[-1]); print('chunk', $c, d['ms_per_step'], d['config']['phase_ms'])"
done
