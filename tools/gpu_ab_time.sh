#!/bin/bash
# Wall-clock A/B of library builds on the default bench (from the repo root via gpurun):
#   tools/gpu_ab_time.sh <rounds> <lib.so>...   -> one "lib ms_per_step" line per run, alternating
set -o pipefail
R=$1; shift
for r in $(seq "$R"); do
    for LIB in "$@"; do
        LZ77SSS_LIB="$LIB" timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 20 --warmup 3 \
            > gpurun_out/abt.json 2> gpurun_out/abt.err || exit 1
        python3 -c "import json,sys; d=json.loads(open('gpurun_out/abt.json').read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d['config']['phase_ms'])" "$LIB"
    done
done
