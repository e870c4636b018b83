#!/bin/bash
set -eo pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "golden or c1_seeds or gap_index or medium or (stream_hash and rr) or lsd_base or edge or runs or window" > gpurun_out/pytest_r04o.log 2>&1 || { tail -20 gpurun_out/pytest_r04o.log; exit 1; }
tail -2 gpurun_out/pytest_r04o.log
for sh in 16 18; do
  LZ77SSS_SLOT_CHUNK_SH=$sh timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_r04o_sh$sh.json 2> /dev/null
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_r04o_sh$sh.json').read().strip().splitlines()[-1]); print('sh', $sh, d['ms_per_step'], d['config']['phase_ms'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_r04o" -o run -- python3 "$GRAFT_REPO_ROOT/tools/prof_step.py" rr 3 > /dev/null 2>&1
