#!/bin/bash
set -eo pipefail
timeout -k 10 300 bash tools/lsdcheck.sh
bash tools/gpu_quick.sh r04k "test_gpu_parity or stream_hash or u64 or sharded"
