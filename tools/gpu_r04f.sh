#!/bin/bash
set -eo pipefail
bash tools/gpu_quick.sh r04f "test_gpu_parity or stream_hash or sharded or u64"
