#!/bin/bash
set -eo pipefail
timeout -k 10 300 bash tools/lsdcheck.sh
bash tools/gpu_quick.sh r04r "lsd_base or dense or (stream_hash and rr) or medium"
