#!/bin/bash
# Rehearsal of bench.py's N > 1 path on a one-GPU box (from the repo root via gpurun): two ranks on
# device 0, gloo between them (LZ77SSS_BENCH_SHARE_GPU=1); the driver's runs use one GPU per rank
set -eo pipefail
OUT=$(pwd)/gpurun_out; mkdir -p "$OUT"
LZ77SSS_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 4 --warmup 1 > "$OUT/bench_n2.json" 2> "$OUT/bench_n2.err"
tail -c 1500 "$OUT/bench_n2.json"
