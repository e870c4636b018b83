# kernel stats of one exact-smpl call on the 1 GiB rr text
REPO=$(pwd); OUT=$REPO/gpurun_out/r05f; mkdir -p "$OUT"; cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_rr_exact" -o run -- \
    python3 "$REPO/bench.py" --mode exact --workload rr --steps 2 --warmup 1 --no-cpu-baseline \
    > "$OUT/prof_rr_exact.json" 2> "$OUT/prof_rr_exact.err"
