# greedy lookup-path checks + A/B phase timings (genome, 5 steps each)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "dense or medium_vs_oracle or pred or one_gib or window or bounded" --timeout 300 --timeout-method thread > gpurun_out/pytest_sel.log 2>&1 || { tail -30 gpurun_out/pytest_sel.log; exit 1; }
tail -2 gpurun_out/pytest_sel.log
timeout -k 10 200 python3 tools/phase_stats.py genome 5 || exit 1
LZ77SSS_NO_IPOSR=1 timeout -k 10 200 python3 tools/phase_stats.py genome 5 || exit 1
timeout -k 10 200 python3 tools/phase_stats.py genome 5 || exit 1
