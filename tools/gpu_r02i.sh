# greedy base-build checks + timings
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "dense or medium_vs_oracle or pred or one_gib or golden or window" --timeout 300 --timeout-method thread > gpurun_out/pytest_sel.log 2>&1 || { tail -30 gpurun_out/pytest_sel.log; exit 1; }
tail -2 gpurun_out/pytest_sel.log
for wl in rr genome; do timeout -k 10 200 python3 tools/prof_step.py $wl 2 > gpurun_out/st_$wl.log 2>&1 || exit 1; grep "^step 2" gpurun_out/st_$wl.log | cut -c1-140; done
