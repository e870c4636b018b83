# SSS correctness + timings after a k_q_anchors change
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "sss or adversarial or run or golden or one_gib or medium_vs_oracle" --timeout 300 --timeout-method thread > gpurun_out/pytest_sel.log 2>&1 || { tail -30 gpurun_out/pytest_sel.log; exit 1; }
tail -2 gpurun_out/pytest_sel.log
for wl in rr genome; do timeout -k 10 200 python3 tools/sss_time.py $wl || exit 1; done
timeout -k 10 200 python3 tools/prof_step.py rr 2 > gpurun_out/st_rr.log 2>&1 || exit 1; grep "^step 2" gpurun_out/st_rr.log | cut -c1-140
