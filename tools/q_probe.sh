set -eo pipefail
REPO=$(pwd); mkdir -p gpurun_out/qprobe
cd /tmp && export TMPDIR=/tmp
for t in random256 zeros period50 period150 period1000 rr genome; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d "$REPO/gpurun_out/qprobe/$t" -o run -- python3 "$REPO/tools/q_probe.py" $t > "$REPO/gpurun_out/qprobe/$t.log" 2>&1
  python3 -c "
import csv,sys
r=[x for x in csv.DictReader(open('$REPO/gpurun_out/qprobe/$t/run_kernel_stats.csv')) if 'k_q_anchors' in x['Name'] or 'k_sss_stream' in x['Name']]
print('$t', [(x['Name'][4:16], round(float(x['AverageNs'])/1e3,1)) for x in r])"
done
