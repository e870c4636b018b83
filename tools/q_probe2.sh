set -eo pipefail
REPO=$(pwd); mkdir -p gpurun_out/qprobe2
cd /tmp && export TMPDIR=/tmp
for v in base c1 c2 c3; do
  if [ $v != base ]; then export LZ77SSS_LIB=$REPO/tools/tmp_v/$v/liblz77sss_hip.so; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d "$REPO/gpurun_out/qprobe2/$v" -o run -- python3 "$REPO/tools/q_probe.py" rr > "$REPO/gpurun_out/qprobe2/$v.log" 2>&1
  python3 -c "
import csv
r=[x for x in csv.DictReader(open('$REPO/gpurun_out/qprobe2/$v/run_kernel_stats.csv')) if 'k_q_anchors' in x['Name']]
print('$v', [round(float(x['AverageNs'])/1e3,1) for x in r])"
done
