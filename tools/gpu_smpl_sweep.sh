# exact-smpl tuning sweep on the 1 GiB genome text (unprofiled, 2 runs each): LSCAN SCAN
out=gpurun_out/smpl_sweep.txt; : > $out
for cfg in "8 1024" "32 1024" "128 1024" "512 1024" "128 256" "128 4096"; do
  set -- $cfg
  echo "LSCAN=$1 SCAN=$2" >> $out
  LZ77SSS_SMPL_LSCAN=$1 LZ77SSS_SMPL_SCAN=$2 timeout -k 10 100 python -u tools/smpl_prof.py genome 1024 2 2>&1 | grep "exact z\|smpl_tasks\|smpl_bridges" >> $out || exit 1
done
