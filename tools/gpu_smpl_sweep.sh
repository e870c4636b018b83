# exact-smpl tuning sweep on the 1 GiB genome text (unprofiled, 2 runs each): LANE SCAN CHUNK
out=gpurun_out/smpl_sweep.txt; : > $out
for cfg in "8 4096 256" "8 512 256" "8 1024 256" "0 512 256" "8 512 1024" "8 512 64" "10 512 256"; do
  set -- $cfg
  echo "LANE=$1 SCAN=$2 CHUNK=$3" >> $out
  LZ77SSS_SMPL_LANE=$1 LZ77SSS_SMPL_SCAN=$2 LZ77SSS_SMPL_CHUNK=$3 timeout -k 10 100 python -u tools/smpl_prof.py genome 1024 2 2>&1 | grep "exact z\|smpl_tasks\|smpl_bridges" >> $out || exit 1
done
