# greedy debug laps of one genome factorization (log in gpurun_out/dbg_genome.log)
mkdir -p gpurun_out
LZ77SSS_DEBUG=1 timeout -k 10 300 python3 tools/prof_step.py genome 1 > gpurun_out/dbg_genome.log 2>&1
rc=$?; grep -c . gpurun_out/dbg_genome.log; exit $rc
