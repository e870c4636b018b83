# which phrases the converged greedy chain rolls over (genome), log in gpurun_out/dbg_jump.log
mkdir -p gpurun_out
LZ77SSS_DEBUG=1 LZ77SSS_DEBUG_JUMP=1 timeout -k 10 300 python3 tools/prof_step.py genome 0 > gpurun_out/dbg_jump.log 2>&1
rc=$?; grep "jump" gpurun_out/dbg_jump.log; exit $rc
