# greedy debug lines of a 16 MiB genome factorization with the lockstep query (gpurun_out/qdbg.log)
mkdir -p gpurun_out
LZ77SSS_DEBUG=1 timeout -k 10 ${QT:-60} python3 -u tools/prof_step.py genome 0 ${QSIZE:-16} > gpurun_out/qdbg.log 2>&1
rc=$?; grep -c . gpurun_out/qdbg.log; grep -E "outer|step" gpurun_out/qdbg.log | head -30 | cut -c1-150; exit $rc
