# exact-smpl: parity tests (skipped with NOTEST=1), full-size length hashes, timing, walk profile
if [ -z "$NOTEST" ]; then
  timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_exact.py > gpurun_out/smpl_tests.txt 2>&1 || exit 1
  timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_stream_hashes.py -k "exact" > gpurun_out/smpl_hash.txt 2>&1 || exit 1
fi
timeout -k 10 200 python -u tools/smpl_prof.py genome 1024 3 > gpurun_out/smpl_time_genome.txt 2>&1 || exit 1
[ -n "$NOPROF" ] || LZ77SSS_SMPL_PROF_SPLIT=67108864 LZ77SSS_SMPL_PROF=1 timeout -k 10 200 python -u tools/smpl_prof.py genome 1024 1 > gpurun_out/smpl_prof_genome.txt 2>&1
