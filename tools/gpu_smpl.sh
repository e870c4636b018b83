# exact-smpl: parity tests, full-size length hashes, walk profile
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_exact.py > gpurun_out/smpl_tests.txt 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_stream_hashes.py -k "exact" > gpurun_out/smpl_hash.txt 2>&1 && \
LZ77SSS_SMPL_PROF_SPLIT=67108864 LZ77SSS_SMPL_PROF=1 LZ77SSS_SMPL_CHUNK=${CHUNK:-256} timeout -k 10 200 python -u tools/smpl_prof.py genome > gpurun_out/smpl_prof_genome.txt 2>&1
