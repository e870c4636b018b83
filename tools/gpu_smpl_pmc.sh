# exact-smpl walk kernels: SQ stall counters, HBM bytes and L2 hit rate (one rocprofv3 pass each)
K='k_chunk_walks|k_bridge_walks'
run() { timeout -s KILL 120 rocprofv3 --pmc $1 --kernel-include-regex "$K" -d gpurun_out/smpl_pmc/$2 -o $2 --output-format csv -- python3 tools/smpl_prof.py genome 1024 1 > gpurun_out/smpl_pmc_$2.log 2>&1; }
mkdir -p gpurun_out/smpl_pmc
run "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_BUSY_CYCLES" sq && \
run "FETCH_SIZE" fetch && \
run "TCC_HIT_sum TCC_MISS_sum" tcc
