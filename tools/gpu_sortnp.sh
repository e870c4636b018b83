mkdir -p gpurun_out
timeout -k 10 300 ./tools/microbench/sortbench2 > gpurun_out/sortbench2.log 2>&1 || { cat gpurun_out/sortbench2.log; exit 1; }
cat gpurun_out/sortbench2.log
bash tools/gpu_nopred.sh
