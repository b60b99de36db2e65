bash tools/sweep.sh 1e9 && CFG=c3 bash tools/sweep.sh 1e9 w8 w4 > gpurun_out/sweep_c3.txt && mkdir -p gpurun_out/sw3 && cp gpurun_out/sweep/*.log gpurun_out/sw3/
