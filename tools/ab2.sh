set -o pipefail
L=kcptube_amd/libkfec.so
timeout -k 10 200 env AB_RANDOM=1 python tools/ab.py 2 $L $L:KFEC_GRID_ALL=1 -- 10 13 1400 1048576 > gpurun_out/ab2_103.log 2>&1 || exit 1
timeout -k 10 300 env AB_ITERS=3 python tools/ab.py 1 $L $L:KFEC_GRID_ALL=1 -- 200 255 1440 262144 > gpurun_out/ab2_200.log 2>&1 || exit 1
timeout -k 10 200 python tools/ab.py 2 $L $L:KFEC_GRID_ALL=1 -- 20 23 1400 1048576 > gpurun_out/ab2_1400.log 2>&1 || exit 1
cat gpurun_out/ab2_*.log
