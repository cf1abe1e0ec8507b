set -o pipefail
mkdir -p gpurun_out/ab1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab1/t.log 2>&1 || { tail -40 gpurun_out/ab1/t.log; exit 1; }
tail -1 gpurun_out/ab1/t.log
L=kcptube_amd/libkfec.so; V=kcptube_amd/variants
timeout -k 10 300 python tools/ab.py 3 $L $V/r1.so -- 20 23 1440 1048576 || exit 1
AB_ERASE=random timeout -k 10 300 python tools/ab.py 2 $L $V/r1.so -- 10 13 1400 1048576 || exit 1
AB_ERASE=iid:10000 timeout -k 10 300 python tools/ab.py 2 $L -- 20 23 1440 1048576 || exit 1
AB_ERASE=none timeout -k 10 300 python tools/ab.py 2 $L -- 20 23 1440 1048576 || exit 1
