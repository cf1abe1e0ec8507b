set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gtest.log 2>&1 || { tail -30 gpurun_out/gtest.log; exit 1; }
tail -3 gpurun_out/gtest.log
timeout -k 10 240 python bench.py > gpurun_out/bench_203.json 2> gpurun_out/bench_203.err && cat gpurun_out/bench_203.json
timeout -k 10 200 python bench.py --config 10:3dec --no-cpu > gpurun_out/bench_103.json && cat gpurun_out/bench_103.json
timeout -k 10 200 python bench.py --config 200:55 --no-cpu --steps 5 > gpurun_out/bench_20055.json && cat gpurun_out/bench_20055.json
bash tools/profile.sh r01b
