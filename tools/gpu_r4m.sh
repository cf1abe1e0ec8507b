# round 4: config 5's partition at scale, rehearsed on one GPU: 8 ranks x 512k groups of fec=20:3 (4M global
# groups, 156 GB of HBM), every rank verifying its recovered shards bit-exact; then one rank over the same 4M.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4m; mkdir -p $O
KFEC_BENCH_REHEARSAL=1 timeout -k 10 600 python bench.py --gpus 8 --groups 524288 --no-cpu --steps 5 --warmup 1 > $O/rehearsal_8x512k.json 2> $O/rehearsal_8x512k.err || { tail -20 $O/rehearsal_8x512k.err; exit 1; }
timeout -k 10 300 python bench.py --gpus 1 --groups 4194304 --no-cpu --steps 5 --warmup 1 > $O/single_4M.json 2> $O/single_4M.err || { tail -20 $O/single_4M.err; exit 1; }
cut -c1-400 $O/rehearsal_8x512k.json $O/single_4M.json
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "batch_vs_oracle" > $O/parity_cases.log 2>&1 || { tail -30 $O/parity_cases.log; exit 1; }
tail -1 $O/parity_cases.log
