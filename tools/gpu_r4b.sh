# round 4: worker lease + matrix cache -- side effects, fallback, worker parity, latency with the reference leg,
# batched throughput beside the per-call thread
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4b
mkdir -p $O
timeout -k 10 120 tools/side_effects 400 > $O/side_effects_after.jsonl 2> $O/side_effects_after.err
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_side_effects.py tests/test_gpu_worker.py > $O/tests.log 2>&1
timeout -k 10 120 tools/latency_bench > $O/latency.json 2> $O/latency.err
timeout -k 10 120 tools/latency_bench > $O/latency_2.json 2> $O/latency_2.err
timeout -k 10 200 python tools/concurrent_bench.py > $O/concurrent.json 2> $O/concurrent.err
