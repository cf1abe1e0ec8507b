set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4a
timeout -k 10 120 tools/side_effects 400 > gpurun_out/r4a/side_effects_before.jsonl 2> gpurun_out/r4a/side_effects_before.err
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_multirank.py > gpurun_out/r4a/multirank.log 2>&1
