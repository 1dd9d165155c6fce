set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r06e
timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py -x -v --timeout 400 --timeout-method thread > gpurun_out/r06e/pytest.log 2>&1 && \
timeout -k 10 900 python -u bench.py --steps 1 --warmup 1 --cpu-baseline 0 > gpurun_out/r06e/bench.json 2> gpurun_out/r06e/bench.err
