set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06z2
timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06z2/tests.log 2>&1
tail -n 3 gpurun_out/r06z2/tests.log
