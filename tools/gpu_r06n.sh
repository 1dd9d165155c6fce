set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06n
timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06n/tests.log 2>&1 &&
AB_TAG=r06n AB_CONFIGS="c4 c3 c2" bash tools/ab2.sh base objinl base objinl
