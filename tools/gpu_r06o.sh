set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06o
timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06o/tests.log 2>&1 &&
AB_TAG=r06o AB_CONFIGS="c3 c4 c3" bash tools/ab2.sh base
