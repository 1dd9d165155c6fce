set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06m
timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_bdpt.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06m/tests.log 2>&1 &&
AB_TAG=r06m AB_CONFIGS="c4 c4share" bash tools/ab2.sh base lightinl base
