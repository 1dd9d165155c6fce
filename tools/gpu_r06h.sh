set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r06h
timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py -x -v --timeout 400 --timeout-method thread > gpurun_out/r06h/pytest.log 2>&1 && \
AB_TAG=r06h AB_CONFIGS="c3 c2 c4" bash tools/ab2.sh base && AB_TAG=r06h AB_CONFIGS="c1" AB_ACCEL=wide bash tools/ab2.sh base
