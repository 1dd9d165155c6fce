set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/${TAG:-r06b}
timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py -x -v --timeout 400 --timeout-method thread > gpurun_out/${TAG:-r06b}/pytest.log 2>&1 && \
bash tools/gpu_ab_accel.sh
