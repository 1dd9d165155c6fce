set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r06a
timeout -k 10 1000 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_parity.py::test_tiles_match_oracle tests/test_gpu_trace.py -x -v --timeout 400 --timeout-method thread > gpurun_out/r06a/pytest.log 2>&1
