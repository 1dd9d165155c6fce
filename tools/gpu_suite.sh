# the whole GPU suite (pytest -m gpu) under one time limit, log under gpurun_out/$TAG
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/${TAG:-suite}
timeout -k 10 ${LIMIT:-1000} python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/${TAG:-suite}/pytest_gpu.log 2>&1
