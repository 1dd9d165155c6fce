set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r06d
timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py -x -v --timeout 400 --timeout-method thread > gpurun_out/r06d/pytest.log 2>&1 && \
AB_TAG=r06d AB_ACCEL=wide AB_CONFIGS="c1 c2 c3 c4" bash tools/ab2.sh base anysort0 && \
AB_TAG=r06d AB_ACCEL=lumo AB_CONFIGS="c1 c3" bash tools/ab2.sh base:L=lumo
