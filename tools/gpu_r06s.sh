# k_bounce_q arguments through a per-stream device block (LUMO_BOUNCE_ARGPTR): tests, then A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06s
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06s/tests.log 2>&1 &&
AB_TAG=r06s AB_CONFIGS="c1 c1share c2" bash tools/ab2.sh base argval base argval
