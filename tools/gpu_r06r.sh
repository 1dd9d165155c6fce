# wide walk stack entries in LDS (LUMO_KD_LDS) for the TOP kernels: tests, then A/B 0 / 4 / 8 / 16
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06r
timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06r/tests.log 2>&1 &&
AB_TAG=r06r AB_CONFIGS="c3 c2 c4" bash tools/ab2.sh base:LUMO_KD_LDS=0 base base:LUMO_KD_LDS=4 base:LUMO_KD_LDS=16 base:LUMO_KD_LDS=0 base
