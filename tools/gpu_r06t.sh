# wide builder child order (LUMO_WBVH_ORDER: 1 decreasing box area, -1 increasing): parity, A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06t
LUMO_WBVH_ORDER=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py -x -q --timeout 300 --timeout-method thread -k "full_scale or bistro or dragon_split" > gpurun_out/r06t/tests.log 2>&1 &&
AB_TAG=r06t AB_CONFIGS="c3 c2 c4" bash tools/ab2.sh base base:LUMO_WBVH_ORDER=1 base:LUMO_WBVH_ORDER=-1 base base:LUMO_WBVH_ORDER=1
