# wide-mode launch knobs for C3 / C2: TOP grid and TOP LDS budget
set -o pipefail
cd $GRAFT_REPO_ROOT
AB_TAG=r06u AB_CONFIGS="c3 c2" bash tools/ab2.sh base base:LUMO_TOP_GRID=256 base:LUMO_TOP_GRID=96 base:LUMO_TOP_KB=96 base:LUMO_TOP_KB=64 base base:LUMO_TOP_GRID=256
