set -o pipefail
cd $GRAFT_REPO_ROOT
AB_TAG=r06g AB_CONFIGS="c3 c2" bash tools/ab2.sh base base:LUMO_TOP_GRID=192 base:LUMO_TOP_GRID=256 base:LUMO_TOP=0 base:LUMO_TOP_GRID=64 base:LUMO_RAY_SORT=1
