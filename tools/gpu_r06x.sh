# TOP kernels as 256-thread blocks with the closest-hit walks at 5 waves per SIMD
set -o pipefail
cd $GRAFT_REPO_ROOT
AB_TAG=r06x AB_CONFIGS="c3 c2 c4" bash tools/ab2.sh base tb256c5:LUMO_TOP_KB=31,LUMO_TOP_GRID=640 tb256c5:LUMO_TOP_KB=31,LUMO_TOP_GRID=320 tb256c5:LUMO_TOP_KB=39,LUMO_TOP_GRID=512 base
