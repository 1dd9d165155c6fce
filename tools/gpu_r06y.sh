# TOP kernels as 256-thread blocks at the same waves and CU footprint (4 blocks per CU on half the CUs)
set -o pipefail
cd $GRAFT_REPO_ROOT
AB_TAG=r06y AB_CONFIGS="c3 c2 c4" bash tools/ab2.sh base tb256:LUMO_TOP_KB=39,LUMO_TOP_GRID=512 tb256:LUMO_TOP_KB=78,LUMO_TOP_GRID=256 base tb256:LUMO_TOP_KB=39,LUMO_TOP_GRID=512
