# TOP kernels as several smaller blocks per CU (more waves per SIMD, a smaller TOP set each)
set -o pipefail
cd $GRAFT_REPO_ROOT
AB_TAG=r06w AB_CONFIGS="c3 c2" bash tools/ab2.sh base tb512w6:LUMO_TOP_KB=52,LUMO_TOP_GRID=384 tb256w5:LUMO_TOP_KB=31,LUMO_TOP_GRID=640 tb512w6:LUMO_TOP_KB=52,LUMO_TOP_GRID=768 base
