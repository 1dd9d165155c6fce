# ray sorting ahead of the wide closest-hit walks (LUMO_RAY_SORT 1 octant major, 2 origin major)
set -o pipefail
cd $GRAFT_REPO_ROOT
AB_TAG=r06z3 AB_CONFIGS="c2 c3" bash tools/ab2.sh base base:LUMO_RAY_SORT=1 base:LUMO_RAY_SORT=2 base base:LUMO_RAY_SORT=1
