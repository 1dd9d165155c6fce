set -o pipefail
cd $GRAFT_REPO_ROOT
AB_TAG=r06p AB_CONFIGS="c3" bash tools/ab2.sh norefill sw3 norefill
