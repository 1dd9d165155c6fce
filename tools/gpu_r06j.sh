set -o pipefail
cd $GRAFT_REPO_ROOT
AB_TAG=r06j AB_CONFIGS="c4 c3 c2" bash tools/ab2.sh base anysort1
