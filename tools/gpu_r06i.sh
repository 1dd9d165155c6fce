set -o pipefail
cd $GRAFT_REPO_ROOT
AB_TAG=r06i AB_CONFIGS="c4 c4" bash tools/ab2.sh base && AB_TAG=r06i AB_CONFIGS="c4" AB_ACCEL=lumo bash tools/ab2.sh base
