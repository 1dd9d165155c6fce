# BDPT knobs in wide mode: walk-tail threshold and task groups
set -o pipefail
cd $GRAFT_REPO_ROOT
AB_TAG=r06v AB_CONFIGS="c4 c4share" bash tools/ab2.sh base base:LUMO_BDPT_TAIL=32768 base:LUMO_BDPT_TAIL=131072 base:LUMO_BDPT_GROUPS=3 base:LUMO_BDPT_GROUPS=1 base
