set -eo pipefail
O=gpurun_out/r04y; mkdir -p $O
run() { # name share envs...
  n=$1; sh=$2; shift 2
  env "$@" timeout -k 10 200 python3 bench.py --share $sh --steps 3 --warmup 1 --bistro-frames 0 --cpu-baseline 0 > $O/$n.json 2> $O/$n.err
  python3 -c "import json; d=json.load(open('$O/$n.json')); print('$n', '$sh', d['ms_per_step'])"
}
run s2_auto 0/2 LUMO_X=0
run s2_m2 0/2 LUMO_MERGE=2
run s4_auto 0/4 LUMO_X=0
run s4_m1 0/4 LUMO_MERGE=1
run s4_m4 0/4 LUMO_MERGE=4
run s4_m1h6 0/4 LUMO_MERGE=1 LUMO_HEADS=6
run s8_m8 0/8 LUMO_MERGE=8
