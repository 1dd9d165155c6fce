set -e
for v in w2 w8 base; do
  lib=lumo_amd/liblumo_amd_$v.so; [ $v = base ] && lib=lumo_amd/liblumo_amd.so
  for c in c2 c3; do
    LUMO_AMD_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --config $c --spp 16 --steps 1 --warmup 0 --cpu-baseline 0 > gpurun_out/ab_${v}_$c.json 2> gpurun_out/ab_${v}_$c.err
  done
done
