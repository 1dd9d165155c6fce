set -eo pipefail
mkdir -p gpurun_out/ab
for v in "LUMO_FUSED_SPLIT=0" "LUMO_FUSED_SPLIT=1" "LUMO_FUSED_SPLIT=1 LUMO_SPLIT_GROUPS=4" "LUMO_FUSED_SPLIT=1 LUMO_SPLIT_GROUPS=1"; do
  tag=$(echo $v | tr ' =' '__')
  env $v timeout -k 10 600 python3 tools/share_times.py c1 8 256 > gpurun_out/ab/shares_c1_256_$tag.json
  echo "$v"; tail -c 230 gpurun_out/ab/shares_c1_256_$tag.json; echo
done
echo done
