set -e
mkdir -p gpurun_out
export BENCH_ARGS="--res 512 --spp 256"
bash tools/ab.sh base w3 w5 sh2
for g in 512 1024 4096; do LUMO_LDS_GRID=$g timeout -k 10 300 python bench.py --steps 1 --warmup 1 --cpu-baseline 0 --res 512 --spp 256 > gpurun_out/ab_grid$g.json 2>/dev/null; done
bash tools/pmc.sh sq1 "SQ_WAVES SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES" --steps 1 --warmup 0 --cpu-baseline 0 --res 512 --spp 64
bash tools/pmc.sh sq2 "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_INSTS_VALU_FLOPS_FP64" --steps 1 --warmup 0 --cpu-baseline 0 --res 512 --spp 64
python3 tools/pmc_report.py sq1 sq2 > gpurun_out/pmc_report.txt
echo ok
