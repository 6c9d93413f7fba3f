set -o pipefail
mkdir -p gpurun_out/r1c
timeout -k 10 200 python tools/stamps.py 65536 200 100 > gpurun_out/r1c/stamps.txt 2>&1 || { echo stamps failed; cat gpurun_out/r1c/stamps.txt | tail; exit 1; }
cat gpurun_out/r1c/stamps.txt
bash tools/pmc2.sh r1c "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" "SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum" -- --steps 3 --warmup 1 || exit 1
bash tools/bench_configs.sh r1c_cfgs
