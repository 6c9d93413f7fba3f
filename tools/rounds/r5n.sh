#!/bin/bash
# Round-5 GPU call N (final build): every config's bench line, rocprofv3 trace of config 2, HBM traffic
# of every config's step kernel at its bench window, SQ/TCC counters of configs 2 and 5, and the checker's
# waves-per-workgroup A/B.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5n
mkdir -p $O
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -2 "$O/$n.log" | cut -c1-300
  case $rc in 0) return 0 ;; *) echo "stopping after $n"; exit $rc ;; esac
}
for c in 2 3 4 5; do step bench_config$c 400 python bench.py --config $c; done
step bench_config4_fz0 400 python bench.py --config 4 --fz 0
step bench_config1 300 python bench.py --config 1 --warmup 0 --steps 1
export TMPDIR=/tmp
step prof_c2 400 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- python bench.py --no-cpu-baseline --no-shard-check --config 2
step traffic2 400 bash tools/traffic.sh 2
step traffic3 300 bash tools/traffic.sh 3
step traffic4 400 bash tools/traffic.sh 4
step traffic4_fz0 400 bash tools/traffic.sh 4 --fz 0
step traffic5 400 bash tools/traffic.sh 5
P1="SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVES SQ_WAVE_CYCLES"
P2="SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_THREAD_CYCLES_VALU"
P3="TCC_HIT_sum TCC_MISS_sum"
step pmc_c2 600 bash tools/pmc2.sh r5n_c2 "$P1" "$P2" "$P3" -- --config 2 --warmup 5 --steps 1
step pmc_c5 400 bash tools/pmc2.sh r5n_c5 "$P1" "$P3" -- --config 5 --warmup 5 --steps 1
REPS=2 step ab_lin 600 tools/ab_env.sh r5n/ab_lin "lw2|X=1" "lw1|PAXISIM_LIB=var/v_linlw1.so" "lw4|PAXISIM_LIB=var/v_linlw4.so" -- --config 3
