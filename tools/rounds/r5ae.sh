#!/bin/bash
# Round-5 GPU call AE (final build: pipelined launches gated by the XCD probe): every config's bench line, rocprofv3 trace of config 2, HBM traffic
# of every config's step kernel at its bench window, SQ/TCC counters of configs 2 and 5, and the checker's
# waves-per-workgroup A/B.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5ae
mkdir -p $O
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -2 "$O/$n.log" | cut -c1-300
  case $rc in 0) return 0 ;; *) echo "stopping after $n"; exit $rc ;; esac
}
export TMPDIR=/tmp
step traffic2 400 bash tools/traffic.sh 2
step traffic3 300 bash tools/traffic.sh 3
step traffic4 400 bash tools/traffic.sh 4
step traffic4_fz0 400 bash tools/traffic.sh 4 --fz 0
step traffic5 400 bash tools/traffic.sh 5
mkdir -p profiles && for n in 2 3 4 4_fz0 5; do cp gpurun_out/traffic/traffic_config$n.json profiles/; done
for c in 2 3 4 5; do step bench_config$c 400 python bench.py --config $c; done
step bench_config4_fz0 400 python bench.py --config 4 --fz 0
step bench_config1 300 python bench.py --config 1 --warmup 0 --steps 1
step prof_c2 400 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- python bench.py --no-cpu-baseline --no-shard-check --config 2
step pytest 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
P1="SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVES SQ_WAVE_CYCLES"
P2="SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_THREAD_CYCLES_VALU"
P3="TCC_HIT_sum TCC_MISS_sum"
step pmc_c2 600 bash tools/pmc2.sh r5ae_c2 "$P1" "$P2" "$P3" -- --config 2 --warmup 5 --steps 1
step pmc_c5 400 bash tools/pmc2.sh r5ae_c5 "$P1" "$P3" -- --config 5 --warmup 5 --steps 1
