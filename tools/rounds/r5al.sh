#!/bin/bash
# Round-5 GPU call AL: rocprofv3 kernel traces of configs 3, 4 and 5 beside their HIP events, and
# SQ/TCC counters of config 3 (build 2acd10e7).
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5al
mkdir -p $O
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -1 "$O/$n.log" | cut -c1-300
  case $rc in 0) return 0 ;; *) echo "stopping after $n"; exit $rc ;; esac
}
export TMPDIR=/tmp
for c in 3 4 5; do
  step prof_c$c 400 rocprofv3 --kernel-trace --stats -d $O/prof_c$c -o run --output-format csv -- python bench.py --no-cpu-baseline --no-shard-check --config $c
done
P1="SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVES SQ_WAVE_CYCLES"
P3="TCC_HIT_sum TCC_MISS_sum"
step pmc_c3 400 bash tools/pmc2.sh r5al_c3 "$P1" "$P3" -- --config 3 --warmup 5 --steps 1
