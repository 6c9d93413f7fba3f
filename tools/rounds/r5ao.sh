#!/bin/bash
# Round-5 GPU call AO: every config's bench line on another box (build 2acd10e7), for the spread.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5ao
mkdir -p $O
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"
  case $rc in 0) return 0 ;; *) echo "stopping after $n"; exit $rc ;; esac
}
for c in 2 3 4 5; do step bench_config$c 400 python bench.py --config $c; done
step bench_config4_fz0 400 python bench.py --config 4 --fz 0
