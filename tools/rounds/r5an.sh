#!/bin/bash
# Round-5 GPU call AN: ABD client tables in HBM (var/v_abdcl0.so: 13 tiles per CU by LDS) against LDS (11).
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5an
mkdir -p $O
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -3 "$O/$n.log" | cut -c1-300
  case $rc in 0) return 0 ;; *) echo "stopping after $n"; exit $rc ;; esac
}
REPS=2 step ab_c3 600 tools/ab_env.sh r5an/ab_c3 "lds|X=1" "hbm|PAXISIM_LIB=var/v_abdcl0.so" -- --config 3 --no-shard-check
