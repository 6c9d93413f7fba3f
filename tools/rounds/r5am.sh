#!/bin/bash
# Round-5 GPU call AM: ABD serial kernel at 4 waves per SIMD (128 VGPRs, var/v_abd4.so) against 3.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5am
mkdir -p $O
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -3 "$O/$n.log" | cut -c1-300
  case $rc in 0) return 0 ;; *) echo "stopping after $n"; exit $rc ;; esac
}
REPS=2 step ab_c3 600 tools/ab_env.sh r5am/ab_c3 "w3|X=1" "w4|PAXISIM_LIB=var/v_abd4.so" -- --config 3 --no-shard-check
