#!/bin/bash
# Round-5 GPU call AD: config 3's chunking under pipelining (80-step bench steps).
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5ad
mkdir -p $O
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -6 "$O/$n.log" | cut -c1-300
  case $rc in 0) return 0 ;; *) echo "stopping after $n"; exit $rc ;; esac
}
REPS=2 step ab_c3 900 tools/ab_env.sh r5ad/ab_c3 "s20k4|X=1" "s10k8|PAXISIM_LAUNCH_STEPS=10 PAXISIM_PIPE=8" "s16k5|PAXISIM_LAUNCH_STEPS=16 PAXISIM_PIPE=5" "s40k2|PAXISIM_LAUNCH_STEPS=40" -- --config 3 --no-shard-check
