#!/bin/bash
# Round-5 GPU call AI: pipelined against unpipelined launches again, on another box (configs 5, 2, 3).
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5ai
mkdir -p $O
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -4 "$O/$n.log" | cut -c1-300
  case $rc in 0) return 0 ;; *) echo "stopping after $n"; exit $rc ;; esac
}
REPS=2 step ab_c5 600 tools/ab_env.sh r5ai/ab_c5 "pipe|X=1" "off|PAXISIM_PIPE=1" -- --config 5 --no-shard-check
REPS=2 step ab_c2 600 tools/ab_env.sh r5ai/ab_c2 "pipe|X=1" "off|PAXISIM_PIPE=1 PAXISIM_LAUNCH_STEPS=50" -- --config 2 --no-shard-check
REPS=2 step ab_c3 600 tools/ab_env.sh r5ai/ab_c3 "pipe|X=1" "off|PAXISIM_PIPE=1 PAXISIM_LAUNCH_STEPS=80" -- --config 3 --no-shard-check
