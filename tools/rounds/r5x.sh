#!/bin/bash
# Round-5 GPU call X: config 2's chunk length and compaction cadence under pipelining.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5x
mkdir -p $O
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -6 "$O/$n.log" | cut -c1-300
  case $rc in 0) return 0 ;; *) echo "stopping after $n"; exit $rc ;; esac
}
REPS=2 step ab_c2 900 tools/ab_env.sh r5x/ab_c2 "s50c100|X=1" "s25c50|PAXISIM_LAUNCH_STEPS=25 PAXISIM_COMPACT_EVERY=50" "s25c75|PAXISIM_LAUNCH_STEPS=25 PAXISIM_COMPACT_EVERY=75" "s50c150|PAXISIM_COMPACT_EVERY=150" -- --config 2 --no-shard-check
