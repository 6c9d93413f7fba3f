#!/bin/bash
# Round-5 GPU call AA: chunk length and compaction cadence under pipelining, configs 2, 4 and 5.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5aa
mkdir -p $O
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -6 "$O/$n.log" | cut -c1-300
  case $rc in 0) return 0 ;; *) echo "stopping after $n"; exit $rc ;; esac
}
REPS=2 step ab_c2 900 tools/ab_env.sh r5aa/ab_c2 "s25c75|X=1" "s25c100|PAXISIM_COMPACT_EVERY=100" "s20c60|PAXISIM_LAUNCH_STEPS=20 PAXISIM_COMPACT_EVERY=60" "s30c90|PAXISIM_LAUNCH_STEPS=30 PAXISIM_COMPACT_EVERY=90" -- --config 2 --no-shard-check
REPS=2 step ab_c4 600 tools/ab_env.sh r5aa/ab_c4 "s50c150|X=1" "s50c200|PAXISIM_COMPACT_EVERY=200" "s25c75|PAXISIM_LAUNCH_STEPS=25 PAXISIM_COMPACT_EVERY=75" -- --config 4 --no-shard-check
REPS=2 step ab_c5 600 tools/ab_env.sh r5aa/ab_c5 "s50|X=1" "s25|PAXISIM_LAUNCH_STEPS=25" -- --config 5 --no-shard-check
