#!/bin/bash
# Round-5 GPU call V: pipelined launches on the compacting configs (2 and 4: compaction every 100 /
# 200 steps lets 2 / 4 chunks fuse) and on config 3 (80-step bench steps as 4 chunks of 20).
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5v
mkdir -p $O
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -4 "$O/$n.log" | cut -c1-300
  case $rc in 0) return 0 ;; *) echo "stopping after $n"; exit $rc ;; esac
}
REPS=2 step ab_c2 900 tools/ab_env.sh r5v/ab_c2 "base|X=1" "p2c100|PAXISIM_PIPE=2 PAXISIM_COMPACT_EVERY=100" "p4c200|PAXISIM_PIPE=4 PAXISIM_COMPACT_EVERY=200" "c100|PAXISIM_COMPACT_EVERY=100" -- --config 2 --no-shard-check
REPS=2 step ab_c4 600 tools/ab_env.sh r5v/ab_c4 "base|X=1" "p4c200|PAXISIM_PIPE=4 PAXISIM_COMPACT_EVERY=200" -- --config 4 --no-shard-check
REPS=2 step ab_c3 600 tools/ab_env.sh r5v/ab_c3 "base|X=1" "p4l20|PAXISIM_PIPE=4 PAXISIM_LAUNCH_STEPS=20" -- --config 3 --no-shard-check
