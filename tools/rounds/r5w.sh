#!/bin/bash
# Round-5 GPU call W: pipelined launches as the default (PAXISIM_PIPE 4; compaction every two chunks;
# config 3 in 20-step chunks): the GPU suite, then mirrored A/Bs against the unpipelined launches.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5w
mkdir -p $O
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -4 "$O/$n.log" | cut -c1-300
  case $rc in 0) return 0 ;; *) echo "stopping after $n"; exit $rc ;; esac
}
step pytest 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu
REPS=2 step ab_c2 600 tools/ab_env.sh r5w/ab_c2 "pipe|X=1" "off|PAXISIM_PIPE=1" -- --config 2 --no-shard-check
REPS=2 step ab_c3 600 tools/ab_env.sh r5w/ab_c3 "pipe|X=1" "off|PAXISIM_PIPE=1 PAXISIM_LAUNCH_STEPS=80" -- --config 3 --no-shard-check
REPS=2 step ab_c4 600 tools/ab_env.sh r5w/ab_c4 "pipe|X=1" "off|PAXISIM_PIPE=1" -- --config 4 --no-shard-check
REPS=2 step ab_c5 600 tools/ab_env.sh r5w/ab_c5 "pipe|X=1" "off|PAXISIM_PIPE=1" -- --config 5 --no-shard-check
