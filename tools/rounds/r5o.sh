#!/bin/bash
# Round-5 GPU call O: the two run modes.  Lists the box's PMC counters (for a
# translation-miss pass), then places config 3's arena three ways in mirrored rounds:
# plainly, physically contiguous (PAXISIM_ARENA_CONTIG=1), and behind a freed 120 GB pad.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5o
mkdir -p $O
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -2 "$O/$n.log" | cut -c1-300
  case $rc in 0) return 0 ;; *) echo "stopping after $n"; exit $rc ;; esac
}
export TMPDIR=/tmp
step list 120 rocprofv3 --list-avail
step contig_once 300 env PAXISIM_ARENA_CONTIG=1 python bench.py --no-cpu-baseline --no-shard-check --config 3 --steps 5
REPS=4 step ab_place 900 tools/ab_env.sh r5o/ab_place "plain|X=1" "contig|PAXISIM_ARENA_CONTIG=1" "pad|PAXISIM_ARENA_PAD_MB=120000" -- --config 3 --no-shard-check
