#!/bin/bash
# HBM traffic of the bench's step kernel from PMC counters, as
# MI355X_MICROARCH.md §HBM prescribes: FETCH_SIZE and WRITE_SIZE in separate
# rocprofv3 passes (they cannot share the 4 TCC slots), FETCH_SIZE doubled
# (gfx950 tallies 128-B reads at 64 B), both in KB per dispatch.  Averages
# the timed launches only (the last --steps dispatches of the step kernel).
# Usage: tools/traffic.sh <config> [bench args...]   -> gpurun_out/traffic/traffic_config<c>[_fz0].json
set -o pipefail
CFG=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out/traffic/c$CFG$([[ " $* " == *" --fz 0 "* ]] && echo _fz0)
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for ctr in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace -d "$OUT/p$i" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline --no-shard-check --config "$CFG" "$@" > "$OUT/p$i.log" 2>&1 || { echo "pass $ctr failed rc=$?"; tail -5 "$OUT/p$i.log"; exit 1; }
done
NAME=traffic_config$CFG
[[ " $* " == *" --fz 0 "* ]] && NAME=traffic_config${CFG}_fz0    # config 4's Grid variant has a record of its own
python3 "$R/tools/traffic_summary.py" "$CFG" "$OUT" "$@" > "$R/gpurun_out/traffic/$NAME.json" && cat "$R/gpurun_out/traffic/$NAME.json"
