#!/bin/bash
# Bench variants given as "name|ENV=V ENV2=V" pairs (PAXISIM_LIB selects a library variant).
# Usage: [REPS=n] tools/ab_env.sh <tag> "<name>|<env assignments> [BENCH_ARGS=<args>]" ... -- <bench args>
# With REPS > 1 the variants run in mirrored rounds (A B C, C B A, A B C, ...):
# identical back-to-back runs on one box can land in two modes ~6% apart
# (round 5, gpurun_out/r5c/ab_lin: the same config-3 kernel alternated
# 24.9 / 26.3 ms per launch), so a fixed A B A B order can pin one variant
# to one mode.  Compare medians over rounds (tools/ab_summary.py).
set -o pipefail
TAG=$1; shift
VARS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do VARS+=("$1"); shift; done
[ "$1" == "--" ] && shift
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
REPS=${REPS:-1}
for ((rep = 0; rep < REPS; rep++)); do
  ORDER=("${VARS[@]}")
  if (( rep % 2 == 1 )); then ORDER=(); for ((k = ${#VARS[@]} - 1; k >= 0; k--)); do ORDER+=("${VARS[$k]}"); done; fi
  for v in "${ORDER[@]}"; do
    n=${v%%|*}; e=${v#*|}
    # "BENCH_ARGS=..." (last in a variant's list): extra bench.py arguments of that variant
    extra=""
    if [[ "$e" == *"BENCH_ARGS="* ]]; then extra=${e#*BENCH_ARGS=}; e=${e%%BENCH_ARGS=*}; fi
    f=$n; (( REPS > 1 )) && f=${n}_r$rep
    env $e X_AB=1 timeout -k 10 300 python bench.py --no-cpu-baseline "$@" $extra > "$OUT/$f.json" 2> "$OUT/$f.err" || { echo "$f failed"; tail -5 "$OUT/$f.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/$f.json')); l=d.get('linearizability') or {}; print('$f', '%.4e'%d['value'], round(d['roofline']['avg_launch_ms'],2), d['config']['tiles_per_cu'], round(l.get('scan_s', 0), 3))"
  done
done
(( REPS > 1 )) && python3 "$R/tools/ab_summary.py" "$OUT"
exit 0
