#!/bin/bash
# Bench variants given as "name|ENV=V ENV2=V" pairs (PAXISIM_LIB selects a library variant).
# Usage: tools/ab_env.sh <tag> "<name>|<env assignments>" ... -- <bench args>
set -o pipefail
TAG=$1; shift
VARS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do VARS+=("$1"); shift; done
[ "$1" == "--" ] && shift
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
for v in "${VARS[@]}"; do
  n=${v%%|*}; e=${v#*|}
  env $e timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > "$OUT/$n.json" 2> "$OUT/$n.err" || { echo "$n failed"; tail -5 "$OUT/$n.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$n.json')); print('$n', '%.4e'%d['value'], round(d['roofline']['avg_launch_ms'],2), d['config']['tiles_per_cu'], d['config']['staged_msgs'])"
done
