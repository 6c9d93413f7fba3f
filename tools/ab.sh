#!/bin/bash
# A/B two builds of the library on one bench config, alternating A B A B.
# Usage: tools/ab.sh <tag> <libA> <libB> <bench args...>
set -o pipefail
TAG=$1; A=$2; B=$3; shift 3
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
for round in 1 2; do
  for v in A B; do
    lib=$A; [ $v = B ] && lib=$B
    PAXISIM_LIB=$R/$lib timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > "$OUT/$v$round.json" 2> "$OUT/$v$round.err" \
      || { echo "failed $v"; tail -5 "$OUT/$v$round.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/$v$round.json')); print('$v', '%.4e'%d['value'], round(d['roofline']['avg_launch_ms'],2))"
  done
done
