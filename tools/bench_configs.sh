#!/bin/bash
# Bench lines for BASELINE configs 5, 3 and 4 on the GPU box (each with its
# own bounded CPU-oracle baseline).  Usage: tools/bench_configs.sh <tag>
set -o pipefail
TAG=${1:-cfgs}
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
for c in 5 3 4; do
  timeout -k 10 300 python bench.py --config $c --steps 6 --warmup 2 --cpu-clusters 2048 --cpu-steps 400 \
    > "$OUT/c$c.json" 2> "$OUT/c$c.err" || { echo "config $c failed"; tail -5 "$OUT/c$c.err"; exit 1; }
  cat "$OUT/c$c.json"
done
