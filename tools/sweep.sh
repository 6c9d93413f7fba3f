#!/bin/bash
# Quick scaling sweep of the step kernel: clusters x steps-per-launch.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out/sweep_$1; shift
mkdir -p "$OUT"
for C in 16384 65536 262144 1048576; do
  for S in 10 50; do
    timeout -k 10 200 python "$R/bench.py" --no-cpu-baseline --clusters $C --sim-steps $S --steps 3 --warmup 1 "$@" > "$OUT/c${C}_s${S}.json" 2>/dev/null || { echo "fail C=$C S=$S"; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/c${C}_s${S}.json'));print($C,$S,'%.3g msg/s'%d['value'],'%.2f ms/launch'%d['roofline']['avg_launch_ms'])"
  done
done
