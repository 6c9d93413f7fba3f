#!/bin/bash
# Round-end pass A on the GPU box: parity suite, smoke, and PMC HBM traffic of
# every bench config's step kernel on this build (tools/traffic.sh), copied
# where bench.py looks for it.   Usage: tools/round_end_a.sh <tag>
set -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
bash tools/traffic.sh 2 > "$OUT/traffic2.log" 2>&1 || { echo "traffic 2 failed"; tail -5 "$OUT/traffic2.log"; exit 1; }
for c in 3 4 5; do
  bash tools/traffic.sh $c --steps 6 --warmup 2 > "$OUT/traffic$c.log" 2>&1 || { echo "traffic $c failed"; tail -5 "$OUT/traffic$c.log"; exit 1; }
done
for c in 2 3 4 5; do python3 -c "import json; d=json.load(open('gpurun_out/traffic/traffic_config$c.json')); print($c, d['kernel'], round(d['bytes_per_launch']/1e9,2), 'GB/launch vs alg', round(d['alg_bytes_per_launch']/1e9,2))"; done
