#!/bin/bash
# Launch time vs cluster count (occupancy probe): tools/sweep4.sh <tag> <lib.so> <clusters...>
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
TAG=$1; LIB=$2; shift 2
OUT=$R/gpurun_out/sweep_$TAG
mkdir -p "$OUT"
export PAXISIM_LIB=$R/paxi_amd/variants/$LIB
for C in "$@"; do
  timeout -k 10 200 python "$R/bench.py" --no-cpu-baseline --clusters $C --steps 4 --warmup 2 > "$OUT/c$C.json" 2>/dev/null || { echo "fail C=$C"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/c$C.json'));print('$LIB', $C,'%.3g msg/s'%d['value'],'%.2f ms/launch'%d['roofline']['avg_launch_ms'])"
done
