#!/bin/bash
# Throughput vs cluster count for one library variant: tools/sweep3.sh <tag> <lib.so>
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out/sweep_$1
mkdir -p "$OUT"
export PAXISIM_LIB=$R/paxi_amd/variants/$2
for C in 16384 65536 262144 1048576; do
  timeout -k 10 200 python "$R/bench.py" --no-cpu-baseline --clusters $C --steps 4 --warmup 2 > "$OUT/c$C.json" 2>/dev/null || { echo "fail C=$C"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/c$C.json'));print($C,'%.3g msg/s'%d['value'],'%.2f ms/launch'%d['roofline']['avg_launch_ms'])"
done
