#!/bin/bash
# A/B the config-2 bench over library variants: tools/variants.sh <tag> libX.so ...
set -o pipefail
TAG=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out/var_$TAG
mkdir -p "$OUT"
cd "$R"
for v in "$@"; do
  n=$(basename "$v" .so)
  PAXISIM_LIB="$R/paxi_amd/variants/$v" timeout -k 10 200 python bench.py --no-cpu-baseline --steps 6 --warmup 2 > "$OUT/$n.json" 2> "$OUT/$n.err" || { echo "$n failed"; tail -5 "$OUT/$n.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$n.json'));print('$n', '%.4g msg/s'%d['value'], '%.2f ms/launch'%d['roofline']['avg_launch_ms'], 'unfaithful', d['unfaithful_clusters'])"
done
