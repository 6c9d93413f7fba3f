#!/bin/bash
# msgs/s and launch time vs clusters per GPU and warm-up (config 2).
# Usage: tools/scale_probe.sh <tag>
set -o pipefail
TAG=${1:-scale}
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
for spec in "262144 4 6" "524288 4 6" "1048576 4 6" "1048576 1 4" "524288 12 6"; do
  set -- $spec
  timeout -k 10 200 python bench.py --clusters $1 --warmup $2 --steps $3 --no-cpu-baseline > "$OUT/c$1_w$2.json" 2> "$OUT/c$1_w$2.err" \
    || { echo "failed $spec"; tail -5 "$OUT/c$1_w$2.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/c$1_w$2.json')); print('$spec', '%.3e'%d['value'], round(d['roofline']['avg_launch_ms'],2), d['unfaithful_clusters'])"
done
