#!/bin/bash
# phase check: S=10 with short vs long warm-up, at 64K and 1M clusters
R=$(cd "$(dirname "$0")/.." && pwd)
for C in 65536 1048576; do for W in 1 20; do
  timeout -k 10 200 python "$R/bench.py" --no-cpu-baseline --clusters $C --sim-steps 10 --steps 5 --warmup $W > /tmp/o.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('/tmp/o.json'));print($C,'S=10 warm',$W,'%.3g msg/s'%d['value'],'%.2f ms/launch'%d['roofline']['avg_launch_ms'])"
done; done
