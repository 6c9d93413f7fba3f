#!/bin/bash
# GPU box: round-3 measurement pass on the current build - the GPU suite, smoke,
# every config's bench line, the config-2 rocprofv3 kernel trace + stats, and
# the PMC HBM traffic of configs 2-5 (tools/traffic.sh).   usage: tools/r3_final.sh <tag>
set -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
cd "$R"
bash tools/r3_measure.sh "$TAG" "2 1 3 4 5" || exit $?
for c in 2 3 4 5; do
  bash tools/traffic.sh $c > "gpurun_out/$TAG/traffic$c.log" 2>&1 || { echo "traffic $c failed"; tail -5 "gpurun_out/$TAG/traffic$c.log"; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/traffic/traffic_config$c.json')); print($c, d['kernel'], round(d['bytes_per_launch']/1e9,2), 'GB/launch vs alg', round(d['alg_bytes_per_launch']/1e9,2))"
done
