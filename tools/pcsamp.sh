#!/bin/bash
# GPU box: stochastic PC sampling of the bench's step kernel (where waves stall).
#   usage: tools/pcsamp.sh <tag> <bench args...>
set -o pipefail
TAG=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles \
  --pc-sampling-interval ${PCI:-1048576} -d "$OUT/pc" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline --no-shard-check "$@" > "$OUT/pc.log" 2>&1
rc=$?; tail -n 3 "$OUT/pc.log"; ls -la "$OUT/pc"/* | head; exit $rc
