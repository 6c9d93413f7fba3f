#!/bin/bash
# GPU box: the asynchronous serial kernel (PAXISIM_SERIAL=2) through the GPU
# parity tests, then bench A/B against the serial kernel.  usage: tools/r3_async.sh <tag> ["<configs>"]
set -o pipefail
TAG=$1; CONFIGS=${2:-"2 4 5"}
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
PAXISIM_SERIAL=2 timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests -k "not dist" > "$OUT/pytest_async.log" 2>&1
rc=$?; tail -n 2 "$OUT/pytest_async.log"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" "$OUT/pytest_async.log" | head -20; exit $rc; }
for c in $CONFIGS; do
  bash tools/ab_env.sh "$TAG/c$c" "ser|PAXISIM_SERIAL=1" "asy|PAXISIM_SERIAL=2" -- --config $c --no-shard-check ${BENCH_ARGS:-} || exit 1
done
