#!/bin/bash
# GPU box: serial kernels of every protocol (PAXISIM_SERIAL=1) through the GPU
# suite, then bench A/B against the replica-per-wave kernels on configs 3 and 5.
set -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
PAXISIM_SERIAL=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests -k "not dist" > "$OUT/pytest_serial.log" 2>&1
rc=$?; tail -n 3 "$OUT/pytest_serial.log"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" "$OUT/pytest_serial.log" | head -20; exit $rc; }
for c in ${CONFIGS:-5 3}; do
  bash tools/ab_env.sh "$TAG/c$c" "par|PAXISIM_SERIAL=0" "ser|PAXISIM_SERIAL=1" "serh|PAXISIM_SERIAL=1 PAXISIM_WLDS=0" -- --config $c --no-shard-check ${BENCH_ARGS:-} || exit 1
done
