#!/bin/bash
# GPU box: the serial kernel (PAXISIM_SERIAL=1) - parity suite, then bench A/B
# against the replica-per-wave kernel on configs 2 and 4.  Stops at the first failure.
#   usage: tools/r3_serial.sh <tag> [pytest files]
set -o pipefail
TAG=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
TESTS=${*:-tests/test_parity_gpu.py tests/test_gtraces.py tests/test_compaction_gpu.py}
PAXISIM_SERIAL=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu $TESTS > "$OUT/pytest_serial.log" 2>&1
rc=$?; tail -n 3 "$OUT/pytest_serial.log"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" "$OUT/pytest_serial.log" | head -20; exit $rc; }
for c in ${CONFIGS:-2 4}; do
  bash tools/ab_env.sh "$TAG/c$c" "par|PAXISIM_SERIAL=0" "ser|PAXISIM_SERIAL=1" -- --config $c --no-shard-check ${BENCH_ARGS:-} || exit 1
done
