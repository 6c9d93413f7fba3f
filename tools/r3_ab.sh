#!/bin/bash
# GPU box: the default library through the given GPU tests, then bench A/B of
# library variants on the given configs (variants: name=path, "def" = default).
#   usage: tools/r3_ab.sh <tag> "<configs>" "<pytest files or ->" name=lib ...
set -o pipefail
TAG=$1; CONFIGS=$2; TESTS=$3; shift 3
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
if [ "$TESTS" != "-" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu $TESTS > "$OUT/pytest.log" 2>&1
  rc=$?; tail -n 2 "$OUT/pytest.log"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" "$OUT/pytest.log" | head -20; exit $rc; }
fi
V=()
for a in "$@"; do n=${a%%=*}; l=${a#*=}; [ "$l" = def ] && V+=("$n|PAXISIM_X=0") || V+=("$n|PAXISIM_LIB=$l"); done
for c in $CONFIGS; do
  bash tools/ab_env.sh "$TAG/c$c" "${V[@]}" -- --config $c --no-shard-check ${BENCH_ARGS:-} || exit 1
done
