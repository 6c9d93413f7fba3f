#!/bin/bash
# GPU box, round 3: the GPU parity suite, smoke, every config's bench line,
# the config-2 rocprofv3 kernel trace + stats with the timed-dispatch check.
# Any failure, timeout or signal ends the script.
#   usage: tools/r3_measure.sh <tag> [configs (default "2 1 3 4 5")]
set -o pipefail
TAG=$1
CONFIGS=${2:-"2 1 3 4 5"}
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
stop() { echo "STOP at $1 rc=$2"; exit "$2"; }
if [ -z "${NO_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; tail -n 1 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || { tail -n 40 "$OUT/pytest_gpu.log"; stop pytest $rc; }
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  rc=$?; tail -n 1 "$OUT/smoke.log"; [ $rc -eq 0 ] || stop smoke $rc
fi
for c in $CONFIGS; do
  args="--config $c"
  [ "$c" = 1 ] && args="--config 1 --warmup 0 --steps 1"
  timeout -k 10 600 python -u bench.py $args ${BENCH_ARGS:-} > "$OUT/bench_config$c.json" 2> "$OUT/bench_config$c.err"
  rc=$?; echo "bench c$c rc=$rc"; head -c 300 "$OUT/bench_config$c.json"; echo
  [ $rc -eq 0 ] || { tail -n 5 "$OUT/bench_config$c.err"; stop "bench c$c" $rc; }
done
if [ -z "${NO_PROF:-}" ]; then
  export TMPDIR=/tmp
  ( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline --no-shard-check > "$OUT/prof.log" 2>&1 )
  rc=$?; [ $rc -eq 0 ] || { tail -n 5 "$OUT/prof.log"; stop rocprof $rc; }
  python3 tools/prof_timed.py "$(find "$OUT/prof" -name '*kernel_trace.csv' | head -n1)" 0 "$OUT/bench_config2.json" > "$OUT/prof_timed.json" && cat "$OUT/prof_timed.json"
fi
echo done
