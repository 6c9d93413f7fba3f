#!/bin/bash
# One GPU-box pass: parity tests, smoke, headline bench, rocprofv3 kernel stats.
# Usage: tools/gpu_check.sh <tag> [extra bench args]
set -o pipefail
TAG=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest failed rc=$?"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed rc=$?"; tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 400 python bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed rc=$?"; tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline "$@" > "$OUT/prof.log" 2>&1 || { echo "rocprof failed rc=$?"; tail -20 "$OUT/prof.log"; exit 1; }
find "$OUT/prof" -name '*kernel_stats.csv' -exec cat {} \;
python3 "$R/tools/prof_timed.py" "$(find "$OUT/prof" -name '*kernel_trace.csv' | head -n1)" 0 "$OUT/bench.json" > "$OUT/prof_timed.json" && cat "$OUT/prof_timed.json"
