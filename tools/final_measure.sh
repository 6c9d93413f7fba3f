#!/bin/bash
# Round-end measurement on the GPU box: config-2 bench (with CPU baseline),
# its rocprofv3 kernel trace + stats, PMC HBM traffic, and configs 3-5 lines.
# Usage: tools/final_measure.sh <tag>          -> gpurun_out/<tag>/
set -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 500 python bench.py > "$OUT/bench_config2.json" 2> "$OUT/bench_config2.err" || { echo "bench failed"; tail -5 "$OUT/bench_config2.err"; exit 1; }
cat "$OUT/bench_config2.json"
export TMPDIR=/tmp
( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline > "$OUT/prof.log" 2>&1 ) || { echo "rocprof failed"; tail -5 "$OUT/prof.log"; exit 1; }
python3 tools/prof_timed.py "$(find "$OUT/prof" -name '*kernel_trace.csv' | head -n1)" 0 "$OUT/bench_config2.json" > "$OUT/prof_timed.json" && cat "$OUT/prof_timed.json"
bash tools/traffic.sh 2 || exit 1
for c in 3 4 5; do
  timeout -k 10 500 python bench.py --config $c > "$OUT/bench_config$c.json" 2> "$OUT/bench_config$c.err" || { echo "config $c failed"; tail -5 "$OUT/bench_config$c.err"; exit 1; }
  head -c 300 "$OUT/bench_config$c.json"; echo
done
