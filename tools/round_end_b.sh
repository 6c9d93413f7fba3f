#!/bin/bash
# Round-end pass B on the GPU box: the config-2 bench line (with its CPU
# baseline), its rocprofv3 kernel trace + stats and the timed-dispatch check,
# configs 1 and 3-5 lines (and config 4's Grid variant).   Usage: tools/round_end_b.sh <tag>
set -o pipefail
TAG=$1
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 500 python bench.py > "$OUT/bench_config2.json" 2> "$OUT/bench_config2.err" || { echo "bench failed"; tail -5 "$OUT/bench_config2.err"; exit 1; }
head -c 400 "$OUT/bench_config2.json"; echo
export TMPDIR=/tmp
( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline --no-shard-check > "$OUT/prof.log" 2>&1 ) || { echo "rocprof failed"; tail -5 "$OUT/prof.log"; exit 1; }
python3 tools/prof_timed.py "$(find "$OUT/prof" -name '*kernel_trace.csv' | head -n1)" 0 "$OUT/bench_config2.json" > "$OUT/prof_timed.json" && cat "$OUT/prof_timed.json"
timeout -k 10 300 python bench.py --config 1 --warmup 0 --steps 1 > "$OUT/bench_config1.json" 2> "$OUT/bench_config1.err" || { echo "config 1 failed"; tail -5 "$OUT/bench_config1.err"; exit 1; }
head -c 300 "$OUT/bench_config1.json"; echo
for c in 3 4 5; do
  timeout -k 10 500 python bench.py --config $c > "$OUT/bench_config$c.json" 2> "$OUT/bench_config$c.err" || { echo "config $c failed"; tail -5 "$OUT/bench_config$c.err"; exit 1; }
  head -c 300 "$OUT/bench_config$c.json"; echo
done
timeout -k 10 500 python bench.py --config 4 --fz 0 > "$OUT/bench_config4_fz0.json" 2> "$OUT/bench_config4_fz0.err" || { echo "config 4 fz0 failed"; tail -5 "$OUT/bench_config4_fz0.err"; exit 1; }
head -c 300 "$OUT/bench_config4_fz0.json"; echo
# per-handler stamps need the PXS_STAMPS build (tools/stamps.py; not part of this pass)
echo done
