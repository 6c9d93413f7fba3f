#!/bin/bash
# One iteration on the GPU box: parity tests, then bench lines for the given
# configs and (optionally) the stamps breakdown.  Usage: tools/iter.sh <tag> "<configs>" [stamps-config]
set -o pipefail
TAG=$1; CFGS=$2; ST=$3
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for c in $CFGS; do
  timeout -k 10 400 python bench.py --config $c --no-cpu-baseline > "$OUT/bench_c$c.json" 2> "$OUT/bench_c$c.err" || { echo "bench $c failed"; tail -5 "$OUT/bench_c$c.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_c$c.json')); print('config $c', '%.4e'%d['value'], 'launch ms', round(d['roofline']['avg_launch_ms'],2), 'frac', round(d['roofline']['frac'],4), 'unfaithful', d['unfaithful_clusters'])"
done
if [ -n "$ST" ]; then
  timeout -k 10 300 python tools/stamps.py 65536 1000 300 $ST > "$OUT/stamps$ST.txt" 2>&1 && tail -16 "$OUT/stamps$ST.txt"
fi
