#!/bin/bash
# Rehearse bench.py's N>1 flow (sharding, barrier, all-reduce, max-over-ranks
# timing) with 2 ranks sharing the one GPU of a gpurun box: RCCL refuses two
# ranks on one device, so the stats all-reduce runs over gloo here.
# Usage: tools/dist_rehearsal.sh <tag>
set -o pipefail
TAG=${1:-dist}
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
PAXISIM_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 4 --warmup 1 --clusters 262144 \
  > "$OUT/bench2.json" 2> "$OUT/bench2.err" || { echo "2-rank bench failed rc=$?"; tail -20 "$OUT/bench2.err"; exit 1; }
cat "$OUT/bench2.json"
timeout -k 10 300 python bench.py --steps 4 --warmup 1 --clusters 524288 --no-cpu-baseline > "$OUT/bench1.json" 2> "$OUT/bench1.err" \
  || { echo "1-rank bench failed rc=$?"; tail -20 "$OUT/bench1.err"; exit 1; }
cat "$OUT/bench1.json"
