#!/bin/bash
# GPU box: bench.py's N>1 flow with 2 ranks on the one GPU (stats over gloo:
# RCCL refuses two ranks on one device), then the 1-rank run of the same
# per-GPU workload: rank 1's state digest must equal the 1-rank line's virtual
# rank-1 digest (sharding invariance).   usage: tools/r3_dist.sh <tag>
set -o pipefail
TAG=${1:-dist}
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
A="--steps 2 --warmup 1 --clusters 65536 --no-cpu-baseline"
PAXISIM_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 $A > "$OUT/bench2.json" 2> "$OUT/bench2.err" \
  || { echo "2-rank bench failed rc=$?"; tail -20 "$OUT/bench2.err"; exit 1; }
timeout -k 10 300 python bench.py $A > "$OUT/bench1.json" 2> "$OUT/bench1.err" || { echo "1-rank bench failed rc=$?"; tail -20 "$OUT/bench1.err"; exit 1; }
python3 - "$OUT" <<'PY'
import json, sys
d2 = json.loads(open(sys.argv[1] + "/bench2.json").read().strip().splitlines()[-1])
d1 = json.loads(open(sys.argv[1] + "/bench1.json").read().strip().splitlines()[-1])
g2, g1 = d2["shard_digests"]["digests"], d1["shard_digests"]["digests"]
print("2 ranks:", d2["n_gpus"], "%.4g" % d2["value"], g2)
print("1 rank :", "%.4g" % d1["value"], {k: g1[k] for k in ("0", "1")})
ok = g2["0"] == g1["0"] and g2["1"] == g1["1"]
print("sharding-invariant:", ok)
sys.exit(0 if ok else 1)
PY
