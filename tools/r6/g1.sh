#!/bin/bash
# Round-6 GPU call G1: the GPU suite on the build with the co-located WPaxos instance blocks
# (PAXISIM_WCOLOC, a run-time layout option) under test; config 5's HBM traffic with the co-located
# blocks at windows 16 and 8; mirrored A/B of config 5: packed table (default) against co-located
# blocks, at window 16, and config 5 at window 8 (co-located) beside window 16 with shard digests.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r6g1; mkdir -p $O
. tools/r6/step.sh
export TMPDIR=/tmp
step pytest 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu
step traffic5_coloc 300 env PAXISIM_WCOLOC=1 bash tools/traffic.sh 5 --steps 4 --warmup 5
mv gpurun_out/traffic/traffic_config5.json $O/traffic_config5_coloc.json
step traffic5_coloc_w8 300 env PAXISIM_WCOLOC=1 bash tools/traffic.sh 5 --steps 4 --warmup 5 --window 8
mv gpurun_out/traffic/traffic_config5.json $O/traffic_config5_coloc_w8.json
REPS=2 step ab_c5_coloc 500 tools/ab_env.sh r6g1/ab_c5_coloc "packed|X=1" "coloc|PAXISIM_WCOLOC=1" -- --config 5 --no-shard-check
step c5_w16 200 python bench.py --config 5 --no-cpu-baseline
step c5_w8_coloc 200 env PAXISIM_WCOLOC=1 python bench.py --config 5 --no-cpu-baseline --window 8
