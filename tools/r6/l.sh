#!/bin/bash
# Round-6 GPU call L: the GPU suite with the WPaxos Database values kept in the co-located instance
# blocks (P.wkv), and a mirrored config-5 A/B against the same build with them in kv_val (PAXISIM_WKV=0).
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r6l; mkdir -p $O
. tools/r6/step.sh
step pytest 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu
REPS=2 step ab_c5_wkv 500 tools/ab_env.sh r6l/ab_c5_wkv "wkv|X=1" "kvval|PAXISIM_WKV=0" -- --config 5 --no-shard-check
