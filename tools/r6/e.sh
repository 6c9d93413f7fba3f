#!/bin/bash
# Round-6 GPU call E: config 5 at windows 16 and 8 (speed, flags, per-type counts and shard digests,
# to see whether a smaller window is the same simulation), the idle-skip A/B on config 3 and the
# persistent form on config 5.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r6e; mkdir -p $O
. tools/r6/step.sh
for w in 16 8; do step c5_w$w 300 python bench.py --config 5 --no-cpu-baseline --window $w; done
REPS=2 step ab_c3 400 tools/ab_env.sh r6e/ab_c3 "prod|X=1" "base|PAXISIM_LIB=var/v_base.so" -- --config 3 --no-shard-check
REPS=2 step abp_c5 400 tools/ab_env.sh r6e/abp_c5 "prod|X=1" "persist|PAXISIM_LIB=var/v_persist.so" -- --config 5 --no-shard-check
