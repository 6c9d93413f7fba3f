#!/bin/bash
# Round-6 GPU call I: config 2 re-tuned under persistent pipelined waves, mirrored: the absorb bound
# (PXS_ABSORB_MAX 1 / 3 against 2), 25-step chunks, compaction every 4 chunks.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r6i; mkdir -p $O
. tools/r6/step.sh
REPS=2 step tune_c2 900 tools/ab_env.sh r6i/tune_c2 "prod|X=1" "abs3|PAXISIM_LIB=var/v_abs3.so" "abs1|PAXISIM_LIB=var/v_abs1.so" "ls25|PAXISIM_LAUNCH_STEPS=25" "ce80|PAXISIM_COMPACT_EVERY=80" -- --config 2 --no-shard-check
