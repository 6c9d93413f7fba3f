#!/bin/bash
# Round-6 GPU call N: LLVM scheduling strategies for the headline unit (k_paxos5s), mirrored A/B on config 2.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r6n; mkdir -p $O
. tools/r6/step.sh
REPS=2 step sched_c2 600 tools/ab_env.sh r6n/sched_c2 "prod|X=1" "ilp|PAXISIM_LIB=var/v_ilp.so" "mclause|PAXISIM_LIB=var/v_mclause.so" "bias0|PAXISIM_LIB=var/v_bias0.so" "relaxed|PAXISIM_LIB=var/v_relaxed.so" -- --config 2 --no-shard-check
