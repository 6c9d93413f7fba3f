#!/bin/bash
# Round-6 GPU call D: HBM traffic of config 5 on var/v_base.so (idle-skip and dirty rows off), mirrored
# A/Bs of the product against it on configs 5, 2, 3 and 4, and the persistent pipelined form
# (var/v_persist.so) on configs 2 and 5.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r6d; mkdir -p $O
. tools/r6/step.sh
export TMPDIR=/tmp
step traffic5_base 300 env PAXISIM_LIB=$PWD/var/v_base.so bash tools/traffic.sh 5 --steps 4 --warmup 5
mv gpurun_out/traffic/traffic_config5.json $O/traffic_config5_base.json
REPS=2 step ab_c5 500 tools/ab_env.sh r6d/ab_c5 "prod|X=1" "base|PAXISIM_LIB=var/v_base.so" -- --config 5 --no-shard-check
REPS=2 step ab_c2 500 tools/ab_env.sh r6d/ab_c2 "prod|X=1" "base|PAXISIM_LIB=var/v_base.so" -- --config 2 --no-shard-check
REPS=2 step abp_c2 400 tools/ab_env.sh r6d/abp_c2 "prod|X=1" "persist|PAXISIM_LIB=var/v_persist.so" -- --config 2 --no-shard-check
REPS=2 step ab_c4 300 tools/ab_env.sh r6d/ab_c4 "prod|X=1" "base|PAXISIM_LIB=var/v_base.so" -- --config 4 --no-shard-check
