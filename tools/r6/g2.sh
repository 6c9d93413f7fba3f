#!/bin/bash
# Round-6 GPU call G2: idle-skip / dirty-row A/Bs (product against var/v_base.so) on configs 2, 3, 4, 5,
# the persistent pipelined form (var/v_persist.so) on configs 2 and 5, and config 5's traffic on
# var/v_base.so.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r6g2; mkdir -p $O
. tools/r6/step.sh
export TMPDIR=/tmp
step traffic5_base 300 env PAXISIM_LIB=$PWD/var/v_base.so bash tools/traffic.sh 5 --steps 4 --warmup 5
mv gpurun_out/traffic/traffic_config5.json $O/traffic_config5_base.json
for c in 2 5 3 4; do
  REPS=2 step ab_c$c 400 tools/ab_env.sh r6g2/ab_c$c "prod|X=1" "base|PAXISIM_LIB=var/v_base.so" -- --config $c --no-shard-check
done
REPS=2 step abp_c2 400 tools/ab_env.sh r6g2/abp_c2 "prod|X=1" "persist|PAXISIM_LIB=var/v_persist.so" -- --config 2 --no-shard-check
