#!/bin/bash
# Round-6 GPU call G2: config 5's window and instance layout (W=16 packed table, the default; W=8
# packed; W=8 co-located blocks) and config 4's window (16, 8) in mirrored A/Bs; idle-skip / dirty-row
# A/Bs (product against var/v_base.so) on configs 2, 5 and 3; config 5's traffic on var/v_base.so.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r6g2; mkdir -p $O
. tools/r6/step.sh
export TMPDIR=/tmp
REPS=2 step ab_c5w 600 tools/ab_env.sh r6g2/ab_c5w "w16|X=1" "w8|BENCH_ARGS=--window 8" "w8coloc|PAXISIM_WCOLOC=1 BENCH_ARGS=--window 8" -- --config 5 --no-shard-check
REPS=2 step ab_c4w 400 tools/ab_env.sh r6g2/ab_c4w "w16|X=1" "w8|BENCH_ARGS=--window 8" -- --config 4 --no-shard-check
for c in 2 5 3; do
  REPS=2 step ab_c$c 400 tools/ab_env.sh r6g2/ab_c$c "prod|X=1" "base|PAXISIM_LIB=var/v_base.so" -- --config $c --no-shard-check
done
step traffic5_base 300 env PAXISIM_LIB=$PWD/var/v_base.so bash tools/traffic.sh 5 --steps 4 --warmup 5
mv gpurun_out/traffic/traffic_config5.json $O/traffic_config5_base.json
