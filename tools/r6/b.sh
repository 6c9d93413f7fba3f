#!/bin/bash
# Round-6 GPU call B: the GPU suite on the build with idle replica-steps skipped and dirty-only row
# stores (sim_core.h PXS_SKIP_IDLE / PXS_ROW_DIRTY); the miscompile reproducer's first divergence (the
# ISA predicts slot = 20, the last fault record's step_from); access-class tallies of configs 5 and 2;
# HBM traffic of config 5 on both builds; mirrored A/Bs (product vs var/v_base.so, both flags off) on
# configs 5, 2, 3, 4, and the persistent pipelined form (var/v_persist.so) on configs 2 and 5.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r6b; mkdir -p $O
. tools/r6/step.sh
export TMPDIR=/tmp
step pytest 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu
soft diverge_guard 300 env PAXISIM_LIB=paxi_amd/guard/libpaxisim_absorb.so python -u tools/diverge.py wp_crash 1
step tally5 300 env PAXISIM_LIB=var/v_tally.so python -u tools/tally.py 5 65536 $O/tally_config5.json
step tally2 300 env PAXISIM_LIB=var/v_tally.so python -u tools/tally.py 2 262144 $O/tally_config2.json
step traffic5 400 bash tools/traffic.sh 5 --steps 4 --warmup 5
mv gpurun_out/traffic/traffic_config5.json $O/traffic_config5_product.json
step traffic5_base 400 env PAXISIM_LIB=var/v_base.so bash tools/traffic.sh 5 --steps 4 --warmup 5
mv gpurun_out/traffic/traffic_config5.json $O/traffic_config5_base.json
for c in 5 2 3 4; do
  REPS=2 step ab_c$c 900 tools/ab_env.sh r6b/ab_c$c "prod|X=1" "base|PAXISIM_LIB=var/v_base.so" -- --config $c --no-shard-check
done
for c in 2 5; do
  REPS=2 step abp_c$c 900 tools/ab_env.sh r6b/abp_c$c "prod|X=1" "persist|PAXISIM_LIB=var/v_persist.so" -- --config $c --no-shard-check
done
