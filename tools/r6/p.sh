#!/bin/bash
# Round-6 GPU call P: ABD (config 3) with idle replica-steps skipped but without the dirty-only row
# stores (var/v_abdnodirty.so), mirrored A/B against the product (both).
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r6p; mkdir -p $O
. tools/r6/step.sh
REPS=2 step abd_c3 600 tools/ab_env.sh r6p/abd_c3 "prod|X=1" "nodirty|PAXISIM_LIB=var/v_abdnodirty.so" -- --config 3 --no-shard-check
