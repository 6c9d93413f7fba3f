#!/bin/bash
# Round-6 GPU call O: idle replica-steps skipped in the 9-replica Multi-Paxos kernel (config 4 has no
# random fault process, and 41% of its wave-level replica-steps are idle on the oracle), alone and with
# dirty-only row stores, mirrored A/B on config 4 (and --fz 0).
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r6o; mkdir -p $O
. tools/r6/step.sh
REPS=2 step skip_c4 600 tools/ab_env.sh r6o/skip_c4 "prod|X=1" "skip|PAXISIM_LIB=var/v_skip9.so" "skipdirty|PAXISIM_LIB=var/v_skipdirty9.so" -- --config 4 --no-shard-check
step parity_skip 600 env PAXISIM_LIB=var/v_skipdirty9.so python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_parity_gpu.py tests/test_gtraces.py tests/test_parity_scale_gpu.py -m gpu
