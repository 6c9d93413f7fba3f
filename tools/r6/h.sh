#!/bin/bash
# Round-6 GPU call H: the GPU suite on the build whose 5-replica Multi-Paxos unit runs persistent
# pipelined waves, and mirrored A/Bs of the persistent form in the 9-replica Paxos, WPaxos and ABD
# units (var/v_persist_all.so) on configs 4, 5 and 3.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r6h; mkdir -p $O
. tools/r6/step.sh
step pytest 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu
for c in 4 5 3; do
  REPS=2 step abp_c$c 500 tools/ab_env.sh r6h/abp_c$c "prod|X=1" "persist|PAXISIM_LIB=var/v_persist_all.so" -- --config $c --no-shard-check
done
