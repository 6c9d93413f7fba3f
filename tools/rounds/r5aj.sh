#!/bin/bash
# Round-5 GPU call AJ: tickets by tile group (sim_core.h sim_serial_pipe, q[9]): the pipeline and
# parity-at-scale suites (default groups, and groups of one tile), then mirrored A/Bs against one
# group of all tiles (PAXISIM_PIPE_GROUP=0, the previous order).
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5aj
mkdir -p $O
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -3 "$O/$n.log" | cut -c1-300
  case $rc in 0) return 0 ;; *) echo "stopping after $n"; exit $rc ;; esac
}
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu"
step pytest 600 $T tests/test_pipeline_gpu.py tests/test_parity_scale_gpu.py tests/test_compaction_gpu.py
step pytest_g1 600 env PAXISIM_PIPE_GROUP=1 $T tests/test_pipeline_gpu.py tests/test_parity_wpaxos_gpu.py
for c in 5 2 3 4; do
  REPS=2 step ab_c$c 600 tools/ab_env.sh r5aj/ab_c$c "group|X=1" "flat|PAXISIM_PIPE_GROUP=0" -- --config $c --no-shard-check
done
