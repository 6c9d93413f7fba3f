#!/bin/bash
# Round-5 GPU call S: pipelined serial launches (sim_core.h sim_serial_pipe).  The GPU suite with
# PAXISIM_PIPE=4 (persistent waves), the parity suites with the one-ticket-per-workgroup build
# (var/v_pipe1.so), then mirrored A/Bs on configs 5 and 4 (no compaction: chunks fuse freely).
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5s
mkdir -p $O
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -3 "$O/$n.log" | cut -c1-300
  case $rc in 0) return 0 ;; *) echo "stopping after $n"; exit $rc ;; esac
}
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
step pytest_pipe4 900 env PAXISIM_PIPE=4 $T tests -m gpu
step pytest_pipe1lib 600 env PAXISIM_PIPE=4 PAXISIM_LIB=var/v_pipe1.so $T -m gpu tests/test_parity_gpu.py tests/test_parity_wpaxos_gpu.py tests/test_compaction_gpu.py tests/test_parity_abd_gpu.py
for c in 5 4; do
  REPS=2 step ab_c$c 600 tools/ab_env.sh r5s/ab_c$c "base|X=1" "p4|PAXISIM_PIPE=4" "p4np|PAXISIM_PIPE=4 PAXISIM_LIB=var/v_pipe1.so" -- --config $c --no-shard-check
done
