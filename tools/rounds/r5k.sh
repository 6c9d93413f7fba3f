#!/bin/bash
# Round-5 GPU call K: the batched lane-async build failed the WPaxos crash/faults parity case (r5j):
# its first divergence, and the same source without the SDWA peephole on the WPaxos suites.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5k
mkdir -p $O
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -4 "$O/$n.log" | cut -c1-300
  case $rc in 0|1) return 0 ;; *) echo "stopping after $n"; exit $rc ;; esac
}
step diverge_async16 300 env PAXISIM_LIB=var/v_async16.so python -u tools/diverge.py wp_crash 1
step pytest_async16_nosdwa 400 env PAXISIM_LIB=var/v_async16_nosdwa.so python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_parity_wpaxos_gpu.py tests/test_parity_scale_gpu.py tests/test_database.py tests/test_reply_value.py tests/test_workload_gpu.py
