#!/bin/bash
# Round-5 GPU call I: lane-asynchronous replica progress for WPaxos (PXS_LANE_ASYNC, batch sizes):
# parity of the WPaxos suites on it, then config-5 A/B against the product (mirrored, REPS=2).
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5i
mkdir -p $O
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -4 "$O/$n.log" | cut -c1-300
  case $rc in 0|1) return 0 ;; *) echo "stopping after $n"; exit $rc ;; esac
}
step pytest_async16 400 env PAXISIM_LIB=var/v_async16.so python -u -m pytest -q -x --timeout 120 --timeout-method thread -m gpu \
  tests/test_parity_wpaxos_gpu.py tests/test_parity_scale_gpu.py tests/test_database.py tests/test_reply_value.py tests/test_workload_gpu.py
REPS=2 step ab_c5 1100 tools/ab_env.sh r5i/ab_c5 "prod|X=1" "a4|PAXISIM_LIB=var/v_async4.so" "a16|PAXISIM_LIB=var/v_async16.so" \
  "a32|PAXISIM_LIB=var/v_async32.so" "a64|PAXISIM_LIB=var/v_async64.so" -- --config 5
