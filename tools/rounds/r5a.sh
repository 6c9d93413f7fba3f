#!/bin/bash
# Round-5 GPU call A: the r4l WPaxos absorb reproduction and the first A/Bs.
#  1. tools/diverge.py wp_crash on the r4l reconstruction (PXS_WP_ABSORB=1)
#  2. WPaxos parity suites on the fixed absorb (PXS_WP_ABSORB=2)
#  3. the full GPU suite on the product library
#  4. same-box A/Bs: config 5 product vs absorb=2; config 2 product vs round-4 (r4 sources)
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5a
mkdir -p $O
step() {   # step <name> <timeout> <cmd...>: stop the call on a fault, abort or time limit
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"
  tail -3 "$O/$n.log"
  case $rc in 0|1) return 0 ;; *) echo "stopping after $n"; exit $rc ;; esac
}
step diverge_wpabs1 300 env PAXISIM_LIB=var/libpaxisim_wpabs1.so python -u tools/diverge.py wp_crash 1
step pytest_wpabs2 400 env PAXISIM_LIB=var/libpaxisim_wpabs2.so python -u -m pytest -x -q --timeout 120 \
  --timeout-method thread -m gpu tests/test_parity_wpaxos_gpu.py tests/test_parity_scale_gpu.py \
  tests/test_database.py tests/test_reply_value.py tests/test_m2paxos_kpaxos.py tests/test_workload_gpu.py
step pytest_product 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/
step ab_c5 900 tools/ab_env.sh r5a/ab_c5 "prod1|X=1" "abs2a|PAXISIM_LIB=var/libpaxisim_wpabs2.so" "prod2|X=1" \
  "abs2b|PAXISIM_LIB=var/libpaxisim_wpabs2.so" -- --config 5
step ab_c2 900 tools/ab_env.sh r5a/ab_c2 "prod1|X=1" "r4a|PAXISIM_LIB=var/libpaxisim_r4.so" "prod2|X=1" \
  "r4b|PAXISIM_LIB=var/libpaxisim_r4.so" -- --config 2
step ab_c3 900 tools/ab_env.sh r5a/ab_c3 "prod1|X=1" "r4a|PAXISIM_LIB=var/libpaxisim_r4.so" "prod2|X=1" \
  "r4b|PAXISIM_LIB=var/libpaxisim_r4.so" -- --config 3
