#!/bin/bash
# Round-5 GPU call D: the SDWA-peephole-free build (parity + cost), the miscompile guard on the
# product, and mirrored-order A/Bs (REPS=3) of product / no-SDWA / round 4 / Reply routing.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5d
mkdir -p $O
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -4 "$O/$n.log"
  case $rc in 0|1) return 0 ;; *) echo "stopping after $n"; exit $rc ;; esac
}
step guard 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_miscompile_guard_gpu.py
step pytest_nosdwa 400 env PAXISIM_LIB=var/libpaxisim_nosdwa.so python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/
export REPS=3
step ab_c5 1000 tools/ab_env.sh r5d/ab_c5 "prod|X=1" "nosdwa|PAXISIM_LIB=var/libpaxisim_nosdwa.so" "reply1|PAXISIM_LIB=var/libpaxisim_reply1.so" -- --config 5
step ab_c2 1000 tools/ab_env.sh r5d/ab_c2 "prod|X=1" "nosdwa|PAXISIM_LIB=var/libpaxisim_nosdwa.so" "r4|PAXISIM_LIB=var/libpaxisim_r4.so" -- --config 2
step ab_c3 600 tools/ab_env.sh r5d/ab_c3 "prod|X=1" "nosdwa|PAXISIM_LIB=var/libpaxisim_nosdwa.so" "r4|PAXISIM_LIB=var/libpaxisim_r4.so" -- --config 3
