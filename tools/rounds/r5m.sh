#!/bin/bash
# Round-5 GPU call M: the one-exit send_begin build - GPU suite (with the three guard variants), smoke,
# and balanced A/Bs against the previous product (var/v_prev.so).
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5m
mkdir -p $O
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -4 "$O/$n.log" | cut -c1-300
  case $rc in 0|1) return 0 ;; *) echo "stopping after $n"; exit $rc ;; esac
}
step pytest_gpu 500 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
export REPS=2
step ab_c2 900 tools/ab_env.sh r5m/ab_c2 "oneexit|X=1" "prev|PAXISIM_LIB=var/v_prev.so" -- --config 2
step ab_c5 900 tools/ab_env.sh r5m/ab_c5 "oneexit|X=1" "prev|PAXISIM_LIB=var/v_prev.so" -- --config 5
step ab_c4 900 tools/ab_env.sh r5m/ab_c4 "oneexit|X=1" "prev|PAXISIM_LIB=var/v_prev.so" -- --config 4
