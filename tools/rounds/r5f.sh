#!/bin/bash
# Round-5 GPU call F: GPU suite on the link-late build; the two-mode probe; balanced A/Bs (REPS even:
# every variant sits at as many odd as even positions, so strict run-to-run alternation cancels).
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5f
mkdir -p $O
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -5 "$O/$n.log"
  case $rc in 0|1) return 0 ;; *) echo "stopping after $n"; exit $rc ;; esac
}
step pytest_product 400 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/
step mode_c3 300 python -u tools/mode_probe.py 3 6
step mode_c2 300 python -u tools/mode_probe.py 2 3
REPS=4 step ab_c2_link 1100 tools/ab_env.sh r5f/ab_c2_link "late|X=1" "early|PAXISIM_LIB=var/v_linkearly.so" -- --config 2
REPS=2 step ab_c2_launch 600 tools/ab_env.sh r5f/ab_c2_launch "l50|X=1" "l25|PAXISIM_LAUNCH_STEPS=25" -- --config 2
