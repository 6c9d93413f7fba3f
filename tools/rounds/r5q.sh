#!/bin/bash
# Round-5 GPU call Q: lane-major mailbox records (PXS_REC_LANE_MAJOR=1, the tree) - the GPU suite
# (the miscompile guard's pinned unit predates the layout and is deselected), then mirrored A/Bs
# against the lane-minor build (var/v_recminor.so) on configs 2, 5, 4 and 3.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5q
mkdir -p $O
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -3 "$O/$n.log" | cut -c1-300
  case $rc in 0) return 0 ;; *) echo "stopping after $n"; exit $rc ;; esac
}
step pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --deselect tests/test_miscompile_guard_gpu.py
for c in 2 5 4 3; do
  REPS=2 step ab_c$c 600 tools/ab_env.sh r5q/ab_c$c "major|X=1" "minor|PAXISIM_LIB=var/v_recminor.so" -- --config $c --no-shard-check
done
