#!/bin/bash
# Round-5 GPU call R: how well a launch fills the GPU (tools/wave_times.py, PXS_WAVE_TIMES build):
# per-wave start/end clocks of configs 2, 5, 4 and 3 in their bench windows.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5r
mkdir -p $O
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -4 "$O/$n.log" | cut -c1-400
  case $rc in 0) return 0 ;; *) echo "stopping after $n"; exit $rc ;; esac
}
step wt_c2 300 python tools/wave_times.py 2 40 6
step wt_c2b 300 python tools/wave_times.py 2 150 4
step wt_c5 300 python tools/wave_times.py 5 20 8
step wt_c4 300 python tools/wave_times.py 4 20 8

