#!/bin/bash
# Round-5 GPU call AG: busy fraction of pipelined launches (tools/wave_times.py with a PXS_WAVE_TIMES
# build that records every (tile, chunk) item, var/v_wavetimes_pipe.so).
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5ag
mkdir -p $O
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -3 "$O/$n.log" | cut -c1-300
  case $rc in 0) return 0 ;; *) echo "stopping after $n"; exit $rc ;; esac
}
export PAXISIM_WT_LIB=var/v_wavetimes_pipe.so
step wt_c2 300 python tools/wave_times.py 2 99 6 0 3
step wt_c2b 300 python tools/wave_times.py 2 375 4 0 3
step wt_c5 300 python tools/wave_times.py 5 20 4 0 4
step wt_c4 300 python tools/wave_times.py 4 21 4 0 3
step wt_c3 300 python tools/wave_times.py 3 20 4 0 4
