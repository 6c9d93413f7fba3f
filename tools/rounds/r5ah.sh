#!/bin/bash
# Round-5 GPU call AH: per-item duration, pipelined against unpipelined launches, on one box.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5ah
mkdir -p $O
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -2 "$O/$n.log" | cut -c1-300
  case $rc in 0) return 0 ;; *) echo "stopping after $n"; exit $rc ;; esac
}
export PAXISIM_WT_LIB=var/v_wavetimes_pipe.so
step c5_pipe 300 python tools/wave_times.py 5 20 3 0 4
step c5_off 300 env PAXISIM_PIPE=1 python tools/wave_times.py 5 20 6
step c5_pipe2 300 python tools/wave_times.py 5 20 3 0 4
step c4_off 300 env PAXISIM_PIPE=1 python tools/wave_times.py 4 21 6
step c4_pipe 300 python tools/wave_times.py 4 21 3 0 3
