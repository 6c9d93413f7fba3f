#!/bin/bash
# Round-5 GPU call T: pipelined launches, small and timed (tools/pipe_probe.py).
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5t
mkdir -p $O
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -6 "$O/$n.log" | cut -c1-300
  case $rc in 0) return 0 ;; *) echo "stopping after $n"; exit $rc ;; esac
}
step off 120 env PAXISIM_PIPE=1 python -u tools/pipe_probe.py 256 4 40 10
step np4 60 env PAXISIM_PIPE=4 PAXISIM_LIB=var/v_pipe1.so python -u tools/pipe_probe.py 256 4 40 10
step p4 60 env PAXISIM_PIPE=4 python -u tools/pipe_probe.py 256 4 40 10
