#!/bin/bash
# Round-5 GPU call U: pipelined launches, one ticket per workgroup (sim_core.h sim_serial_pipe):
# the small timed probe, the GPU suite with PAXISIM_PIPE=4, then mirrored A/Bs on configs 5 and 4.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5u
mkdir -p $O
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -4 "$O/$n.log" | cut -c1-300
  case $rc in 0) return 0 ;; *) echo "stopping after $n"; exit $rc ;; esac
}
step p4 60 env PAXISIM_PIPE=4 python -u tools/pipe_probe.py 256 4 40 10
step p4big 120 env PAXISIM_PIPE=4 python -u tools/pipe_probe.py 20000 3 200 50
step pytest_pipe4 900 env PAXISIM_PIPE=4 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu
for c in 5 4; do
  REPS=2 step ab_c$c 600 tools/ab_env.sh r5u/ab_c$c "base|X=1" "p4|PAXISIM_PIPE=4" -- --config $c --no-shard-check
done
