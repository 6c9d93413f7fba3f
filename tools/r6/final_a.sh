#!/bin/bash
# Round-6 final build, call 1 of 2: the GPU suite, smoke, and the HBM traffic of every config's step
# kernel at its default bench window (tools/traffic.sh: FETCH_SIZE / WRITE_SIZE passes).  The traffic
# records go into profiles/ before call 2's bench lines, which attach them by build id.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r6fa3; mkdir -p $O
. tools/r6/step.sh
export TMPDIR=/tmp
step pytest 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step traffic2 400 bash tools/traffic.sh 2
step traffic3 300 bash tools/traffic.sh 3
step traffic4 300 bash tools/traffic.sh 4
step traffic4_fz0 300 bash tools/traffic.sh 4 --fz 0
step traffic5 400 bash tools/traffic.sh 5
# ABD with idle-skip but without the dirty rows (var/v_abdnodirty.so), mirrored, for the record
REPS=2 step abd_c3 500 tools/ab_env.sh r6fa3/abd_c3 "prod|X=1" "nodirty|PAXISIM_LIB=var/v_abdnodirty.so" -- --config 3 --no-shard-check
