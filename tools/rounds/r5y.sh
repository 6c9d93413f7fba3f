#!/bin/bash
# Round-5 GPU call Y (final build, pipelined launches): every config's bench line, rocprofv3 trace of config 2, HBM traffic
# of every config's step kernel at its bench window, SQ/TCC counters of configs 2 and 5, and the checker's
# waves-per-workgroup A/B.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5y
mkdir -p $O
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -2 "$O/$n.log" | cut -c1-300
  case $rc in 0) return 0 ;; *) echo "stopping after $n"; exit $rc ;; esac
}
for c in 2 3 4 5; do step bench_config$c 400 python bench.py --config $c; done
step bench_config4_fz0 400 python bench.py --config 4 --fz 0
step bench_config1 300 python bench.py --config 1 --warmup 0 --steps 1
export TMPDIR=/tmp
step prof_c2 400 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- python bench.py --no-cpu-baseline --no-shard-check --config 2
step pytest 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
