#!/bin/bash
# Round-5 GPU call AK: the tree as committed (build 2acd10e7) - GPU suite, smoke, headline bench line.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5ak
mkdir -p $O
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -2 "$O/$n.log" | cut -c1-300
  case $rc in 0) return 0 ;; *) echo "stopping after $n"; exit $rc ;; esac
}
step pytest 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_config2 400 python bench.py
