#!/bin/bash
# Round-5 GPU call AB: config 2 in 20-step chunks (bench.py LAUNCH_DEFAULT): HBM traffic, bench line,
# rocprofv3 trace.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5ab
mkdir -p $O
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -2 "$O/$n.log" | cut -c1-300
  case $rc in 0) return 0 ;; *) echo "stopping after $n"; exit $rc ;; esac
}
export TMPDIR=/tmp
step traffic2 400 bash tools/traffic.sh 2
mkdir -p profiles && cp gpurun_out/traffic/traffic_config2.json profiles/traffic_config2.json
step bench_config2 400 python bench.py --config 2
step prof_c2 400 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- python bench.py --no-cpu-baseline --no-shard-check --config 2
