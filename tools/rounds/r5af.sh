#!/bin/bash
# Round-5 GPU call AF: batched pair swap in compaction (PXS_SWAP_BATCH=8): the compaction and parity
# suites, then mirrored A/Bs against the per-array swap (var/v_swap0.so) on configs 2 and 4.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5af
mkdir -p $O
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -4 "$O/$n.log" | cut -c1-300
  case $rc in 0) return 0 ;; *) echo "stopping after $n"; exit $rc ;; esac
}
step pytest 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_compaction_gpu.py tests/test_parity_gpu.py tests/test_pipeline_gpu.py tests/test_parity_scale_gpu.py
REPS=2 step ab_c2 600 tools/ab_env.sh r5af/ab_c2 "batch|X=1" "swap0|PAXISIM_LIB=var/v_swap0.so" -- --config 2 --no-shard-check
REPS=2 step ab_c4 600 tools/ab_env.sh r5af/ab_c4 "batch|X=1" "swap0|PAXISIM_LIB=var/v_swap0.so" -- --config 4 --no-shard-check
