#!/bin/bash
# Round-6 final build, call 3: rocprofv3 kernel traces + stats of configs 3, 4 and 5's bench runs (their
# timed step-kernel dispatches, to set beside the bench lines' HIP-event averages).
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r6fc; mkdir -p $O
. tools/r6/step.sh
export TMPDIR=/tmp
for c in 3 4 5; do
  step prof_c$c 400 rocprofv3 --kernel-trace --stats -d $O/prof_c$c -o run --output-format csv -- python bench.py --no-cpu-baseline --no-shard-check --config $c
done
