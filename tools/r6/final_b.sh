#!/bin/bash
# Round-6 final build, call 2 of 2: every config's bench line (CPU baseline and sampled parity on), the
# rocprofv3 kernel trace + stats of config 2's bench run, and the SQ / TCC counter sets of configs 2 and 5.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r6fb3; mkdir -p $O
. tools/r6/step.sh
export TMPDIR=/tmp
for c in 2 3 4 5; do step bench_config$c 400 python bench.py --config $c; done
step bench_config4_fz0 400 python bench.py --config 4 --fz 0
step bench_config1 300 python bench.py --config 1 --warmup 0 --steps 1
step prof_c2 400 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- python bench.py --no-cpu-baseline --no-shard-check --config 2
P1="SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVES SQ_WAVE_CYCLES"
P3="TCC_HIT_sum TCC_MISS_sum"
step pmc_c2 400 bash tools/pmc2.sh r6fb3_c2 "$P1" "$P3" -- --config 2 --warmup 5 --steps 1
step pmc_c5 400 bash tools/pmc2.sh r6fb3_c5 "$P1" "$P3" -- --config 5 --warmup 5 --steps 1
