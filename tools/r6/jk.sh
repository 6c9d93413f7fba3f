#!/bin/bash
# Round-6 GPU calls J + K in one: config 5's access-class tally at its new default (window 8, co-located
# instance blocks, var/v_tally.so from the final sources), then bench.py's N>1 flow rehearsed with two
# ranks sharing the box's GPU (tools/dist_rehearsal.sh) on the final build.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r6j; mkdir -p $O gpurun_out/r6k
. tools/r6/step.sh
step tally5 300 env PAXISIM_LIB=var/v_tally.so python -u tools/tally.py 5 65536 $O/tally_config5_w8coloc.json
step dist 600 bash tools/dist_rehearsal.sh r6k/dist
