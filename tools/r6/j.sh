#!/bin/bash
# Round-6 GPU call J: config 5's access-class tally at its new default (window 8, co-located instance
# blocks), on var/v_tally.so built from the final sources.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r6j; mkdir -p $O
. tools/r6/step.sh
step tally5 300 env PAXISIM_LIB=var/v_tally.so python -u tools/tally.py 5 65536 $O/tally_config5_w8coloc.json
