#!/bin/bash
# Round-6 GPU call C: access-class tallies of configs 5 and 2 (var/v_tally.so) and the HBM traffic of
# config 5 on the product (its var/v_base.so pass failed on a relative library path: call D).
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r6c; mkdir -p $O
. tools/r6/step.sh
export TMPDIR=/tmp
step tally5 300 env PAXISIM_LIB=var/v_tally.so python -u tools/tally.py 5 65536 $O/tally_config5.json
step tally2 300 env PAXISIM_LIB=var/v_tally.so python -u tools/tally.py 2 262144 $O/tally_config2.json
step traffic5 300 bash tools/traffic.sh 5 --steps 4 --warmup 5
mv gpurun_out/traffic/traffic_config5.json $O/traffic_config5_product.json
