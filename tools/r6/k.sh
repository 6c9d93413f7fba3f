#!/bin/bash
# Round-6 GPU call K: bench.py's N>1 flow rehearsed with two ranks sharing the box's GPU (gloo
# statistics; tools/dist_rehearsal.sh) on the final build, whose Multi-Paxos kernels run persistent waves.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r6k; mkdir -p $O
. tools/r6/step.sh
step dist 600 bash tools/dist_rehearsal.sh r6k/dist
