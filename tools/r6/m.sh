#!/bin/bash
# Round-6 GPU call M: the library rebuilt from the final sources (4aaf19ef4e4b9881) after the rejected
# experiment: the GPU suite, smoke, and the default bench line (its build id must match the traffic
# record it attaches).
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r6m; mkdir -p $O
. tools/r6/step.sh
step pytest 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 400 python bench.py
