#!/bin/bash
# Round-6 GPU call A: the copy-peak probe in the guide's shape, the pipeline suite (with the
# give-up readout test), the pipe probe on the shipped form, then the rebuilt persistent form
# (var/v_persist.so, PXS_PIPE_PERSIST=1) under a short spin limit so a stuck wait names itself.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r6a; mkdir -p $O
. tools/r6/step.sh
step copy_bw 120 tools/probe/copy_bw
step pytest_pipe 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_pipeline_gpu.py
step probe_ship 90 env PAXISIM_PIPE=4 python -u tools/pipe_probe.py 256 4 40 10
soft probe_persist 120 env PAXISIM_PIPE=4 PAXISIM_PIPE_SPIN=65536 PAXISIM_LIB=var/v_persist.so python -u tools/pipe_probe.py 256 4 40 10
soft probe_persist_big 120 env PAXISIM_PIPE=4 PAXISIM_PIPE_SPIN=65536 PAXISIM_LIB=var/v_persist.so python -u tools/pipe_probe.py 20000 4 40 10
soft pytest_persist 400 env PAXISIM_LIB=var/v_persist.so python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_pipeline_gpu.py -k paxos
step bench_c2 300 python bench.py --no-cpu-baseline
step bench_c2_w64 300 python bench.py --no-cpu-baseline --window 64
