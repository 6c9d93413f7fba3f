#!/bin/bash
# Round-5 GPU call L: does a one-exit send_begin (PXS_SEND_ONE_EXIT) remove the miscompile from the two
# reproducers (the pinned absorb unit, the batched lane-async unit)?
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5l
mkdir -p $O
for lib in var/v_absorb242_oneexit.so var/v_async16_oneexit.so var/v_async16.so; do
  L=$(basename $lib .so)
  timeout -k 10 120 env PAXISIM_LIB=$lib python tools/sink_guard.py wp_crash > $O/$L.json 2> $O/$L.err
  rc=$?; echo "$L rc=$rc $(tail -c 150 $O/$L.json)"
  case $rc in 0|1) ;; *) echo "stopping after $L"; exit $rc ;; esac
done
timeout -k 10 400 env PAXISIM_LIB=var/v_async16_oneexit.so python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_parity_wpaxos_gpu.py tests/test_parity_scale_gpu.py tests/test_database.py tests/test_reply_value.py tests/test_workload_gpu.py > $O/pytest_async16_oneexit.log 2>&1
echo "pytest rc=$?"; tail -3 $O/pytest_async16_oneexit.log
