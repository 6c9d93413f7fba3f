#!/bin/bash
# Round-5 GPU call B:
#  1. pass bisection of the WPaxos absorb miscompile (tools/bisect_pass.sh variants, tools/sink_guard.py wp_crash)
#  2. first divergence of the PXS_WP_ABSORB=2 build (the r4l reconstruction)
#  3. the GPU suite on a build without -disable-machine-sink (var/libpaxisim_sink.so)
#  4. A/Bs: config 3 placement (product / drain-free, agrslot = round-4 ISA, r4), MachineSink on/off, loop alignment
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5b
mkdir -p $O
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -3 "$O/$n.log"
  case $rc in 0|1) return 0 ;; *) echo "stopping after $n"; exit $rc ;; esac
}
for lib in var/bisect_wpabs1_*.so; do
  L=$(basename $lib .so)
  timeout -k 10 120 env PAXISIM_LIB=$lib python tools/sink_guard.py wp_crash > $O/$L.json 2> $O/$L.err
  rc=$?; echo "$L rc=$rc $(tail -c 200 $O/$L.json)"
  case $rc in 0|1) ;; *) echo "stopping after $L"; exit $rc ;; esac
done
step diverge_wpabs2 300 env PAXISIM_LIB=var/libpaxisim_wpabs2.so python -u tools/diverge.py wp_crash 1
step pytest_sink 400 env PAXISIM_LIB=var/libpaxisim_sink.so python -u -m pytest -q --timeout 120 \
  --timeout-method thread -m gpu tests/
step ab_c3 900 tools/ab_env.sh r5b/ab_c3 "prod1|X=1" "slot1|PAXISIM_LIB=var/libpaxisim_agrslot.so" "r4a|PAXISIM_LIB=var/libpaxisim_r4.so" \
  "prod2|X=1" "slot2|PAXISIM_LIB=var/libpaxisim_agrslot.so" "al6|PAXISIM_LIB=var/libpaxisim_al6.so" "sink|PAXISIM_LIB=var/libpaxisim_sink.so" -- --config 3
step ab_c2 900 tools/ab_env.sh r5b/ab_c2 "prod1|X=1" "sink1|PAXISIM_LIB=var/libpaxisim_sink.so" "al6a|PAXISIM_LIB=var/libpaxisim_al6.so" \
  "prod2|X=1" "sink2|PAXISIM_LIB=var/libpaxisim_sink.so" "al6b|PAXISIM_LIB=var/libpaxisim_al6.so" -- --config 2
step ab_c5 900 tools/ab_env.sh r5b/ab_c5 "prod1|X=1" "sink1|PAXISIM_LIB=var/libpaxisim_sink.so" "al6a|PAXISIM_LIB=var/libpaxisim_al6.so" \
  "prod2|X=1" "sink2|PAXISIM_LIB=var/libpaxisim_sink.so" "al6b|PAXISIM_LIB=var/libpaxisim_al6.so" -- --config 5
step ab_c4 600 tools/ab_env.sh r5b/ab_c4 "prod1|X=1" "sink1|PAXISIM_LIB=var/libpaxisim_sink.so" -- --config 4
step linst 300 env PAXISIM_LIB=var/libpaxisim_linst.so python bench.py --no-cpu-baseline --no-shard-check --config 3
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1; echo "counters rc=$?"
