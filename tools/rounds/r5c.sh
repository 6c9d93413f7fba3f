#!/bin/bash
# Round-5 GPU call C:
#  1. pass bisection refinement (limits 35003-35007) and pass-disable flags on the WPaxos absorb miscompile
#  2. linearizability scan vs the checker kernel's occupancy (PXS_LIN_MINW) and the MachineSink flag
#  3. rocprofv3 kernel stats of config 2 on the product (cmp_swap share); SQC instruction-cache counters
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5c
mkdir -p $O
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -3 "$O/$n.log"
  case $rc in 0|1) return 0 ;; *) echo "stopping after $n"; exit $rc ;; esac
}
for lib in var/bisect_wpabs1_*.so var/wpabs1_no*.so; do
  L=$(basename $lib .so)
  timeout -k 10 120 env PAXISIM_LIB=$lib python tools/sink_guard.py wp_crash > $O/$L.json 2> $O/$L.err
  rc=$?; echo "$L rc=$rc $(tail -c 120 $O/$L.json)"
  case $rc in 0|1) ;; *) echo "stopping after $L"; exit $rc ;; esac
done
step ab_lin 1200 tools/ab_env.sh r5c/ab_lin "prod|X=1" "w5|PAXISIM_LIB=var/lin_w5.so" "w6|PAXISIM_LIB=var/lin_w6.so" \
  "w7|PAXISIM_LIB=var/lin_w7.so" "w5ns|PAXISIM_LIB=var/lin_w5_nosink.so" "w6ns|PAXISIM_LIB=var/lin_w6_nosink.so" \
  "w7ns|PAXISIM_LIB=var/lin_w7_nosink.so" "w6b|PAXISIM_LIB=var/lin_w6.so" "w5b|PAXISIM_LIB=var/lin_w5.so" -- --config 3
export TMPDIR=/tmp
step prof_c2 400 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- python bench.py --no-cpu-baseline --no-shard-check --config 2
for c in SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d $O/pmc_$c -o run --output-format csv -- python bench.py --no-cpu-baseline --no-shard-check --config 2 --steps 4 --warmup 2 > $O/pmc_$c.log 2>&1
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
