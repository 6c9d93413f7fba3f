#!/bin/bash
# GPU box: MachineSink workaround candidates and performance attribution (round 3).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r3f}; mkdir -p $OUT
ok() { [ $1 -le 1 ] || { echo "STOP rc=$1"; exit $1; }; }
for v in inl_sink1 inl_split0; do
  PAXISIM_LIB=var/old/$v.so timeout -k 10 240 python -u var/old/tools/diverge.py wp_crash 250 > $OUT/div_$v.log 2>&1
  rc=$?; echo "div_$v rc=$rc: $(tail -n 1 $OUT/div_$v.log)"; ok $rc
done
PAXISIM_LIB=var/def_split0.so timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_parity_gpu.py tests/test_parity_wpaxos_gpu.py > $OUT/pytest_split0.log 2>&1
rc=$?; echo "pytest split0 rc=$rc: $(tail -n 1 $OUT/pytest_split0.log)"; ok $rc
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_parity_wpaxos_gpu.py tests/test_m2paxos_kpaxos.py tests/test_trace.py tests/test_reply_value.py tests/test_agreement.py > $OUT/pytest_wlds.log 2>&1
rc=$?; echo "pytest wlds rc=$rc: $(tail -n 1 $OUT/pytest_wlds.log)"; ok $rc
B="--no-cpu-baseline --no-shard-check"
bench() {   # name config env...
  local name=$1 c=$2; shift 2
  env "$@" timeout -k 10 300 python -u bench.py --config $c $B > $OUT/bench_$name.json 2> $OUT/bench_$name.err
  local rc=$?
  python3 -c "import json,sys; d=json.loads(open('$OUT/bench_$name.json').read().strip().splitlines()[-1]); print('$name', 'c$c', '%.3g msg/s'%d['value'], 'launch %.2f ms'%d['roofline']['avg_launch_ms'])" 2>/dev/null || echo "$name rc=$rc"
  ok $rc
}
bench def5 5
bench def5_hbm 5 PAXISIM_WLDS=0
bench def2 2
bench split2 2 PAXISIM_LIB=var/def_split0.so
bench split5 5 PAXISIM_LIB=var/def_split0.so
bench sink2 2 PAXISIM_LIB=var/def_sink.so
bench sink5 5 PAXISIM_LIB=var/def_sink.so
exit 0
