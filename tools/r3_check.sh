#!/bin/bash
# GPU box: diagnostic variants of the WPaxos divergence, then the GPU suite and
# the config-3 bench (linearizability scan timing).  Any timeout / signal / fault
# ends the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r3b}
mkdir -p "$OUT"
stop() { echo "STOP at $1 rc=$2"; exit "$2"; }
for v in ${VARIANTS:-}; do
  PAXISIM_LIB=var/$v.so timeout -k 10 240 python -u tools/diverge.py wp_crash 250 > "$OUT/div_$v.log" 2>&1
  rc=$?; echo "div_$v rc=$rc"; tail -n 4 "$OUT/div_$v.log"
  [ $rc -le 1 ] || stop "div_$v" $rc
done
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $TESTS > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -n 15 "$OUT/pytest_gpu.log"
  [ $rc -eq 0 ] || stop pytest $rc
fi
if [ -n "${BENCH:-}" ]; then
  for c in $BENCH; do
    timeout -k 10 600 python -u bench.py --config $c ${BENCH_ARGS:-} > "$OUT/bench_c$c.json" 2> "$OUT/bench_c$c.err"
    rc=$?; echo "bench c$c rc=$rc"; tail -c 1500 "$OUT/bench_c$c.json"; echo
    [ $rc -eq 0 ] || stop "bench c$c" $rc
  done
fi
exit 0
