#!/bin/bash
# GPU box: machine-sink hypothesis for the register clobber (round-2 verdict item 1)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r3d; mkdir -p $OUT
for v in inl_nosink inl_nopsink; do
  PAXISIM_LIB=var/$v.so timeout -k 10 240 python -u tools/diverge.py wp_crash 250 > $OUT/div_$v.log 2>&1
  rc=$?; echo "div_$v rc=$rc"; tail -n 3 $OUT/div_$v.log; [ $rc -le 1 ] || exit $rc
done
PAXISIM_LIB=var/def_nosink.so timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_parity_gpu.py tests/test_parity_wpaxos_gpu.py > $OUT/pytest_def_nosink.log 2>&1
rc=$?; echo "pytest def_nosink rc=$rc"; tail -n 5 $OUT/pytest_def_nosink.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_parity_gpu.py > $OUT/pytest_def.log 2>&1
rc=$?; echo "pytest default rc=$rc"; grep -E "FAILED|passed|failed" $OUT/pytest_def.log | tail -n 8
exit 0
