#!/bin/bash
# GPU box: locate the first GPU/oracle divergence of the inlined-agreement build
# (round-2 verdict item 1).  Exit codes 0/1 of diverge.py are results; anything
# else (a timeout, a signal, a fault) ends the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r3a}
mkdir -p "$OUT"
run() {   # name lib chunk [spl]
  local name=$1 lib=$2; shift 2
  PAXISIM_LIB=$lib timeout -k 10 240 python -u tools/diverge.py wp_crash "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -n 30 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
run def_250 paxi_amd/libpaxisim.so 250
run inl_250 var/inl.so 250
run inl_10 var/inl.so 10
run inl_1 var/inl.so 1
run inlal_250 var/inl_al.so 250
exit 0
