#!/bin/bash
# Round-6 GPU call helper: `step <name> <timeout s> <command...>` runs one GPU step under its own time
# limit, logs to $O/<name>.log and ends the call on the first failure (no GPU step after a fault).
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -4 "$O/$n.log" | cut -c1-400
  case $rc in 0) return 0 ;; *) echo "stopping after $n"; exit $rc ;; esac
}
# soft: a Python error (rc 1, e.g. a PaxisimError the library raised after its kernels ended) is
# reported and the call goes on; a time limit, abort or fault still ends it
soft() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -4 "$O/$n.log" | cut -c1-400
  case $rc in 0|1) return 0 ;; *) echo "stopping after $n"; exit $rc ;; esac
}
