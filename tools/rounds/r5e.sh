#!/bin/bash
# Round-5 GPU call E: GPU suite + smoke on the product (per-unit flags, Reply routing, miscompile guards),
# the r4l reconstruction without the SDWA peephole, and mirrored A/Bs of each unit's flag choice.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r5e
mkdir -p $O
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"; tail -4 "$O/$n.log"
  case $rc in 0|1) return 0 ;; *) echo "stopping after $n"; exit $rc ;; esac
}
step pytest_product 400 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_wpabs2_nosdwa 400 env PAXISIM_LIB=var/libpaxisim_wpabs2_nosdwa.so python -u -m pytest -q --timeout 120 \
  --timeout-method thread -m gpu tests/test_parity_wpaxos_gpu.py tests/test_parity_scale_gpu.py tests/test_database.py \
  tests/test_m2paxos_kpaxos.py tests/test_workload_gpu.py
export REPS=3
step ab_c2 900 tools/ab_env.sh r5e/ab_c2 "prod|X=1" "p5sdwa|PAXISIM_LIB=var/v_p5sdwa.so" -- --config 2
step ab_c5 900 tools/ab_env.sh r5e/ab_c5 "prod|X=1" "wpflag|PAXISIM_LIB=var/v_wpflag.so" -- --config 5
step ab_c4 900 tools/ab_env.sh r5e/ab_c4 "prod|X=1" "p9nosdwa|PAXISIM_LIB=var/v_p9nosdwa.so" -- --config 4
step ab_c3 600 tools/ab_env.sh r5e/ab_c3 "prod|X=1" "abdnoflag|PAXISIM_LIB=var/v_abdnoflag.so" -- --config 3
