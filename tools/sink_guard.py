"""Run the parity cases that caught the kernels' miscompiles (DESIGN.md §5.3:
round 3's pre-RA MachineSink, round 5's WPaxos absorb variant) on the library
PAXISIM_LIB names and print, as one JSON line, which of them diverge from the
oracle.  tests/test_miscompile_guard_gpu.py runs it on the guard variant
(paxi_amd/guard/libpaxisim_absorb.so) and on the product library;
tools/bisect_pass.sh's pass-bisection libraries are judged with it too.

  PAXISIM_LIB=paxi_amd/guard/libpaxisim_absorb.so python tools/sink_guard.py wp_crash
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from paxi_amd import abi  # noqa: E402
from paxi_amd.sim import Simulation, build_id  # noqa: E402
import oracle_lib as ol  # noqa: E402


def paxos_random(npz):
    # tests/test_parity_gpu.py::test_faults_random_process (generic-N kernel at N = 4, 7)
    cfg = abi.make_config(npz=npz, clusters=300, seed=42, window=16, mbox_cap=16, max_delay=4)
    wl = abi.make_workload(outstanding=8, target=0)
    fp = abi.make_fault_process(drop_ppm=3000, drop_len=25, slow_ppm=3000, slow_len=25, slow_min=1, slow_max=4)
    return cfg, wl, fp, [], 400


def wp_crash():
    # tests/test_parity_wpaxos_gpu.py::test_leader_crash_and_scripted_faults (tools/diverge.py wp_crash)
    cfg = abi.make_config(protocol=abi.WPAXOS, npz=[3, 3, 3], keys=8, clusters=100, seed=5, window=16, mbox_cap=24,
                          max_delay=2, policy_threshold=3)
    wl = abi.make_workload(outstanding=6, target=[0, 3, 6, 1, 4, 7], locality_ppm=700_000)
    faults = [abi.make_fault(abi.FAULT_CRASH, 0, step_from=60, step_to=160),
              abi.make_fault(abi.FAULT_FLAKY, 3, dst=abi.ALL_DST, param=200_000, step_from=0, step_to=300),
              abi.make_fault(abi.FAULT_SLOW, 6, dst=7, param=2, step_from=20, step_to=120)]
    return cfg, wl, None, faults, 250


CASES = {"paxos_n4": lambda: paxos_random([2, 2]), "paxos_n7": lambda: paxos_random([7]), "wp_crash": wp_crash}


def diverges(case):
    cfg, wl, fp, faults, steps = CASES[case]()
    g, o = Simulation(cfg, wl, fp, faults), ol.OracleSim(cfg, wl, fp, faults)
    g.step(steps)
    o.step(steps)
    bad = [r.as_tuple() for r in g.read_state()] != [r.as_tuple() for r in o.read_state()]
    if cfg.protocol in abi.PER_KEY:
        bad = bad or [i.as_tuple() for i in g.read_instances()] != [i.as_tuple() for i in o.read_instances()]
    g.close()
    o.close()
    return bad


if __name__ == "__main__":
    names = sys.argv[1:] or list(CASES)   # e.g. `wp_crash` alone for a pass bisection (tools/bisect_pass.sh)
    print(json.dumps({"lib": os.environ.get("PAXISIM_LIB", "paxi_amd/libpaxisim.so"), "build_id": build_id(),
                      "diverged": {c: diverges(c) for c in names}}), flush=True)
