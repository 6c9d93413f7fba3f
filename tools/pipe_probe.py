"""Diagnostic: one small Multi-Paxos batch stepped through pipelined launches
(PAXISIM_PIPE, sim_core.h sim_serial_pipe), timed per call and checked
against the oracle at the end; prints as it goes, so a stuck launch shows
which call it was.

  PAXISIM_PIPE=4 python tools/pipe_probe.py [clusters] [calls] [steps per call] [steps per launch]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from paxi_amd import abi  # noqa: E402
from paxi_amd.sim import Simulation  # noqa: E402


def main():
    clusters, calls, per, S = (int(a) for a in (sys.argv[1:5] + ["256", "4", "40", "10"][len(sys.argv) - 1:]))
    cfg = abi.make_config(npz=[5], clusters=clusters, seed=42, window=32, mbox_cap=16, max_delay=4,
                          steps_per_launch=S)
    wl = abi.make_workload(outstanding=8, target=0)
    fp = abi.make_fault_process(drop_ppm=2000, drop_len=20, slow_ppm=2000, slow_len=20, slow_min=1, slow_max=4)
    print("pipe", os.environ.get("PAXISIM_PIPE"), "lib", os.environ.get("PAXISIM_LIB"), "clusters", clusters,
          flush=True)
    with Simulation(cfg, wl, fp) as g:
        for k in range(calls):
            t = time.perf_counter()
            g.step(per)
            g.sync()
            print(f"call {k}: {per} steps in {time.perf_counter() - t:.3f} s", flush=True)
        gs = [s.as_tuple() for s in g.read_state()]
    import oracle_lib
    o = oracle_lib.OracleSim(cfg, wl, fp)
    o.step(calls * per)
    os_ = [s.as_tuple() for s in o.read_state()]
    bad = [i for i, (a, b) in enumerate(zip(gs, os_)) if a != b]
    print("replica states equal to the oracle:", not bad, "first differing:", bad[:5], flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
