"""Find the first step at which the GPU and the oracle diverge on one parity case.

Runs the HIP library (PAXISIM_LIB selects a variant build) and the oracle side
by side, `chunk` steps at a time, and compares every replica's state and every
instance after each chunk.  At the first difference it prints the step, the
differing records of both backends, and (when the chunk is one step) the inbox
each differing replica had at that step on both backends.

Usage: python tools/diverge.py <case> [chunk] [steps_per_launch]
  case: wp_crash  (test_parity_wpaxos_gpu.py::test_leader_crash_and_scripted_faults)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from paxi_amd import abi  # noqa: E402
from paxi_amd.sim import Simulation  # noqa: E402
import oracle_lib as ol  # noqa: E402


def case_wp_crash(spl):
    cfg = abi.make_config(protocol=abi.WPAXOS, npz=[3, 3, 3], keys=8, clusters=100, seed=5, window=16, mbox_cap=24,
                          max_delay=2, policy_threshold=3, steps_per_launch=spl)
    wl = abi.make_workload(outstanding=6, target=[0, 3, 6, 1, 4, 7], locality_ppm=700_000)
    faults = [abi.make_fault(abi.FAULT_CRASH, 0, step_from=60, step_to=160),
              abi.make_fault(abi.FAULT_FLAKY, 3, dst=abi.ALL_DST, param=200_000, step_from=0, step_to=300),
              abi.make_fault(abi.FAULT_SLOW, 6, dst=7, param=2, step_from=20, step_to=120)]
    return cfg, wl, None, faults, 250


CASES = {"wp_crash": case_wp_crash}


def main():
    case = sys.argv[1]
    chunk = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    spl = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    cfg, wl, fp, faults, total = CASES[case](spl)
    g = Simulation(cfg, wl, fp, faults)
    o = ol.OracleSim(cfg, wl, fp, faults)
    N, K = g.N, abi.n_instances(cfg)
    t = 0
    prev_in = None
    while t < total:
        n = min(chunk, total - t)
        if n == 1:
            prev_in = {}
        g.step(n)
        o.step(n)
        t += n
        gs, os_ = g.read_state(), o.read_state()
        gi, oi = g.read_instances(), o.read_instances()
        bad = [i for i in range(len(gs)) if gs[i].as_tuple() != os_[i].as_tuple()]
        badi = [i for i in range(len(gi)) if gi[i].as_tuple() != oi[i].as_tuple()]
        if bad or badi:
            print(f"FIRST DIVERGENCE after step {t} (chunk {n}, steps_per_launch {spl}, lib {os.environ.get('PAXISIM_LIB')})")
            for i in bad[:6]:
                print(f"  state cluster {i // N} replica {i % N}\n    gpu    {gs[i].as_tuple()}\n    oracle {os_[i].as_tuple()}")
            for i in badi[:12]:
                print(f"  inst cluster {i // (N * K)} replica {i // K % N} key {i % K}\n"
                      f"    gpu    {gi[i].as_tuple()}\n    oracle {oi[i].as_tuple()}")
            print(f"  {len(bad)} replica states and {len(badi)} instances differ")
            if n == 1:   # replay to the step before and show what the differing replicas received
                g.close()
                g2 = Simulation(cfg, wl, fp, faults)
                o2 = ol.OracleSim(cfg, wl, fp, faults)
                if t > 1:
                    g2.step(t - 1)
                    o2.step(t - 1)
                seen = set()
                for i in bad[:4] + [j // K for j in badi[:4]]:
                    c, r = i // N, i % N
                    if (c, r) in seen:
                        continue
                    seen.add((c, r))
                    gin, oin = g2.read_inbox(c, r), o2.read_inbox(c, r)
                    print(f"  inbox at step {t - 1} of cluster {c} replica {r} (src, hdr, ballot, slot, cid):"
                          f" {'equal' if gin == oin else 'DIFFERENT'}")
                    print(f"    gpu    {gin}\n    oracle {oin}")
            return 1
        print(f"step {t}: equal", flush=True)
    print("no divergence")
    return 0


if __name__ == "__main__":
    sys.exit(main())
