"""Agreement scan coverage (client.go:279-320 Consensus).

A follower cut off from the leader stalls at execute 0 while the leader runs
300 slots ahead.  A request at the follower (-ephemeral_leader,
paxos/replica.go:61) makes it run phase 1; the acceptors' P1bs carry only
uncommitted entries (paxos.go:149-155), so it re-proposes from slot 0 and
executes other commands in slots the others executed long ago — the
reference's own gap, here in Multi-Paxos.  The lagging
replica's executed prefix must be compared with the first executor's however
far behind it runs: with the default ring the violation is found; with a
1-entry ring (the old 8-checkpoint horizon's situation) it is not, and the
coverage counters say so."""
import pytest

from paxi_amd import abi
import oracle_lib as ol


def scenario(ring=0):
    cfg = abi.make_config(npz=[3], clusters=3, seed=3, window=16, mbox_cap=16, max_delay=0, ephemeral_leader=1,
                          agree_ring=ring)
    wl = abi.make_workload(outstanding=1, target=[0], max_requests=300)
    faults = [abi.make_fault(abi.FAULT_DROP, src, 2, step_from=0, step_to=1000, cluster_lo=0, cluster_hi=1)
              for src in (0, 1)]
    return cfg, wl, faults


def drive(sim):
    sim.step(1000)
    cid = 1 << 20
    for _ in range(40):               # one request per step: few live ghost entries, the model stays faithful
        sim.inject(0, 2, cid)
        cid += 1
        sim.step(1)
    sim.step(20)


def test_lagging_divergence_detected_oracle():
    cfg, wl, faults = scenario()
    o = ol.OracleSim(cfg, wl, faults=faults)
    drive(o)
    s = o.read_state(0, 1)
    assert s[0].execute == 300 and s[2].execute == 40      # 260 slots of lag, beyond 8 x 16
    assert all(not (r.flags & abi.F_UNFAITHFUL) for r in s)
    st = o.stats()
    assert st.agree_mismatch >= 2 and st.agree_missed == 0
    assert o.check() == 1                                  # cluster 0 only; 1 and 2 agree
    lo = ol.OracleSim(*scenario(ring=1)[:2], faults=scenario(ring=1)[2])
    drive(lo)
    assert lo.check() == 0 and lo.stats().agree_missed > 0   # the old horizon misses it, and says so


@pytest.mark.gpu
@pytest.mark.parametrize("ring", [0, 1])
def test_lagging_divergence_detected_gpu(ring):
    from paxi_amd.sim import Simulation
    cfg, wl, faults = scenario(ring)
    g, o = Simulation(cfg, wl, faults=faults), ol.OracleSim(cfg, wl, faults=faults)
    drive(g)
    drive(o)
    assert [r.as_tuple() for r in g.read_state()] == [r.as_tuple() for r in o.read_state()]
    assert g.stats().as_dict() == o.stats().as_dict()
    assert g.check() == o.check() == (1 if ring == 0 else 0)
