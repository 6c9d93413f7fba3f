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


# ---- arrivals in one step: the coverage counters are order-free ------------
def same_step_case(clusters=640):
    """Replicas 1..4 of every cluster commit slots 0..15 in one step through
    P3s delivered from replica 0 (paxos.go:313-343), executing commands A, B, B
    and C: all four reach digest checkpoint 1 in that step.  Applied in replica
    order, replica 1 records A and the three others mismatch; had replica 2
    arrived first, only two would.  Every link is dropped and no worker runs,
    so only the delivered records move (paxi_amd.trace.replay_setup)."""
    from paxi_amd import trace
    cfg = abi.make_config(npz=[5], clusters=clusters, seed=9, window=16, mbox_cap=16, max_delay=0)
    wl = abi.make_workload(outstanding=1, target=[0])
    faults = trace.replay_setup(wl, 5)
    return cfg, wl, faults


def deliver_same_step(sim, clusters):
    base = {1: 100, 2: 200, 3: 200, 4: 300}
    for c in range(clusters):
        for r, b in base.items():
            sim.deliver(c, r, 0, [(0, abi.MSG_P3, 0, s, b + s) for s in range(16)])
    sim.step(1)


def test_same_step_arrivals_oracle():
    cfg, wl, faults = same_step_case(4)
    o = ol.OracleSim(cfg, wl, faults=faults)
    deliver_same_step(o, 4)
    st = o.stats()
    assert (st.agree_compared, st.agree_mismatch, st.agree_missed) == (3 * 4, 3 * 4, 0)


@pytest.mark.gpu
def test_same_step_arrivals_gpu():
    """The GPU's waves race within a step; the counters come out in replica
    order anyway (per-step arrival lists drained after the barrier)."""
    from paxi_amd.sim import Simulation
    cfg, wl, faults = same_step_case()
    g, o = Simulation(cfg, wl, faults=faults), ol.OracleSim(cfg, wl, faults=faults)
    for s in (g, o):
        deliver_same_step(s, cfg.clusters)
    gs, os_ = g.stats(), o.stats()
    assert (gs.agree_compared, gs.agree_mismatch, gs.agree_missed) == (3 * 640, 3 * 640, 0)
    assert gs.as_dict() == os_.as_dict()
    assert g.check() == o.check() == 640
    g.close()


def agmax_case():
    """KPaxos (per-key instances, kpaxos/replica.go), N=5, 16 keys: replica 1
    receives, in one step, P3s for slots 0..15 of every key (four peers x 64
    records), so it reaches 16 checkpoints in that step.  The first AGMAX = 8
    are applied to the ring (each the first arrival of its key: recorded), the
    other 8 count as missed - on both backends."""
    from paxi_amd import trace
    cfg = abi.make_config(protocol=abi.KPAXOS, npz=[5], keys=16, clusters=64, seed=9, window=16, mbox_cap=64,
                          max_delay=0)
    wl = abi.make_workload(outstanding=1, target=[0])
    return cfg, wl, trace.replay_setup(wl, 5)


def deliver_agmax(sim, clusters):
    for c in range(clusters):
        for j, src in enumerate((0, 2, 3, 4)):
            recs = [(0, abi.MSG_P3 | (k << 16), 0, s, 1 + 16 * k + s) for k in range(4 * j, 4 * j + 4)
                    for s in range(16)]
            sim.deliver(c, 1, src, recs)
    sim.step(1)


def test_arrivals_beyond_agmax_count_as_missed_oracle():
    cfg, wl, faults = agmax_case()
    o = ol.OracleSim(cfg, wl, faults=faults)
    deliver_agmax(o, 2)
    st = o.stats()
    assert (st.agree_compared, st.agree_missed, st.agree_mismatch) == (0, 8 * 2, 0)
    assert all(i.execute == 16 for i in o.read_instances(0, 1)[16:32])


@pytest.mark.gpu
def test_arrivals_beyond_agmax_count_as_missed_gpu():
    from paxi_amd.sim import Simulation
    cfg, wl, faults = agmax_case()
    g, o = Simulation(cfg, wl, faults=faults), ol.OracleSim(cfg, wl, faults=faults)
    for s in (g, o):
        deliver_agmax(s, cfg.clusters)
    assert g.stats().as_dict() == o.stats().as_dict()
    assert g.stats().agree_missed == 8 * 64
    assert [i.as_tuple() for i in g.read_instances()] == [i.as_tuple() for i in o.read_instances()]
    g.close()
