"""EPaxos (epaxos/replica.go, epaxos/instance.go; FastQuorum quorum.go:65-67).

Known answers derived by hand from the Go source (derivations in the
docstrings), checked on the oracle; GPU parity under -m gpu.  A=1.1, B=1.2,
C=1.3 (replicas 0, 1, 2)."""
import pytest

from paxi_amd import abi
import oracle_lib as ol


def ep_cfg(npz=(3,), clusters=1, seed=1, keys=1, **kw):
    kw.setdefault("window", 16)
    kw.setdefault("mbox_cap", 16)
    kw.setdefault("max_delay", 1)
    return abi.make_config(protocol=abi.EPAXOS, npz=list(npz), clusters=clusters, seed=seed, keys=keys, **kw)


@pytest.mark.parametrize("seed", [1, 9])
def test_single_write_fast_path(seed):
    """N=5, one request at A: PreAccept to the 4 peers (replica.go:138-144);
    the replies all arrive together and the second one makes the quorum
    FastQuorum (size 3 >= 5*3/4, quorum.go:66) with nothing changed and every
    dep committed, so A commits on the fast path (replica.go:225-243), executes
    and replies, then broadcasts Commit; the later replies find the instance
    COMMITTED (replica.go:197).  12 messages; everyone executes cmd 1 once."""
    o = ol.OracleSim(ep_cfg(npz=(5,), seed=seed, keys=4), abi.make_workload(outstanding=1, max_requests=1, target=[0]))
    o.step(10)
    st = o.stats().as_dict()
    assert st["delivered"] == {"PreAccept": 4, "PreAcceptReply": 4, "Commit": 4}
    assert st["commits"] == 1 and st["replies"] == 1
    assert [o.exec_log(0, r) for r in range(5)] == [[1]] * 5
    s = o.read_state()
    assert s[0].slot == 0 and all(r.execute == 1 and r.executions == 1 for r in s)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_conflict_slow_path(seed):
    """N=3, one key: A gets cmd 1 and B cmd 2 at step 0; links B->C and C->A
    are slowed by one step.
      t0  A, B: instance 0 of their own log, seq 0, PreAccept to the others.
      t1  A handles B's PreAccept: conflicts[A][k] = 0 is not above dep 0, but
          maxSeqPerKey[k] = 0, so seq 1 (replica.go:58-80) -> reply seq 1; B
          likewise answers A with seq 1.  C gets only A's (B->C slowed): seq 0.
      t2  A: B's reply is the first, and FastQuorum at N=3 is 2 (3*3/4): the
          merge raised seq 0 -> 1, so `changed` -> slow path, Accept (seq 1).
          B: A's reply the same -> Accept.  C: B's PreAccept: seq 1 -> reply.
      t3  everyone answers the Accepts it has; the late PreAcceptReplies find
          ACCEPTED instances (replica.go:197).  C gets B's Accept at t4.
      t4  A, B: an AcceptReply makes a Majority: commit, execute their own
          command (the other log's instance 0 is only ACCEPTED: break,
          replica.go:372), broadcast Commit.
      t5  A executes cmd 2, B cmd 1; C executes cmd 1 (Commit A), t6 cmd 2.
    20 messages, 2 commits; execution orders A [1,2], B [2,1], C [1,2] — the
    reference executes conflicting commands in different orders."""
    wl = abi.make_workload(outstanding=2, target=[0, 1], max_requests=1)
    f = [abi.make_fault(abi.FAULT_SLOW, 1, 2, 1), abi.make_fault(abi.FAULT_SLOW, 2, 0, 1)]
    o = ol.OracleSim(ep_cfg(seed=seed), wl, faults=f)
    o.step(10)
    st = o.stats().as_dict()
    assert st["delivered"] == {"PreAccept": 4, "PreAcceptReply": 4, "Accept": 4, "AcceptReply": 4, "Commit": 4}
    assert st["commits"] == 2 and st["replies"] == 2
    assert [o.exec_log(0, r) for r in range(3)] == [[1, 2], [2, 1], [1, 2]]


@pytest.mark.parametrize("seed", [1, 5])
def test_nil_gap_reexecutes(seed):
    """execute() skips a nil instance without advancing executed[id]
    (replica.go:362-383) and nothing marks an instance EXECUTED, so every later
    call runs the committed instances after the gap again.  N=3, both workers
    at A (the second from step 1), A->C dropped at steps 0 and 2: C never
    hears of A's instance 0 (PreAccept and Commit lost) but gets 1, 2, 3.
    C executes 2 (t4); then 2 again and 3 (t6); then 2, 3 and 4 (t7)."""
    wl = abi.make_workload(outstanding=2, target=[0, 0], max_requests=2, start_step=[0, 1])
    f = [abi.make_fault(abi.FAULT_DROP, 0, 2, step_from=0, step_to=1),
         abi.make_fault(abi.FAULT_DROP, 0, 2, step_from=2, step_to=3)]
    o = ol.OracleSim(ep_cfg(seed=seed), wl, faults=f)
    o.step(20)
    assert [o.exec_log(0, r) for r in range(3)] == [[1, 2, 3, 4], [1, 2, 3, 4], [2, 2, 3, 2, 3, 4]]
    inst = o.read_instances()
    assert (inst[6].slot, inst[6].execute, inst[6].p1_acks) == (3, 0, 0)   # C: A's log stuck before slot 0
    assert o.stats().dropped == 2


@pytest.mark.gpu
@pytest.mark.parametrize("npz,keys,faults", [((3,), 1, False), ((5,), 4, True), ((2, 2, 3), 8, True)])
def test_gpu_parity(npz, keys, faults):
    from test_parity_wpaxos_gpu import run_and_compare
    N = sum(npz)
    wl = abi.make_workload(outstanding=N, target=list(range(N)))
    fp = abi.make_fault_process(drop_ppm=1500, drop_len=10, slow_ppm=3000, slow_len=20, slow_min=1,
                                slow_max=3) if faults else None
    sc = [abi.make_fault(abi.FAULT_CRASH, 1, step_from=60, step_to=90)] if faults else []
    cfg = ep_cfg(npz=npz, clusters=130, seed=11, keys=keys, window=32, mbox_cap=32, max_delay=3)
    st = run_and_compare(cfg, wl, fp, sc, chunks=(70, 53))
    assert st["commits"] > 0


@pytest.mark.gpu
def test_gpu_kats():
    """The hand-derived traces above on the device: counts and executed digests."""
    from paxi_amd.sim import Simulation
    cases = [(ep_cfg(npz=(5,), keys=4), abi.make_workload(outstanding=1, max_requests=1, target=[0]), [], 10),
             (ep_cfg(), abi.make_workload(outstanding=2, target=[0, 1], max_requests=1),
              [abi.make_fault(abi.FAULT_SLOW, 1, 2, 1), abi.make_fault(abi.FAULT_SLOW, 2, 0, 1)], 10),
             (ep_cfg(), abi.make_workload(outstanding=2, target=[0, 0], max_requests=2, start_step=[0, 1]),
              [abi.make_fault(abi.FAULT_DROP, 0, 2, step_from=0, step_to=1),
               abi.make_fault(abi.FAULT_DROP, 0, 2, step_from=2, step_to=3)], 20)]
    for cfg, wl, f, steps in cases:
        cfg.steps_per_launch = 1
        g, o = Simulation(cfg, wl, faults=f), ol.OracleSim(cfg, wl, faults=f)
        g.step(steps)
        o.step(steps)
        assert [r.as_tuple() for r in g.read_state()] == [r.as_tuple() for r in o.read_state()]
        assert g.stats().as_dict() == o.stats().as_dict()
