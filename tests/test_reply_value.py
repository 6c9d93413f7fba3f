"""Reply.Value (message.go:42-48): the value Execute returns - the key's value
before the command (db.go:103-114) - travels back on every reply
(paxos.go:352-362, epaxos/replica.go:373-379); ABD replies to a read with the
value it read (abd/replica.go:145-150); ReplyWhenCommit replies carry none
(paxos.go:300-304).  Values are command ids (a write's value is its cid), 0 is
nil.  The worker's last reply is readable through paxisim_read_client."""
import pytest

from paxi_amd import abi
import oracle_lib as ol


def single_worker(protocol=abi.PAXOS, npz=(3,), **kw):
    cfg = abi.make_config(protocol=protocol, npz=list(npz), clusters=kw.pop("clusters", 2), seed=4, window=16,
                          mbox_cap=16, max_delay=0, kv=1, keys=kw.pop("keys", 1), **kw)
    wl = abi.make_workload(outstanding=1, target=[0], write_ppm=500_000, max_requests=60)
    return cfg, wl


def replies(sim, steps, cluster=0):
    """(cid, reply value) of every reply the worker receives, stepping one step at a time."""
    out, last = [], sim.read_client(cluster)[0]
    for _ in range(steps):
        sim.step(1)
        cur = sim.read_client(cluster)[0]
        if cur[1] != last[1] or (cur[0] == 0 and last[0] != 0):   # a reply arrived: next request issued / done
            out.append((last[0], cur[2]))
        last = cur
    return out


@pytest.mark.parametrize("protocol", [abi.PAXOS, abi.EPAXOS])
def test_reply_value_is_the_previous_value_oracle(protocol):
    """One worker, one key: each reply holds the cid of the last write executed
    before the command (0 before the first write), reads and writes alike."""
    cfg, wl = single_worker(protocol)
    o = ol.OracleSim(cfg, wl)
    got = replies(o, 400)
    assert len(got) == 60
    last_write, want = 0, []
    for cid, _ in got:
        want.append((cid, last_write))
        if o.command(0, cid)[1]:
            last_write = cid
    assert got == want


def test_abd_read_reply_holds_the_read_value_oracle():
    cfg, wl = single_worker(abi.ABD, npz=(5,))
    o = ol.OracleSim(cfg, wl)
    got = replies(o, 400)
    assert len(got) == 60
    last_write = 0
    for cid, v in got:
        if o.command(0, cid)[1]:
            assert v == 0                                  # Reply{Command} for a write
            last_write = cid
        else:
            assert v == last_write                         # one worker: reads see the last write


def test_reply_when_commit_has_no_value_oracle():
    cfg, wl = single_worker(reply_when_commit=1)
    o = ol.OracleSim(cfg, wl)
    assert all(v == 0 for _, v in replies(o, 400))


@pytest.mark.gpu
@pytest.mark.parametrize("protocol,npz", [(abi.PAXOS, (3,)), (abi.PAXOS, (5,)), (abi.EPAXOS, (3,)),
                                          (abi.ABD, (5,)), (abi.WPAXOS, (3, 3, 3))])
def test_reply_values_gpu(protocol, npz):
    """Every worker's (cid, issued, reply value) on the GPU equals the oracle's,
    step by step for one cluster and at the end for a batch with forwarding
    and several workers."""
    from paxi_amd.sim import Simulation
    kw = {"keys": 4} if protocol in (abi.WPAXOS, abi.ABD) else {}
    cfg, wl = single_worker(protocol, npz, **kw)
    g, o = Simulation(cfg, wl), ol.OracleSim(cfg, wl)
    assert replies(g, 300) == replies(o, 300)
    g.close()
    cfg = abi.make_config(protocol=protocol, npz=list(npz), clusters=130, seed=8, window=16, mbox_cap=24,
                          max_delay=2, kv=1, keys=4)
    n = abi.n_replicas(cfg)
    wl = abi.make_workload(outstanding=6, target=[w % n for w in range(6)], write_ppm=400_000)
    fp = abi.make_fault_process(drop_ppm=2000, drop_len=10, slow_ppm=2000, slow_len=10, slow_min=1, slow_max=2)
    g, o = Simulation(cfg, wl, fp), ol.OracleSim(cfg, wl, fp)
    g.step(250)
    o.step(250)
    for c in range(cfg.clusters):
        assert g.read_client(c) == o.read_client(c), f"cluster {c}"
    assert any(v for c in range(cfg.clusters) for (_, _, v) in g.read_client(c))
    g.close()
