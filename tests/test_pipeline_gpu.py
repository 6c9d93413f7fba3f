"""Pipelined serial launches (sim_core.h sim_serial_pipe) are
invisible: K chunks of a launch's steps run as (tile, chunk) tickets, each
tile's chunks in order, and every replica state, instance and statistic must
equal the oracle's and the unpipelined run's.  The launch count shows the
chunks were fused."""
import pytest

from paxi_amd import abi
import oracle_lib as ol
from test_parity_gpu import assert_same

pytestmark = pytest.mark.gpu


def _run(monkeypatch, pipe, cfg, wl, fp=None, faults=(), steps=(200, 200)):
    from paxi_amd.sim import Simulation
    monkeypatch.setenv("PAXISIM_PIPE", str(pipe))
    g = Simulation(cfg, wl, fp, faults)
    for n in steps:
        g.step(n)
    g.sync()
    _, launches = g.kernel_time()
    return g, launches


def _oracle(cfg, wl, fp=None, faults=(), steps=(200, 200)):
    o = ol.OracleSim(cfg, wl, fp, faults)
    o.step(sum(steps))
    return o


@pytest.mark.parametrize("clusters", [64, 1000, 4096 + 17])
def test_paxos_pipelined_matches_oracle_and_fuses(monkeypatch, clusters):
    """Multi-Paxos with Drop/Slow and compaction (every two chunks when pipelined)."""
    cfg = abi.make_config(npz=[5], clusters=clusters, seed=11, window=16, mbox_cap=32, max_delay=4,
                          steps_per_launch=20)
    wl = abi.make_workload(outstanding=8, target=0)
    fp = abi.make_fault_process(drop_ppm=5000, drop_len=20, slow_ppm=5000, slow_len=20, slow_min=1, slow_max=4)
    g, k4 = _run(monkeypatch, 4, cfg, wl, fp)
    o = _oracle(cfg, wl, fp)
    assert_same(g, o, "pipe 4")
    g.close()
    g1, k1 = _run(monkeypatch, 1, cfg, wl, fp)
    assert k1 == 400 // 20 and k4 < k1, (k1, k4)        # two chunks per launch between compactions
    g1.close()


def test_wpaxos_pipelined_matches_oracle(monkeypatch):
    """WPaxos (no compaction: up to four chunks per launch), a leader crash mid-run."""
    cfg = abi.make_config(protocol=abi.WPAXOS, npz=[3, 3, 3], keys=8, clusters=700, seed=5, window=16,
                          mbox_cap=24, max_delay=0, policy_threshold=3, steps_per_launch=25)
    wl = abi.make_workload(outstanding=9, target=list(range(9)), locality_ppm=700_000)
    faults = [abi.make_fault(abi.FAULT_CRASH, src=0, step_from=150, step_to=260)]
    g, k4 = _run(monkeypatch, 4, cfg, wl, None, faults)
    o = _oracle(cfg, wl, None, faults)
    assert_same(g, o, "wpaxos pipe 4")
    gi, oi = g.read_instances(), o.read_instances()
    assert [x.as_tuple() for x in gi] == [x.as_tuple() for x in oi]
    assert k4 == 400 // 100, k4
    g.close()


def test_abd_pipelined_matches_oracle(monkeypatch):
    cfg = abi.make_config(protocol=abi.ABD, npz=[5], clusters=1500, seed=3, keys=16, history=512,
                          steps_per_launch=10)
    wl = abi.make_workload(outstanding=4, target=[0, 1, 2, 3], write_ppm=500_000, keys=16)
    g, k4 = _run(monkeypatch, 4, cfg, wl, steps=(80, 40))
    o = _oracle(cfg, wl, steps=(80, 40))
    assert_same(g, o, "abd pipe 4")
    assert g.linearizable()[:2] == o.linearizable()[:2]   # (anomalies, ops); the GPU adds partitions skipped
    assert k4 == 2 + 1, k4                                 # 80 = 2 x 4 chunks, 40 = 1 x 4
    g.close()


def test_gave_up_wait_fails_every_readout(monkeypatch):
    """A chunk wait that gives up leaves its tile unstepped; the library must
    say so at the next call of every kind, never return partial stats or state
    (ADVICE r5).  PAXISIM_PIPE_SPIN=0 makes the first unsatisfied poll give up:
    with one tile the waves of chunks 1..K-1 start while chunk 0 runs."""
    from paxi_amd.sim import PaxisimError, Simulation
    cfg = abi.make_config(npz=[5], clusters=64, seed=11, window=16, mbox_cap=32, max_delay=4,
                          steps_per_launch=20)
    wl = abi.make_workload(outstanding=8, target=0)
    monkeypatch.setenv("PAXISIM_PIPE", "4")
    monkeypatch.setenv("PAXISIM_PIPE_SPIN", "0")
    g = Simulation(cfg, wl)
    g.step(400)
    for name, call in [("sync", g.sync), ("stats", g.stats), ("read_state", g.read_state),
                       ("kernel_time", g.kernel_time), ("check", g.check)]:
        with pytest.raises(PaxisimError, match="chunk wait timed out") as e:
            call()
        assert "done[tile]" in str(e.value), name      # the stuck wait names itself
    g.close()
