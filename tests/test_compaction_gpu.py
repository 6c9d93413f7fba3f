"""Live-cluster compaction is invisible: clusters that reach
a fixed point (empty mailboxes; Paxi has no timers or retries) are frozen and
packed behind the live ones, and requests injected into frozen clusters wake
them with their link fault process replayed.  Every result must stay
bit-exact with the CPU oracle, which knows nothing of slots."""
import pytest

from paxi_amd import abi
import oracle_lib as ol
from test_parity_gpu import assert_same

pytestmark = pytest.mark.gpu


def _pair(cfg, wl, fp=None, faults=()):
    from paxi_amd.sim import Simulation
    return Simulation(cfg, wl, fp, faults), ol.OracleSim(cfg, wl, fp, faults)


def _logs_same(g, o, clusters, N):
    for c in clusters:
        for r in range(N):
            e = min(x.execute for x in o.read_state(c, 1))
            a = [x.as_tuple() for x in g.read_log(c, r, e - 3, 24)]
            b = [x.as_tuple() for x in o.read_log(c, r, e - 3, 24)]
            assert a == b, f"log of cluster {c} replica {r}"


def test_clusters_die_and_freeze(monkeypatch):
    """Heavy Drop/Slow: most clusters stall for good (a P2a lost to a majority
    is never retried) and are frozen; state matches the oracle throughout."""
    monkeypatch.setenv("PAXISIM_COMPACT_EVERY", "20")
    cfg = abi.make_config(npz=[5], clusters=2048 + 37, seed=5, window=16, mbox_cap=32, max_delay=4,
                          steps_per_launch=10)
    wl = abi.make_workload(outstanding=8, target=0)
    fp = abi.make_fault_process(drop_ppm=20000, drop_len=40, slow_ppm=10000, slow_len=30, slow_min=1, slow_max=4)
    g, o = _pair(cfg, wl, fp)
    active = []
    for k in range(8):
        g.step(75)
        o.step(75)
        assert_same(g, o, f"chunk {k}")
        active.append(g.active_clusters())
    assert active[-1] < cfg.clusters // 2, active       # compaction really ran
    _logs_same(g, o, range(0, cfg.clusters, 97), 5)


def test_wake_frozen_clusters_by_injection(monkeypatch):
    """Workers stop after max_requests, clusters go quiet and freeze; requests
    injected later (http.go:99) wake them, with their link fault windows
    replayed over the frozen steps."""
    monkeypatch.setenv("PAXISIM_COMPACT_EVERY", "16")
    cfg = abi.make_config(npz=[3], clusters=640, seed=31, window=16, mbox_cap=16, max_delay=3,
                          ephemeral_leader=1, steps_per_launch=8)
    wl = abi.make_workload(outstanding=3, target=[0, 1, 2], max_requests=6)
    fp = abi.make_fault_process(drop_ppm=8000, drop_len=20, slow_ppm=8000, slow_len=20, slow_min=1, slow_max=3)
    g, o = _pair(cfg, wl, fp)
    g.step(200)
    o.step(200)
    assert_same(g, o, "quiet")
    assert g.active_clusters() < 128
    cid = 1 << 22
    for rnd in range(4):
        for c in range(rnd, 640, 37):
            g.inject(c, (c + rnd) % 3, cid)
            o.inject(c, (c + rnd) % 3, cid)
            cid += 1
        g.step(60)
        o.step(60)
        assert_same(g, o, f"wake round {rnd}")
    _logs_same(g, o, range(0, 640, 37), 3)


def test_compaction_on_equals_off(monkeypatch):
    """The same run with compaction disabled gives identical per-replica state."""
    cfg = abi.make_config(npz=[5], clusters=700, seed=77, mbox_cap=32, steps_per_launch=25)
    wl = abi.make_workload(outstanding=8, target=0)
    fp = abi.make_fault_process(drop_ppm=15000, drop_len=30, slow_ppm=5000, slow_len=30, slow_min=1, slow_max=4)
    from paxi_amd.sim import Simulation
    res = []
    for flag in ("1", "0"):
        monkeypatch.setenv("PAXISIM_COMPACT", flag)
        monkeypatch.setenv("PAXISIM_COMPACT_EVERY", "25")
        s = Simulation(cfg, wl, fp)
        s.step(500)
        res.append(([x.as_tuple() for x in s.read_state()], s.stats().as_dict(), s.check(), s.active_clusters()))
        s.close()
    assert res[0][:3] == res[1][:3]
    assert res[0][3] < res[1][3] == cfg.clusters


@pytest.mark.parametrize("period", ["3", "2"])
def test_phase_binning_is_invisible(monkeypatch, period):
    """Phase binning reorders every live cluster's slot at each
    compaction by the step residue it was busiest at; the state is bit-exact
    with the oracle, and with compaction off, including the wake path."""
    monkeypatch.setenv("PAXISIM_PHASE_SORT", "1")
    monkeypatch.setenv("PAXISIM_PHASE_PERIOD", period)
    monkeypatch.setenv("PAXISIM_COMPACT_EVERY", "20")
    cfg = abi.make_config(npz=[5], clusters=2048 + 37, seed=9, window=16, mbox_cap=32, max_delay=4,
                          steps_per_launch=10)
    wl = abi.make_workload(outstanding=8, target=0)
    fp = abi.make_fault_process(drop_ppm=3000, drop_len=40, slow_ppm=3000, slow_len=30, slow_min=1, slow_max=4)
    g, o = _pair(cfg, wl, fp)
    for k in range(6):
        g.step(70)
        o.step(70)
        assert_same(g, o, f"chunk {k}")
    cid = 1 << 22
    for c in range(0, cfg.clusters, 41):                   # wake frozen clusters too
        g.inject(c, 0, cid)
        o.inject(c, 0, cid)
        cid += 1
    g.step(60)
    o.step(60)
    assert_same(g, o, "after wake")
    _logs_same(g, o, range(0, cfg.clusters, 97), 5)
