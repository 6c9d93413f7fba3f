"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle on the
same seeded inputs — bit-exact replica state (ballot, slot, execute, active,
digest of the executed history, flags, per-type delivered counts) and totals."""
import json
import os

import pytest

from paxi_amd import abi
import oracle_lib as ol

pytestmark = pytest.mark.gpu
KATS = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "kats.json")))


def _sim():
    from paxi_amd.sim import Simulation
    return Simulation


def run_both(cfg, wl, fp=None, faults=(), steps=200, chunks=None):
    g = _sim()(cfg, wl, fp, faults)
    o = ol.OracleSim(cfg, wl, fp, faults)
    for n in (chunks or [steps]):
        g.step(n)
        o.step(n)
    return g, o


def assert_same(g, o, ctx=""):
    gs, os_ = g.read_state(), o.read_state()
    N = g.N
    for i in range(len(gs)):
        a, b = gs[i].as_tuple(), os_[i].as_tuple()
        assert a == b, f"{ctx} cluster {i // N} replica {i % N}:\n gpu={a}\n cpu={b}"
    gst, ost = g.stats().as_dict(), o.stats().as_dict()
    assert gst == ost, f"{ctx} stats\n gpu={gst}\n cpu={ost}"
    assert g.check() == o.check()
    return gst


def test_config1_kats_on_gpu():
    k = KATS["config1"]
    cfg = abi.make_config(npz=k["npz"], clusters=1, seed=1, max_delay=0)
    wl = abi.make_workload(outstanding=1, max_requests=k["writes"], target=0)
    g, o = run_both(cfg, wl, steps=3010)
    st = assert_same(g, o, "config1")
    assert st["delivered"] == k["delivered"] and st["delivered_total"] == k["delivered_total"]
    leader = g.read_state()[0]
    assert leader.ballot == k["leader_ballot"] and leader.slot == k["leader_slot"]
    assert leader.execute == k["leader_execute"] and leader.active == 1


@pytest.mark.parametrize("npz", [[3], [5], [3, 3, 3], [2, 2], [7]])
def test_faults_random_process(npz):
    cfg = abi.make_config(npz=npz, clusters=300, seed=42, window=16, mbox_cap=16, max_delay=4)
    wl = abi.make_workload(outstanding=8, target=0)
    fp = abi.make_fault_process(drop_ppm=3000, drop_len=25, slow_ppm=3000, slow_len=25, slow_min=1, slow_max=4)
    g, o = run_both(cfg, wl, fp, steps=400)
    st = assert_same(g, o, f"npz={npz}")
    assert st["dropped"] > 0 and st["commits"] > 0


def test_steps_per_launch_invariance():
    fp = abi.make_fault_process(drop_ppm=3000, drop_len=25, slow_ppm=3000, slow_len=25, slow_min=1, slow_max=4)
    wl = abi.make_workload(outstanding=8, target=0)
    res = []
    for S in (1, 7, 64):
        cfg = abi.make_config(npz=[5], clusters=130, seed=9, steps_per_launch=S)
        g = _sim()(cfg, wl, fp)
        g.step(100)
        g.step(57)
        res.append([s.as_tuple() for s in g.read_state()])
    assert res[0] == res[1] == res[2]


def test_sharding_by_cluster_base():
    """Global cluster ids key the PRNG: a split over two handles equals one handle."""
    wl = abi.make_workload(outstanding=4, target=0)
    fp = abi.make_fault_process(drop_ppm=3000, drop_len=25, slow_ppm=3000, slow_len=25, slow_min=1, slow_max=4)
    whole = _sim()(abi.make_config(npz=[5], clusters=200, seed=3), wl, fp)
    whole.step(150)
    a = _sim()(abi.make_config(npz=[5], clusters=77, seed=3), wl, fp)
    b = _sim()(abi.make_config(npz=[5], clusters=123, cluster_base=77, seed=3), wl, fp)
    a.step(150)
    b.step(150)
    w = [s.as_tuple() for s in whole.read_state()]
    assert w == [s.as_tuple() for s in a.read_state()] + [s.as_tuple() for s in b.read_state()]


def test_scripted_faults_crash_reelection():
    """Config-4 shape: FGrid 3x3, leader crash, ephemeral leader elsewhere."""
    cfg = abi.make_config(npz=[3, 3, 3], clusters=128, seed=5, q1=abi.Q_FGRID_Q1, q2=abi.Q_FGRID_Q2, fz=1,
                          ephemeral_leader=1, mbox_cap=24)
    wl = abi.make_workload(outstanding=4, target=[0, 0, 3, 3])
    faults = [abi.make_fault(abi.FAULT_CRASH, 0, step_from=60),
              abi.make_fault(abi.FAULT_FLAKY, 4, dst=abi.ALL_DST, param=100000, step_from=10, step_to=200),
              abi.make_fault(abi.FAULT_DROP, 5, dst=1, step_from=30, step_to=90),
              abi.make_fault(abi.FAULT_SLOW, 6, dst=abi.ALL_DST, param=3, step_from=0, step_to=300)]
    g, o = run_both(cfg, wl, None, faults, chunks=[50, 150, 100])
    st = assert_same(g, o, "crash")
    assert st["discarded"] > 0


@pytest.mark.parametrize("q", [(abi.Q_GRID_ROW, abi.Q_GRID_COLUMN, 0), (abi.Q_FGRID_Q1, abi.Q_FGRID_Q2, 2),
                               (abi.Q_ZONE_MAJORITY, abi.Q_ZONE_MAJORITY, 0), (abi.Q_ALL, abi.Q_FAST, 0)])
def test_quorum_kinds(q):
    cfg = abi.make_config(npz=[3, 3, 3], clusters=96, seed=11, q1=q[0], q2=q[1], fz=q[2], ephemeral_leader=1)
    wl = abi.make_workload(outstanding=6, target=[0, 4, 8])
    fp = abi.make_fault_process(drop_ppm=2000, drop_len=15, slow_ppm=2000, slow_len=15, slow_min=1, slow_max=3)
    g, o = run_both(cfg, wl, fp, steps=300)
    assert_same(g, o, f"q={q}")


@pytest.mark.parametrize("opt", ["thrifty", "rwc", "forwarding"])
def test_options(opt):
    kw = dict(npz=[5], clusters=100, seed=21)
    wl = abi.make_workload(outstanding=5, target=0)
    if opt == "thrifty":
        kw["thrifty"] = 1
    elif opt == "rwc":
        kw["reply_when_commit"] = 1
    else:
        wl = abi.make_workload(outstanding=6, target=[0, 1, 2, 3, 4, 2])
    fp = abi.make_fault_process(drop_ppm=2000, drop_len=15, slow_ppm=2000, slow_len=15, slow_min=1, slow_max=4)
    g, o = run_both(abi.make_config(**kw), wl, fp, steps=300)
    assert_same(g, o, opt)


def test_edge_small_window_and_mailbox():
    """Tight W and M force window/mailbox overflow paths; flags must agree."""
    cfg = abi.make_config(npz=[5], clusters=200, seed=77, window=8, mbox_cap=8, max_delay=6)
    wl = abi.make_workload(outstanding=8, target=0)
    fp = abi.make_fault_process(drop_ppm=5000, drop_len=40, slow_ppm=8000, slow_len=30, slow_min=2, slow_max=6)
    g, o = run_both(cfg, wl, fp, steps=400)
    st = assert_same(g, o, "tight")
    assert st["flagged"][0] > 0  # window overflow exercised


def test_single_cluster_and_ragged_tail():
    """1 cluster and 65 clusters (one full tile + a 1-lane ragged tile)."""
    for n in (1, 65):
        cfg = abi.make_config(npz=[5], clusters=n, seed=123)
        wl = abi.make_workload(outstanding=3, target=0)
        g, o = run_both(cfg, wl, steps=120)
        assert_same(g, o, f"C={n}")


def test_oversized_workgroup_image_is_refused():
    """16 replicas with 15-step delays need 174 KB of mailbox counts in LDS: EUNSUPP, not a crash."""
    from paxi_amd.sim import PaxisimError
    with pytest.raises(PaxisimError, match="exceeds LDS"):
        _sim()(abi.make_config(npz=[16], clusters=64, max_delay=14), abi.make_workload())


def test_window64_n9():
    """N=9 with SURVEY 8's 64-slot window: the serial kernel keeps the windows in
    HBM (the replica-per-wave kernel's 160 KB of LDS could not hold them)."""
    cfg = abi.make_config(npz=[3, 3, 3], clusters=130, seed=6, window=64, q1=abi.Q_FGRID_Q1, q2=abi.Q_FGRID_Q2, fz=1)
    wl = abi.make_workload(outstanding=8, target=0)
    fp = abi.make_fault_process(drop_ppm=3000, drop_len=25, slow_ppm=3000, slow_len=25, slow_min=1, slow_max=4)
    g, o = run_both(cfg, wl, fp, steps=300)
    assert_same(g, o, "N=9 W=64")


def test_window32_n5():
    """W=32 still fits at N=5 (one workgroup per CU)."""
    cfg = abi.make_config(npz=[5], clusters=200, seed=4, window=32)
    wl = abi.make_workload(outstanding=8, target=0)
    fp = abi.make_fault_process(drop_ppm=3000, drop_len=25, slow_ppm=3000, slow_len=25, slow_min=1, slow_max=4)
    g, o = run_both(cfg, wl, fp, steps=300)
    assert_same(g, o, "W=32")


def test_late_workers_crash_failover():
    """Config-4 shape: clients turn from the crashed leader 1.1 to 2.1 (start_step), FGrid fz=1."""
    cfg = abi.make_config(npz=[3, 3, 3], clusters=130, seed=8, q1=abi.Q_FGRID_Q1, q2=abi.Q_FGRID_Q2, fz=1,
                          ephemeral_leader=1, mbox_cap=24, max_delay=0)
    wl = abi.make_workload(outstanding=8, target=[0, 0, 0, 0, 3, 3, 3, 3], start_step=[0, 0, 0, 0, 90, 90, 90, 90])
    g, o = run_both(cfg, wl, None, [abi.make_fault(abi.FAULT_CRASH, 0, step_from=90)], chunks=[60, 60, 120])
    st = assert_same(g, o, "failover")
    s = g.read_state()
    assert st["discarded"] > 0 and all(s[c * 9 + 3].active == 1 for c in range(130))


def test_inject_and_read_log():
    """Injected client requests (http.go:99) and the log windows, entry by entry."""
    cfg = abi.make_config(npz=[5], clusters=70, seed=13, window=16, mbox_cap=16, max_delay=3, ephemeral_leader=1)
    wl = abi.make_workload(outstanding=2, target=0, max_requests=40)
    fp = abi.make_fault_process(drop_ppm=20000, drop_len=5, slow_ppm=20000, slow_len=5, slow_min=1, slow_max=3)
    g = _sim()(cfg, wl, fp)
    o = ol.OracleSim(cfg, wl, fp)
    cid = 1 << 20
    for step in range(12):
        for c in range(0, 70, 3):
            r = (c + step) % 5
            g.inject(c, r, cid)
            o.inject(c, r, cid)
            cid += 1
        g.step(9)
        o.step(9)
    assert_same(g, o, "inject")
    for c in range(0, 70, 7):
        for r in range(5):
            e = min(x.execute for x in o.read_state(c, 1))
            a = [x.as_tuple() for x in g.read_log(c, r, e - 2, 20)]
            b = [x.as_tuple() for x in o.read_log(c, r, e - 2, 20)]
            assert a == b, f"cluster {c} replica {r}"
