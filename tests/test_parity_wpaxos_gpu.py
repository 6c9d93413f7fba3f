"""GPU parity for WPaxos (BASELINE config 5 semantics): the HIP path through the
C-ABI against the CPU oracle on the same seeded inputs — bit-exact per-replica
state, per-(replica, key) kpaxos instance state, totals and the agreement scan."""
import pytest

from paxi_amd import abi
import oracle_lib as ol

pytestmark = pytest.mark.gpu


def _sim():
    from paxi_amd.sim import Simulation
    return Simulation


def wp_config(clusters, keys=8, seed=5, **kw):
    kw.setdefault("window", 16)
    kw.setdefault("mbox_cap", 24)
    kw.setdefault("max_delay", 0)
    kw.setdefault("policy_threshold", 3)
    return abi.make_config(protocol=abi.WPAXOS, npz=kw.pop("npz", [3, 3, 3]), keys=keys, clusters=clusters,
                           seed=seed, **kw)


def run_and_compare(cfg, wl, fp=None, faults=(), chunks=(300,)):
    g = _sim()(cfg, wl, fp, faults)
    o = ol.OracleSim(cfg, wl, fp, faults)
    for n in chunks:
        g.step(n)
        o.step(n)
    N = g.N
    gs, os_ = g.read_state(), o.read_state()
    for i in range(len(gs)):
        assert gs[i].as_tuple() == os_[i].as_tuple(), f"cluster {i // N} replica {i % N}"
    gi, oi = g.read_instances(), o.read_instances()
    K = abi.n_instances(cfg)
    for i in range(len(gi)):
        assert gi[i].as_tuple() == oi[i].as_tuple(), f"cluster {i // (N * K)} replica {i // K % N} key {i % K}"
    gst, ost = g.stats().as_dict(), o.stats().as_dict()
    assert gst == ost
    assert g.check() == o.check()
    g.close()
    return gst


def test_config5_shape_locality70():
    wl = abi.make_workload(outstanding=9, target=list(range(9)), locality_ppm=700_000)
    st = run_and_compare(wp_config(200), wl, chunks=(150, 173))
    assert st["commits"] > 0 and st["delivered"].get("LeaderChange", 0) > 0


@pytest.mark.parametrize("fz", [0, 1, 2])
def test_faults_and_fgrid(fz):
    wl = abi.make_workload(outstanding=9, target=list(range(9)), locality_ppm=700_000)
    fp = abi.make_fault_process(drop_ppm=2000, drop_len=20, slow_ppm=2000, slow_len=20, slow_min=1, slow_max=3)
    st = run_and_compare(wp_config(130, fz=fz, max_delay=3), wl, fp, chunks=(200, 101))
    assert st["dropped"] > 0


def test_leader_crash_and_scripted_faults():
    wl = abi.make_workload(outstanding=6, target=[0, 3, 6, 1, 4, 7], locality_ppm=700_000)
    faults = [abi.make_fault(abi.FAULT_CRASH, 0, step_from=60, step_to=160),
              abi.make_fault(abi.FAULT_FLAKY, 3, dst=abi.ALL_DST, param=200_000, step_from=0, step_to=300),
              abi.make_fault(abi.FAULT_SLOW, 6, dst=7, param=2, step_from=20, step_to=120)]
    run_and_compare(wp_config(100, max_delay=2), wl, faults=faults, chunks=(250,))


@pytest.mark.parametrize("adaptive,thr", [(0, 3), (1, 0), (1, 1)])
def test_policy_modes(adaptive, thr):
    wl = abi.make_workload(outstanding=9, target=list(range(9)), locality_ppm=500_000)
    run_and_compare(wp_config(96, adaptive=adaptive, policy_threshold=thr), wl, chunks=(200,))


def test_single_key_uniform_and_thrifty():
    wl = abi.make_workload(outstanding=4, target=[0, 4, 8, 2])
    run_and_compare(wp_config(70, keys=1, thrifty=1), wl, chunks=(200,))


def test_two_zones_many_keys_tight_window():
    wl = abi.make_workload(outstanding=8, target=[0, 1, 2, 3], locality_ppm=800_000)
    run_and_compare(wp_config(65, keys=32, npz=[2, 2], window=8, mbox_cap=8), wl, chunks=(240,))


def test_reference_gap_reproduced_on_gpu():
    """The seeded divergence of test_oracle_wpaxos's KAT also appears on the GPU."""
    wl = abi.make_workload(outstanding=9, target=list(range(9)), locality_ppm=700_000)
    fp = abi.make_fault_process(drop_ppm=2000, drop_len=20, slow_ppm=2000, slow_len=20, slow_min=1, slow_max=3)
    g = _sim()(wp_config(1, seed=7, cluster_base=26, max_delay=3), wl, fp)
    g.step(10)
    assert g.check() == 1
    g.close()


@pytest.mark.parametrize("dist", [dict(distribution="zipfan"), dict(distribution="order"),
                                  dict(distribution="conflict", conflicts=25)])
def test_key_distributions(dist):
    """WPaxos with the benchmark's key distributions (benchmark.go:202-233),
    with and without zone locality."""
    cfg = wp_config(160, keys=7)
    for loc in (0, 500_000):
        wl = abi.make_workload(outstanding=6, target=[0, 3, 6, 1, 4, 7], locality_ppm=loc, keys=7, **dist)
        run_and_compare(cfg, wl, chunks=(120, 80))


@pytest.mark.parametrize("policy,kw", [(abi.POLICY_MAJORITY, dict(policy_interval=1)),
                                       (abi.POLICY_MAJORITY, dict(policy_interval=25)),
                                       (abi.POLICY_EMA, dict(policy_alpha=0.3)),
                                       (abi.POLICY_EMA, dict(policy_alpha=0.85))])
def test_majority_and_ema_policies(policy, kw):
    """majority / ema leader migration (policy.go:71-130) with the step as the
    clock: instance state incl. the policy state is bit-exact."""
    cfg = wp_config(192, keys=6, policy=policy, **kw)
    wl = abi.make_workload(outstanding=9, target=list(range(9)), locality_ppm=600_000)
    fp = abi.make_fault_process(drop_ppm=2000, drop_len=20)
    st = run_and_compare(cfg, wl, fp, chunks=(250, 150))
    assert st["delivered"]["LeaderChange"] > 0


@pytest.mark.parametrize("wlds,wcoloc", [("0", "0"), ("1", "0"), ("0", "1")])
def test_both_instance_layouts(wlds, wcoloc, monkeypatch):
    """The serial kernel's homes for the kpaxos scalars - the packed HBM
    table (default since round 4), the tile image's word planes
    (PAXISIM_WLDS=1) and (round 6, PAXISIM_WCOLOC=1) one block per instance
    holding its scalars and its window - under faults, with the Database on:
    all equal the oracle.  (Round 3's first serial WPaxos build lost instance
    state between replica-steps; this keeps every layout under test.)"""
    monkeypatch.setenv("PAXISIM_WLDS", wlds)
    monkeypatch.setenv("PAXISIM_WCOLOC", wcoloc)
    wl = abi.make_workload(outstanding=9, target=list(range(9)), locality_ppm=700_000, write_ppm=600_000)
    fp = abi.make_fault_process(drop_ppm=1000, drop_len=10, slow_ppm=2000, slow_len=10, slow_min=1, slow_max=2)
    st = run_and_compare(wp_config(130, max_delay=2, kv=1), wl, fp, chunks=(120, 97))
    assert st["commits"] > 0
