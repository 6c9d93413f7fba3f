"""GPU parity for ABD (abd/replica.go): replica KV digests, op counters,
per-type message counts, the recorded op histories and the linearizability
scan (checker.go) are bit-exact against the CPU oracle."""
import pytest

from paxi_amd import abi
import oracle_lib as ol

pytestmark = pytest.mark.gpu


def make(clusters, npz=(5,), outstanding=4, target=(0, 1, 2, 3), write_ppm=500_000, keys=8, history=64, seed=13,
         fp=None, faults=(), **dist):
    from paxi_amd.sim import Simulation
    cfg = abi.make_config(protocol=abi.ABD, npz=list(npz), clusters=clusters, seed=seed, keys=keys, history=history)
    wl = abi.make_workload(outstanding=outstanding, target=list(target), write_ppm=write_ppm, keys=keys, **dist)
    return Simulation(cfg, wl, fp, faults), ol.OracleSim(cfg, wl, fp, faults)


def same(g, o, steps, hist_clusters=8):
    for n in steps:
        g.step(n)
        o.step(n)
    gs, os_ = g.read_state(), o.read_state()
    for i in range(len(gs)):
        assert gs[i].as_tuple() == os_[i].as_tuple(), f"replica record {i}"
    assert g.stats().as_dict() == o.stats().as_dict()
    for c in range(min(hist_clusters, g.cfg.clusters)):
        assert g.history(c) == o.history(c), f"history of cluster {c}"
    a, n, skipped = g.linearizable()
    oa, on = o.linearizable()
    assert skipped == 0 and (a, n) == (oa, on)
    return a, n


def test_abd_no_faults():
    g, o = make(300)
    a, n = same(g, o, [100, 60])
    assert n > 0 and a > 0          # concurrent coordinators: versioning anomalies (abd/replica.go:123)


def test_abd_single_coordinator_is_linearizable():
    g, o = make(200, target=(2,))
    a, n = same(g, o, [150])
    assert n > 0 and a == 0


@pytest.mark.parametrize("npz", [(3,), (5,), (2, 2, 3)])
def test_abd_with_faults(npz):
    fp = abi.make_fault_process(drop_ppm=3000, drop_len=20, slow_ppm=3000, slow_len=20, slow_min=1, slow_max=4)
    faults = [abi.make_fault(abi.FAULT_CRASH, 1, step_from=40, step_to=90),
              abi.make_fault(abi.FAULT_FLAKY, 0, param=200_000, step_from=0, step_to=120)]
    g, o = make(256, npz=npz, target=(0, 1, 2, 0), fp=fp, faults=faults)
    same(g, o, [70, 80])


@pytest.mark.parametrize("dist", [dict(distribution="order"), dict(distribution="conflict", conflicts=40),
                                  dict(distribution="zipfan"), dict(distribution="normal", mu=3.0, sigma=5.0),
                                  dict(distribution="exponential", lam=0.3)])
def test_abd_key_distributions(dist):
    """Bconfig.Distribution (benchmark.go:202-233): the GPU's key draws, and so
    every op, history and the linearizability scan, match the oracle."""
    g, o = make(192, keys=13, **dist)
    same(g, o, [90, 40])


def test_history_export_from_device(tmp_path):
    """paxi_amd.history over the device's records equals the oracle's, and
    WriteFile output (history.go:74-113) is byte-identical."""
    from paxi_amd.history import History
    g, o = make(16, keys=4, history=128)
    same(g, o, [400])

    class _O:
        cfg = g.cfg

        def history(self, c):
            return o.history(c)
    hg, ho = History.from_simulation(g), History.from_simulation(_O())
    for c, (a, b) in enumerate(zip(hg, ho)):
        a.write_file(str(tmp_path / f"g{c}"))
        b.write_file(str(tmp_path / f"o{c}"))
        assert (tmp_path / f"g{c}.csv").read_text() == (tmp_path / f"o{c}.csv").read_text()
        assert len(a.operations) > 10


def test_history_straight_after_step():
    """paxisim_history right after paxisim_step, with no other read between:
    the read must wait for the step kernels on the handle's stream."""
    g, o = make(4096, keys=4, history=64)
    g.step(120)
    o.step(120)
    for c in (0, 2047, 4095):
        assert g.history(c) == o.history(c)
