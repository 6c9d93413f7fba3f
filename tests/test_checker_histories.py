"""checker_test.go:6-136 through the simulator's own history path: each of the
reference's 10 histories is loaded into an ABD handle (History.ReadFile,
history.go:115-178 -> paxisim_history_load) and checked by
History.Linearizable (history.go:55-71).  The oracle runs here; the GPU
lin_kernel runs under -m gpu.  Expected anomaly counts are the reference
test's own assertions (tests/golden/kats.json "checker")."""
import pytest

from paxi_amd import abi
import oracle_lib as ol
from test_oracle_kats import KATS

CASES = KATS["checker"]


def as_ops(case):
    """(input, output, start, end) -> (key, is_write, value, start, end)."""
    ops = []
    for i, o, s, e in case["ops"]:
        ops.append((0, 1, i, s, e) if i is not None else (0, 0, o, s, e))
    return ops


def expected(case, n):
    e = case["expect"]
    return n == 0 if e == "zero" else (n > 0 if e == "nonzero" else n == e)


def cfg_for(clusters):
    cfg = abi.make_config(protocol=abi.ABD, npz=[3], clusters=clusters, keys=1, history=16)
    return cfg, abi.make_workload(outstanding=1, max_requests=1, target=[0])


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_checker_history_oracle(case):
    sim = ol.OracleSim(*cfg_for(1))
    sim.history_load(0, 0, as_ops(case))
    a, n = sim.linearizable()
    assert n == len(case["ops"]) and expected(case, a)
    assert a == ol.linearizable([tuple(o) for o in case["ops"]])


def test_history_load_validates():
    sim = ol.OracleSim(*cfg_for(1))
    with pytest.raises(RuntimeError):
        sim.history_load(0, 0, [(0, 1, 1, 0, 1)] * 17)      # beyond history capacity
    with pytest.raises(RuntimeError):
        sim.history_load(0, 3, [(0, 1, 1, 0, 1)])           # replica out of range


@pytest.mark.gpu
def test_checker_histories_gpu():
    """All 10 histories at once, one per cluster (spread over replicas), on the
    GPU lin_kernel: per-case anomaly counts equal the reference test's and
    the oracle's."""
    from paxi_amd.sim import Simulation
    for case in CASES:
        g = Simulation(*cfg_for(3))
        o = ol.OracleSim(*cfg_for(3))
        ops = as_ops(case)
        # the same history split over two replicas of cluster 1 (canonical
        # order: replica 0's ops, then replica 1's) and whole in cluster 2
        for s in (g, o):
            s.history_load(1, 0, ops[: len(ops) // 2])
            s.history_load(1, 1, ops[len(ops) // 2:])
            s.history_load(2, 2, ops)
        ga, gn, gsk = g.linearizable()
        oa, on = o.linearizable()
        assert gsk == 0 and (ga, gn) == (oa, on) == (oa, 2 * len(ops)), case["name"]
        single = ol.linearizable([tuple(x) for x in case["ops"]])
        assert ga == 2 * single and expected(case, single), case["name"]
        g.close()
