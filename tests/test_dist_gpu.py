"""Multi-GPU through the C-ABI (paxisim_dist_*, RCCL): on a one-GPU box the
communicators have one member, which still runs the whole path — RCCL
opened at run time, the all-reduce on the handle's stream, stats packing."""
import pytest

from paxi_amd import abi

pytestmark = pytest.mark.gpu


def _sim(clusters=200, base=0):
    from paxi_amd.sim import Simulation
    cfg = abi.make_config(npz=[5], clusters=clusters, cluster_base=base, seed=42, mbox_cap=32)
    fp = abi.make_fault_process(drop_ppm=3000, drop_len=25, slow_ppm=3000, slow_len=25, slow_min=1, slow_max=4)
    return Simulation(cfg, abi.make_workload(outstanding=8, target=0), fp)


def test_dist_clique_one_handle():
    from paxi_amd.sim import Dist
    s = _sim()
    s.step(120)
    d = Dist([s])
    tot, ms = d.stats()
    assert tot.as_dict() == s.stats().as_dict()
    assert ms == pytest.approx(s.kernel_time()[0])
    sums, maxes = d.allreduce([[1, 2, 3, 1 << 40]], [[2.5, -1.0]])
    assert sums == [1, 2, 3, 1 << 40] and maxes == [2.5, -1.0]
    d.close()


def test_dist_rank_communicator():
    """paxisim_dist_unique_id + paxisim_dist_init_rank, as bench.py --gpus N uses them per rank."""
    from paxi_amd import dist as pdist
    from paxi_amd.sim import Dist
    s = _sim(clusters=130, base=1000)
    s.step(90)
    d = Dist.join(s, Dist.unique_id(), 1, 0)
    vals = pdist.stats_counters({"delivered_total": 7, "commits": 3, "replies": 2, "dropped": 1,
                                 "client_requests": 5}, 11, 0, [0] * 8, active=130)
    tot, maxes = pdist.reduce_counters_abi(d, vals, [0.25, 3.0])
    assert tot["delivered_total"] == 7 and tot["alg_bytes"] == 11 and tot["active"] == 130 and maxes == [0.25, 3.0]
    assert d.stats()[0].as_dict() == s.stats().as_dict()
    d.close()
