"""Multi-process path of paxi_amd.dist on the CPU: world_size 2 over gloo.

The GPU kernel cannot run here, so each rank drives the CPU oracle on its own
cluster shard (the oracle stands in for the device in this test only).  Checks
that range sharding + PRNG keyed by global cluster id + the all-reduce of
counters reproduce the unsharded run exactly."""
import os
import socket

import pytest
import torch.multiprocessing as mp

from paxi_amd import abi
from paxi_amd import dist as pdist

PER_RANK = 48
STEPS = 150


def _cfg(clusters, base):
    cfg = abi.make_config(npz=[5], clusters=clusters, cluster_base=base, seed=17)
    wl = abi.make_workload(outstanding=4, target=0)
    fp = abi.make_fault_process(drop_ppm=3000, drop_len=20, slow_ppm=3000, slow_len=20, slow_min=1, slow_max=4)
    return cfg, wl, fp


def _counters(sim):
    st = sim.stats().as_dict()
    d = {k: st[k] for k in ("delivered_total", "commits", "replies", "dropped", "client_requests")}
    return pdist.stats_counters(d, 0, sim.check(), st["flagged"], agree_compared=st["agree_compared"],
                                agree_missed=st["agree_missed"], active=sim.cfg.clusters,
                                active_start=sim.cfg.clusters)


def _worker(rank, world, port, q):
    import torch.distributed as dist
    import oracle_lib
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    base, n = pdist.shard(PER_RANK, rank)
    sim = oracle_lib.OracleSim(*_cfg(n, base))
    sim.step(STEPS)
    tot, (tmax,) = pdist.reduce_counters(_counters(sim), [float(rank + 1)])
    states = [s.as_tuple() for s in sim.read_state()]
    q.put((rank, tot, tmax, states))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_ranges():
    assert [pdist.shard(100, r) for r in range(3)] == [(0, 100), (100, 100), (200, 100)]


@pytest.mark.timeout(300)
def test_two_rank_gloo_matches_single_process():
    import oracle_lib
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in procs])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    whole = oracle_lib.OracleSim(*_cfg(2 * PER_RANK, 0))
    whole.step(STEPS)
    want = _counters(whole)
    for rank, tot, tmax, _ in res:
        assert tmax == 2.0                                   # max over ranks
        assert {k: int(v) for k, v in tot.items()} == {k: int(v) for k, v in want.items()}
    assert res[0][3] + res[1][3] == [s.as_tuple() for s in whole.read_state()]
