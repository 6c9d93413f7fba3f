"""A step's replica-steps are independent: every send lands in
a bucket of a later step, and every box has one writer (a socket box its
source replica, a client box the worker's target replica).  (The device drains
the agreement-ring arrivals in replica order after the step; the oracle applies
them as they come, which only decides whose digest a checkpoint records first.)  The serial
kernel's busiest-first order (sim_core.h replica_order) rests
on this: each lane may run its cluster's replicas in any order.  GPU parity
pins the kernel to the oracle in index order; this CPU test pins the oracle's
index order to other orders - reversed, and shuffled per (cluster, step) - on
the bench's own workloads (configs 2-5, built by bench.workload, with their
faults), comparing every replica state, every per-key instance, the Databases
and the ABD op histories."""
import argparse
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from paxi_amd import abi  # noqa: E402
import oracle_lib as ol  # noqa: E402

CLUSTERS = 192
THREADS = min(8, os.cpu_count() or 1)


def run(cfg_id, order, steps, fz=1):
    a = argparse.Namespace(window=None, mbox=None, kv=1, history=512, clusters=CLUSTERS, sim_steps=None,
                           warmup=2, steps=20, crash_step=None, fz=fz)
    for k, v in bench.DEFAULTS[cfg_id].items():
        if getattr(a, k, None) is None:
            setattr(a, k, v)
    a.crash_step = 300                                   # inside the run: the re-election path is covered
    cfg, wl, fp, faults, _ = bench.workload(cfg_id, CLUSTERS, 0, 0, a)
    o = ol.OracleSim(cfg, wl, fp, faults)
    o.set_replica_order(order)
    o.step(steps, threads=THREADS)
    N = abi.n_replicas(cfg)
    out = {"state": [r.as_tuple() for r in o.read_state()]}
    if cfg.protocol in abi.PER_KEY:
        out["inst"] = [i.as_tuple() for i in o.read_instances()]
    if cfg.protocol == abi.ABD:
        out["hist"] = [o.history(c) for c in range(0, CLUSTERS, 7)]
    elif cfg.kv:
        out["kv"] = [o.read_kv(c, r, cfg.keys) for c in range(0, CLUSTERS, 11) for r in range(N)]
    out["delivered"] = sum(sum(r.delivered) for r in o.read_state())
    o.close()
    return out


@pytest.mark.parametrize("cfg_id,steps,fz", [(2, 1200, 1), (3, 400, 1), (4, 900, 1), (4, 900, 0), (5, 900, 1)])
def test_replica_order_does_not_change_the_step(cfg_id, steps, fz):
    base = run(cfg_id, 0, steps, fz)
    assert base["delivered"] > 0
    for order in (1, 2):
        other = run(cfg_id, order, steps, fz)
        for k in base:
            assert other[k] == base[k], f"config {cfg_id} fz={fz}: {k} differs with replica order {order}"


def test_bad_order_mode_is_rejected():
    cfg = abi.make_config(npz=[3], clusters=2)
    o = ol.OracleSim(cfg, abi.make_workload())
    with pytest.raises(RuntimeError):
        o.set_replica_order(3)
    o.close()
