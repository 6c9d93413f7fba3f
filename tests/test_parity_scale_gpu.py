"""Parity at the benchmarked scale and regime (round-2 verdict item 2): each
BASELINE config is built exactly as bench.workload builds it, at its full
per-GPU cluster count, run over the whole horizon the bench times (config 2:
10,000 steps with compaction; 3: 2,000; 4 and 5: 5,000), and at least 256
sampled clusters - random ones, WOVF- and GHOST-flagged ones and frozen ones -
are rerun on the oracle and compared bit for bit (tests/parity_sample.py)."""
import argparse
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import parity_sample  # noqa: E402

pytestmark = pytest.mark.gpu

# (config, bench steps incl. warm-up = the driver's --warmup 5 --steps 20)
HORIZON = {2: 25, 3: 25, 4: 25, 5: 25}


def bench_args(cfg_id, fz=1):
    a = argparse.Namespace(window=None, mbox=None, kv=1, history=512, clusters=None, sim_steps=None, warmup=5,
                           steps=20, crash_step=None, fz=fz)
    for k, v in bench.DEFAULTS[cfg_id].items():
        if getattr(a, k, None) is None:
            setattr(a, k, v)
    a.crash_step = a.warmup * a.sim_steps
    return a


@pytest.mark.parametrize("cfg_id,fz", [(2, 1), (3, 1), (4, 1), (4, 0), (5, 1)])
def test_sampled_parity_at_scale(cfg_id, fz):
    """fz applies to config 4: FGrid fz=1, or (fz=0) the Grid variant GridRow/GridColumn."""
    from paxi_amd.sim import Simulation
    a = bench_args(cfg_id, fz)
    cfg, wl, fp, faults, _ = bench.workload(cfg_id, a.clusters, 0, 0, a)
    steps = HORIZON[cfg_id] * a.sim_steps
    sim = Simulation(cfg, wl, fp, faults)
    for _ in range(HORIZON[cfg_id]):
        sim.step(a.sim_steps)
    sim.sync()
    picks = parity_sample.choose(sim)
    res = parity_sample.check(sim, cfg, wl, fp, faults, steps, picks)
    sim.close()
    print(f"config {cfg_id} (fz={fz}): {res}")
    assert res["compared"] >= 256
    assert res["equal"] == res["compared"], res["mismatches"]
    if cfg_id == 2:   # the timed regime: flagged and frozen clusters are in the sample
        assert res["by_kind"]["wovf"] > 0 and res["by_kind"]["ghost"] > 0 and res["by_kind"]["frozen"] > 0
