"""The bounded model's faithfulness at the window the bench uses (round-3
verdict item 6).

Go's log is a map: unbounded.  The simulator keeps a window of W slots per
instance and flags every place where the bound could change behaviour
(WOVF / GHOST mark that the bound was touched, UNFAITHFUL that it may have
been observed).  The claim the headline rests on is "a cluster without
UNFAITHFUL behaves exactly as with an unbounded log".  GPU-vs-oracle parity
cannot test it - both sides implement the same bound - so this test runs the
oracle twice on the bench's own workloads (configs 2, 4 and 5, built by
bench.workload), at the bench's window W = 16 and at W = 64, over the bench's
whole horizon, and asserts that every cluster unflagged at W = 16 has the same
replica states (flags aside from WOVF / GHOST) and the same instances at W = 64.
Configs 2, 4 and 5 run at 512 clusters each (CPU only)."""
import argparse
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from paxi_amd import abi  # noqa: E402
import oracle_lib as ol  # noqa: E402

WINDOW_FLAGS = abi.F_WOVF | abi.F_GHOST
CLUSTERS = 512
THREADS = min(8, os.cpu_count() or 1)


def run(cfg_id, window, steps, fz=1):
    a = argparse.Namespace(window=window, mbox=None, kv=1, history=512, clusters=CLUSTERS, sim_steps=None,
                           warmup=5, steps=20, crash_step=None, fz=fz)
    for k, v in bench.DEFAULTS[cfg_id].items():
        if getattr(a, k, None) is None:
            setattr(a, k, v)
    a.crash_step = a.warmup * a.sim_steps
    cfg, wl, fp, faults, _ = bench.workload(cfg_id, CLUSTERS, 0, 0, a)
    o = ol.OracleSim(cfg, wl, fp, faults)
    o.step(steps, threads=THREADS)
    st = [r.as_tuple() for r in o.read_state()]
    inst = [i.as_tuple() for i in o.read_instances()] if cfg.protocol in abi.PER_KEY else None
    N, I = abi.n_replicas(cfg), abi.n_instances(cfg)
    o.close()
    return st, inst, N, I


def strip(t):
    """A replica state tuple without the window-bound flags (index 4 = flags)."""
    return t[:4] + (t[4] & ~WINDOW_FLAGS,) + t[5:]


@pytest.mark.parametrize("cfg_id,steps,fz,w", [(2, 10_000, 1, 16), (4, 5_000, 1, 16), (4, 5_000, 0, 16),
                                              (5, 5_000, 1, 16), (4, 5_000, 1, 8), (5, 5_000, 1, 8)])
def test_unflagged_clusters_equal_a_wider_window(cfg_id, steps, fz, w):
    """Also W = 8 for configs 4 and 5, which never reach the bound there (round 6: config 5's
    bench runs at W = 8)."""
    s16, i16, N, I = run(cfg_id, w, steps, fz)
    s64, i64, _, _ = run(cfg_id, 64, steps, fz)
    faithful = touched = 0
    for c in range(CLUSTERS):
        reps16, reps64 = s16[c * N:(c + 1) * N], s64[c * N:(c + 1) * N]
        if any(r[4] & abi.F_UNFAITHFUL for r in reps16):
            continue
        faithful += 1
        touched += any(r[4] & WINDOW_FLAGS for r in reps16)
        assert [strip(r) for r in reps16] == [strip(r) for r in reps64], f"cluster {c}"
        if i16 is not None:
            assert i16[c * N * I:(c + 1) * N * I] == i64[c * N * I:(c + 1) * N * I], f"cluster {c} instances"
    print(f"config {cfg_id} fz={fz}: {faithful}/{CLUSTERS} clusters unflagged at W={w}, "
          f"{touched} of them touched the window bound (WOVF/GHOST)")
    assert faithful >= CLUSTERS // 2
    if cfg_id == 2:
        assert touched > 0        # the comparison covers clusters that hit the bound
