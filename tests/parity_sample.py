"""Sampled GPU-vs-oracle parity at BASELINE scale (test infrastructure: the
oracle is the checker here, never the thing measured).

A batch of a BASELINE config runs on the GPU over its whole horizon; a sample
of its clusters is then rerun one by one on the oracle (each as a one-cluster
handle with cluster_base = its global id: the PRNG and the scripted faults are
keyed by global id, so the oracle computes the same trajectory) and compared
replica by replica (paxisim_read_state), instance by instance for the per-key
protocols (read_instances) and op by op for ABD (paxisim_history).  The
sample mixes clusters chosen at random with clusters that carry the bounded
model's flags (WOVF, GHOST: the rules of DESIGN.md §3.6 at work) and
clusters that compaction froze (paxisim_read_activity), so that every regime
the timed region contains is in it.  The reference is paxos/paxos.go:86-376,
abd/replica.go:50-157 and wpaxos/replica.go:42-108 as the oracle restates them.
"""
import concurrent.futures
import os
import random

from paxi_amd import abi
import oracle_lib as ol

F_WOVF, F_GHOST = 0x01, 0x02


def cluster_flags(states, N):
    out = []
    for c in range(len(states) // N):
        f = 0
        for r in range(N):
            f |= states[c * N + r].flags
        out.append(f)
    return out


def choose(sim, n_random=256, n_flag=64, n_frozen=32, scan=65536, seed=7):
    """{category: [local cluster ids]} drawn from the GPU handle's state."""
    C = sim.cfg.clusters
    rng = random.Random(seed)
    lo = rng.randrange(0, max(1, C - scan + 1))
    n = min(scan, C)
    flags = cluster_flags(sim.read_state(lo, n), sim.N)
    act = sim.activity(lo, n)
    pick = {
        "random": sorted(rng.sample(range(C), min(n_random, C))),
        "wovf": [lo + i for i, f in enumerate(flags) if f & F_WOVF][:n_flag],
        "ghost": [lo + i for i, f in enumerate(flags) if f & F_GHOST][:n_flag],
        "frozen": [lo + i for i, a in enumerate(act) if a is not None][:n_frozen],
    }
    return pick


def _one(cfg, wl, fp, faults, gid, steps, per_key, abd):
    c = abi.Config.from_buffer_copy(cfg)
    c.clusters = 1
    c.cluster_base = gid
    o = ol.OracleSim(c, wl, fp, faults)
    o.step(steps)
    st = [s.as_tuple() for s in o.read_state()]
    inst = [i.as_tuple() for i in o.read_instances()] if per_key else None
    hist = o.history(0) if abd else None
    o.close()
    return st, inst, hist


def check(sim, cfg, wl, fp, faults, steps, picks, threads=None):
    """Rerun every picked cluster on the oracle to `steps` (the GPU handle must
    be at that step) and compare.  Returns a summary dict."""
    per_key = cfg.protocol in (abi.WPAXOS, abi.M2PAXOS, abi.KPAXOS)
    abd = cfg.protocol == abi.ABD and cfg.history > 0
    cl = sorted(set(c for v in picks.values() for c in v))
    base = cfg.cluster_base
    threads = threads or min(16, os.cpu_count() or 1)
    with concurrent.futures.ThreadPoolExecutor(threads) as ex:
        futs = {c: ex.submit(_one, cfg, wl, fp, faults, base + c, steps, per_key, abd) for c in cl}
        got = {c: f.result() for c, f in futs.items()}
    bad = []
    for c in cl:
        st, inst, hist = got[c]
        if [s.as_tuple() for s in sim.read_state(c, 1)] != st:
            bad.append((c, "state"))
        elif per_key and [i.as_tuple() for i in sim.read_instances(c, 1)] != inst:
            bad.append((c, "instances"))
        elif abd and sim.history(c) != hist:
            bad.append((c, "history"))
    return {"compared": len(cl), "equal": len(cl) - len(bad), "mismatches": bad[:8],
            "by_kind": {k: len(v) for k, v in picks.items()}}
