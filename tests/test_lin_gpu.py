"""History.Linearizable (history.go:55-71, checker.go:69-104) on the GPU
checker without a size cap: seeded random register histories with concurrent
writes, stale reads and never-written reads, partitions from a few ops to
several hundred (above LIN_SMAX = 128 they take lin_big_kernel's path), loaded
through History.ReadFile's device path (paxisim_history_load) and checked
against the oracle's restatement; plus the tie-order known answer of DESIGN.md
§3.7 (sort.Sort(byTime) is not stable in Go; here ties keep canonical order)."""
import random

import pytest

from paxi_amd import abi
import oracle_lib as ol
from test_oracle_kats import KATS


def gen_partition(rng, n):
    """n ops of one key: (is_write, value, start, end); unique write values."""
    ops, writes, t, nextv = [], [], 0, 1
    for _ in range(n):
        t += rng.choice((0, 0, 1, 1, 2, 3))
        start = t
        end = start + rng.choice((0, 1, 2, 3, 5, 8))
        if rng.random() < 0.5:
            ops.append((1, nextv, start, end))
            writes.append((nextv, start, end))
            nextv += 1
        else:
            done = [w for w in writes if w[2] < start]
            conc = [w for w in writes if w[2] >= start]
            r = rng.random()
            if r < 0.08 or not writes:
                v = 0                                              # the initial (nil) value
            elif r < 0.25 and len(done) > 1:
                v = rng.choice(done[:-1])[0]                       # stale
            elif r < 0.5 and conc:
                v = rng.choice(conc)[0]                            # a concurrent write
            else:
                v = (done or writes)[-1][0]                        # the latest completed write
            ops.append((0, v, start, end))
    return ops


def gen_future_reads(rng, n):
    """n ops of one key where a read may return any write's value, one that
    starts only after the read ended too: merges then refine a write's end
    below its start, which makes edges u -> t with u.start > t.end that
    cut() removes (checker.go:93-100), and exercises the checker's
    cyclic-state shortcut and its fallback (lin_kernel.h LinReg::run)."""
    kinds, t = [], 0
    for _ in range(n):
        t += rng.choice((0, 0, 1, 1, 2, 3))
        kinds.append((t, t + rng.choice((0, 1, 2, 3, 5, 8)), rng.random() < 0.5))
    nw = sum(1 for k in kinds if k[2])
    ops, v = [], 1
    for (start, end, w) in kinds:
        if w:
            ops.append((1, v, start, end))
            v += 1
        else:
            ops.append((0, 0 if rng.random() < 0.05 or nw == 0 else rng.randint(1, nw), start, end))
    return ops


def load(sims, cluster, key, ops, N, H):
    """Spread one partition over the replicas' histories (canonical order: replica 0 first)."""
    per = -(-len(ops) // N)
    for r in range(N):
        part = ops[r * per:(r + 1) * per]
        for s in sims:
            s.extra.setdefault((cluster, r), [])
            s.extra[(cluster, r)] += [(key, w, v, st, en) for (w, v, st, en) in part]
    assert per <= H


def run_case(seed, sizes, N=5, H=256, gen=gen_partition):
    rng = random.Random(seed)
    keys = len(sizes[0])
    cfg = abi.make_config(protocol=abi.ABD, npz=[N], clusters=len(sizes), keys=keys, history=H)
    wl = abi.make_workload(outstanding=1, max_requests=1, target=[0])
    from paxi_amd.sim import Simulation
    g, o = Simulation(cfg, wl), ol.OracleSim(cfg, wl)
    g.extra, o.extra = {}, {}
    expect = 0
    for c, row in enumerate(sizes):
        for k, n in enumerate(row):
            ops = gen(rng, n)
            expect += ol.linearizable([(v if w else None, None if w else v, s, e) for (w, v, s, e) in ops])
            load((g, o), c, k, ops, N, H)
    for (c, r), ops in g.extra.items():
        g.history_load(c, r, ops)
        o.history_load(c, r, ops)
    ga, gn, gsk = g.linearizable()
    oa, on = o.linearizable()
    g.close()
    return (ga, gn, gsk), (oa, on), expect


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_small_partitions_match_oracle(seed):
    sizes = [[1 + (7 * c + 13 * k + seed) % 128 for k in range(6)] for c in range(12)]
    (ga, gn, gsk), (oa, on), expect = run_case(seed, sizes)
    assert gsk == 0 and gn == on == sum(map(sum, sizes))
    assert ga == oa == expect and expect > 0


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [11, 12])
def test_future_reads_match_oracle(seed):
    """Reads of writes that start later: cut() removes edges, so the
    cyclic-state shortcut must fall back to the DFS exactly where the
    reference's Cycle() / cut would change the graph; register path (at most
    128 ops) and big path."""
    sizes = [[1 + (11 * c + 17 * k + seed) % 128 for k in range(6)] for c in range(10)] + [[129, 200, 64, 90, 128, 5]]
    (ga, gn, gsk), (oa, on), expect = run_case(seed, sizes, gen=gen_future_reads)
    assert gsk == 0 and gn == on == sum(map(sum, sizes))
    assert ga == oa == expect and expect > 0


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [4, 5])
def test_large_partitions_take_the_big_path(seed):
    """Partitions of 127..700 ops: the ones above 128 are checked by
    lin_big_kernel (HBM scratch), with nothing skipped."""
    sizes = [[127, 128, 129], [300, 5, 700], [64, 65, 200]]
    (ga, gn, gsk), (oa, on), expect = run_case(seed, sizes, H=256)
    assert gsk == 0 and gn == on == sum(map(sum, sizes))
    assert ga == oa == expect


@pytest.mark.gpu
def test_partitions_beyond_4096_ops():
    """Partitions of 4097 and 5000 ops need more than one bit-set word per
    lane (lin_big_kernel<4>): still equal to the oracle."""
    sizes = [[4097], [5000], [300]]
    (ga, gn, gsk), (oa, on), expect = run_case(6, sizes, N=5, H=1024)
    assert gsk == 0 and gn == on == sum(map(sum, sizes))
    assert ga == oa == expect


@pytest.mark.gpu
def test_partition_beyond_the_bit_sets_is_reported_skipped():
    """More than 16384 ops in one (cluster, key): counted in `skipped`, its ops
    not in `ops` (include/paxisim.h), the other partitions still checked."""
    from paxi_amd.sim import Simulation
    rng = random.Random(8)
    N, H = 5, 3600
    cfg = abi.make_config(protocol=abi.ABD, npz=[N], clusters=2, keys=2, history=H)
    wl = abi.make_workload(outstanding=1, max_requests=1, target=[0])
    g = Simulation(cfg, wl)
    big, small = gen_partition(rng, 16385), gen_partition(rng, 200)
    per = -(-len(big) // N)
    for r in range(N):
        ops = [(0, w, v, st, en) for (w, v, st, en) in big[r * per:(r + 1) * per]]
        if r == 0:
            ops += [(1, w, v, st, en) for (w, v, st, en) in small]
        g.history_load(1, r, ops)
    a, n, skipped = g.linearizable()
    g.close()
    assert skipped == 1 and n == 200
    assert a == ol.linearizable([(v if w else None, None if w else v, s, e) for (w, v, s, e) in small])


def tie_ops(order):
    return [tuple(o) for o in KATS["lin_tie_order"][order]]


def test_tie_order_kat_oracle():
    """The same five ops in two canonical orders that differ only among equal
    starts: ties keep canonical order, and the count depends on it."""
    k = KATS["lin_tie_order"]
    assert ol.linearizable(tie_ops("a")) == k["expect_a"]
    assert ol.linearizable(tie_ops("b")) == k["expect_b"]
    assert k["expect_a"] != k["expect_b"]


@pytest.mark.gpu
def test_tie_order_kat_gpu():
    from paxi_amd.sim import Simulation
    k = KATS["lin_tie_order"]
    cfg = abi.make_config(protocol=abi.ABD, npz=[3], clusters=2, keys=1, history=16)
    wl = abi.make_workload(outstanding=1, max_requests=1, target=[0])
    for order, want in (("a", k["expect_a"]), ("b", k["expect_b"])):
        g = Simulation(cfg, wl)
        ops = [(0, 1, i, s, e) if i is not None else (0, 0, o, s, e) for (i, o, s, e) in tie_ops(order)]
        g.history_load(1, 1, ops)
        assert g.linearizable() == (want, len(ops), 0)
        g.close()
