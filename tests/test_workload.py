"""Workload key distributions (benchmark.go:202-233, paxi_amd.workload) on the
CPU: the probability tables restate the Go generators, and the oracle draws
keys with those probabilities.  The GPU draws are pinned to the oracle by
tests/test_parity_abd_gpu.py::test_abd_key_distributions."""
import math

import numpy as np
import pytest

from paxi_amd import abi
from paxi_amd import workload as W
import oracle_lib as ol


def test_zipf_table_matches_closed_form():
    p = W.zipf_pmf(16, 2.0, 1.0)
    z = sum((1 + k) ** -2.0 for k in range(16))
    assert abs(p[0] - 1 / z) < 1e-12 and abs(p[15] - 16 ** -2.0 / z) < 1e-12
    with pytest.raises(ValueError):
        W.zipf_pmf(16, 1.0, 1.0)      # math/rand.NewZipf needs s > 1


def test_exponential_is_not_folded():
    """int(ExpFloat64()/Lambda) is unbounded (benchmark.go:232-233): the table
    holds the exact mass of keys [0, keys), and the rest lies beyond key_tail
    (not aliased onto real keys)."""
    keys, lam = 10, 0.05
    exact = [math.exp(-lam * j) - math.exp(-lam * (j + 1)) for j in range(keys)]
    assert np.allclose(W.exponential_pmf(keys, lam), exact, atol=1e-12)
    w = abi.make_workload(distribution="exponential", keys=keys, lam=lam)
    assert abs(w.key_tail / 2 ** 32 - (1 - math.exp(-lam * keys))) < 1e-9
    p = W.expected_pmf(w, keys)
    assert np.allclose(p, exact, atol=1e-9) and abs(sum(p) + math.exp(-lam * keys) - 1) < 1e-9


@pytest.mark.parametrize("mu,sigma,keys", [(0.0, 60.0, 16), (8.0, 3.0, 16), (5.0, 0.7, 9)])
def test_normal_table_restates_go_truncation_and_wrap(mu, sigma, keys):
    """int(NormFloat64()*Sigma+Mu) truncates toward zero, then wraps with
    `for key < 0 {key += K}; for key > K {key -= K}` (benchmark.go:221-227)."""
    K = keys - 1
    x = np.random.default_rng(1).normal(mu, sigma, 2_000_000)
    k = np.trunc(x).astype(np.int64)
    neg = k < 0
    k[neg] += K * ((-k[neg] + K - 1) // K)
    big = k > K
    k[big] -= K * ((k[big] - 1) // K)
    assert k.min() >= 0 and k.max() <= K
    emp = np.bincount(k, minlength=keys) / len(k)
    assert np.abs(emp - np.array(W.normal_pmf(keys, mu, sigma))).max() < 2e-3


def test_cdf_table_is_monotone_and_exact_for_thresholds():
    w = abi.make_workload(distribution="zipfan", keys=12, zipfian_s=1.5, zipfian_v=2.0)
    cdf = [w.key_cdf[i] for i in range(11)]
    assert cdf == sorted(cdf) and w.distribution == abi.DIST_TABLE
    assert np.allclose(W.expected_pmf(w, 12), W.zipf_pmf(12, 1.5, 2.0), atol=1e-9)


def test_unknown_distribution_is_rejected():
    with pytest.raises(ValueError):
        abi.make_workload(distribution="pareto", keys=8)          # benchmark.go:235-236
    with pytest.raises(ValueError):
        abi.make_workload(distribution="normal")                 # table needs keys


def test_oracle_rejects_bad_workloads():
    cfg = abi.make_config(protocol=abi.ABD, npz=[3], clusters=4, keys=8)
    wl = abi.make_workload(distribution="conflict", conflicts=50)
    wl.conflicts = 101
    with pytest.raises(RuntimeError):
        ol.OracleSim(cfg, wl)
    wl = abi.make_workload(distribution="zipfan", keys=8)
    wl.key_cdf[3] = 0
    with pytest.raises(RuntimeError):
        ol.OracleSim(cfg, wl)


def _abd_keys(dist, keys=16, clusters=256, steps=200, **kw):
    cfg = abi.make_config(protocol=abi.ABD, npz=[3], clusters=clusters, seed=3, keys=keys, history=512)
    wl = abi.make_workload(outstanding=4, target=[0, 1, 2, 0], write_ppm=500_000, distribution=dist, keys=keys, **kw)
    o = ol.OracleSim(cfg, wl)
    o.step(steps)
    ks = [op[0] for c in range(clusters) for op in o.history(c)]
    return np.bincount(ks, minlength=keys) / len(ks), len(ks), wl


@pytest.mark.parametrize("dist,kw", [("zipfan", {}), ("normal", dict(mu=6.0, sigma=4.0)),
                                     ("exponential", dict(lam=0.15)), ("conflict", dict(conflicts=30)),
                                     ("uniform", {})])
def test_oracle_draws_follow_the_distribution(dist, kw):
    emp, n, wl = _abd_keys(dist, **kw)
    exp = np.array(W.expected_pmf(wl, 16))
    exp[-1] += 1.0 - exp.sum()     # exponential: a tail draw is recorded on the last key (and flagged)
    assert n > 20000
    tol = 4 * np.sqrt(exp * (1 - exp) / n) + 2e-3
    assert np.all(np.abs(emp - exp) <= tol), (emp, exp)


def test_order_distribution_is_the_issue_counter():
    """One worker: the i-th command (cid = i) is on key i mod K."""
    keys = 8
    cfg = abi.make_config(protocol=abi.ABD, npz=[3], clusters=2, seed=3, keys=keys, history=64)
    wl = abi.make_workload(outstanding=1, target=0, distribution="order")
    o = ol.OracleSim(cfg, wl)
    o.step(60)
    ops = o.history(0)
    assert len(ops) > 5
    assert [op[0] for op in ops] == [(i + 1) % keys for i in range(len(ops))]


# ---- the reference's key semantics beyond the plain tables (round-3 verdict, f1) ----

def _commands(o, cluster, cids):
    return [o.command(cluster, c) for c in cids]


def test_exponential_tail_draws_raise_unfaithful():
    """A tail draw is a key beyond the model's key space: the replica using it
    raises UNFAITHFUL; with a negligible tail nothing is flagged."""
    for lam, flagged in ((0.15, True), (3.0, False)):
        cfg = abi.make_config(npz=[3], clusters=32, seed=4, keys=16, kv=1)
        wl = abi.make_workload(outstanding=4, target=0, write_ppm=500_000, distribution="exponential", keys=16,
                               lam=lam)
        o = ol.OracleSim(cfg, wl)
        o.step(300)
        tail = [c for c in range(32) if any(o.command(c, cid)[0] == 16 for cid in range(1, 200))]
        unf = [c for c, st in enumerate(zip(*[iter(o.read_state())] * 3)) if any(r.flags & abi.F_UNFAITHFUL for r in st)]
        assert bool(unf) == flagged and set(unf) <= set(tail)
        o.close()


def test_conflict_uses_the_literal_key_zero():
    """benchmark.go:213-214: a conflict draw is key 0, not Min; with Min != 0
    that is a key of its own (index key_space), the rest Min + counter."""
    cfg = abi.make_config(protocol=abi.ABD, npz=[3], clusters=4, keys=9)
    wl = abi.make_workload(distribution="conflict", conflicts=40, key_min=100, key_space=8)
    o = ol.OracleSim(cfg, wl)
    ks = [k for k, _ in _commands(o, 1, range(1, 3000))]
    assert set(ks) == set(range(9))
    assert abs(ks.count(8) / len(ks) - 0.40) < 0.03
    assert [W.key_value(wl, 9, k) for k in (0, 7, 8)] == [100, 107, 0]
    assert W.key_index(wl, 9, 0) == 8 and W.key_index(wl, 9, 103) == 3
    assert all(k == (cid % 8) for cid, k in zip(range(1, 3000), ks) if k != 8)
    o.close()
    wl0 = abi.make_workload(distribution="conflict", conflicts=40, key_space=8)   # Min = 0: key 0 is index 0
    o = ol.OracleSim(cfg, wl0)
    assert max(k for k, _ in _commands(o, 1, range(1, 500))) < 8
    o.close()
    with pytest.raises(RuntimeError):   # the literal key needs an index beyond key_space
        ol.OracleSim(cfg, abi.make_workload(distribution="conflict", conflicts=40, key_min=100, key_space=9))


@pytest.mark.parametrize("mu0,K,expect", [
    (5.5, 7, ([5.5, 6, 0, 1, 2, 3, 4, 5], 1)),            # int(6.5) = 6, then 7 % 7 = 0: the wrap
    (-3.5, 7, ([-3.5, -2, -1, 0, 1, 2, 3, 4, 5, 6], 3)),  # int(-2.5) = -2 (toward zero); Go's % keeps the sign
    (0.0, 1, ([0.0, 0.0], 1)),
])
def test_mu_sequence_restates_go(mu0, K, expect):
    """b.Mu = float64(int(b.Mu+1) % b.K) (benchmark.go:138)."""
    mus, loop = W.mu_sequence(mu0, K)
    assert (mus, loop) == (list(map(float, expect[0])), expect[1])


def test_moving_mu_draws_follow_each_tables_distribution():
    """Bconfig.Move: command cid draws from the normal of the Mu its issue count
    reaches, (cid-1) // move_every moves after the start; the sequence wraps
    from K-1 to 0 and then cycles (benchmark.go:137-140, 221-227)."""
    keys, every = 8, 97
    wl = abi.make_workload(distribution="normal", keys=keys, mu=5.5, sigma=1.2, move_every=every)
    mus, loop = W.mu_sequence(5.5, keys - 1)
    assert (wl.move_tables, wl.move_loop) == (len(mus), loop)
    cfg = abi.make_config(protocol=abi.ABD, npz=[3], clusters=64, keys=keys)
    o = ol.OracleSim(cfg, wl)
    n_ep = len(mus) + 3                                # past the end: the cycle repeats
    counts = np.zeros((n_ep, keys))
    for c in range(64):
        for cid, (k, _) in zip(range(1, every * n_ep + 1), _commands(o, c, range(1, every * n_ep + 1))):
            counts[(cid - 1) // every, k] += 1
    o.close()
    for e in range(n_ep):
        t = e if e < len(mus) else loop + (e - loop) % (len(mus) - loop)
        exp = np.array(W.normal_pmf(keys, mus[t], 1.2))
        emp = counts[e] / counts[e].sum()
        tol = 4 * np.sqrt(exp * (1 - exp) / counts[e].sum()) + 3e-3
        assert np.all(np.abs(emp - exp) <= tol), (e, mus[t], emp, exp)
    # the keys follow Mu across the wrap (Mu 6 -> 0): int() truncates, so Mu = 6 puts its mass on 5..7
    assert counts[1][5:].sum() > 0.7 * counts[1].sum() and counts[2].argmax() == 0


def test_bad_key_workloads_are_rejected():
    cfg = abi.make_config(protocol=abi.ABD, npz=[3], clusters=2, keys=8)
    with pytest.raises(RuntimeError):
        ol.OracleSim(cfg, abi.make_workload(key_space=9))                          # beyond keys
    ol.OracleSim(cfg, abi.make_workload(distribution="uniform", key_space=4)).close()
    with pytest.raises(ValueError):
        abi.make_workload(distribution="zipfan", keys=8, move_every=5)            # Move is normal's
    w = abi.make_workload(distribution="normal", keys=8, move_every=5)
    w.move_loop = w.move_tables
    with pytest.raises(RuntimeError):
        ol.OracleSim(cfg, w)


def test_conflict_with_min_needs_its_own_key_index():
    """check_keys refuses conflict with key_min != 0 and key_space >= keys; the
    Python helpers raise the same ValueError instead of an IndexError."""
    with pytest.raises(ValueError):
        abi.make_workload(distribution="conflict", conflicts=40, key_min=100, keys=8)
    wl = abi.make_workload(distribution="conflict", conflicts=40, key_min=100)   # keys unknown here
    with pytest.raises(ValueError):
        W.expected_pmf(wl, 8)
    with pytest.raises(ValueError):
        W.key_value(wl, 8, 0)
    ok = abi.make_workload(distribution="conflict", conflicts=40, key_min=100, key_space=7, keys=8)
    p = W.expected_pmf(ok, 8)
    assert abs(sum(p) - 1.0) < 1e-9 and abs(p[7] - 0.4) < 1e-9
