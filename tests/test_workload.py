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


def test_exponential_fold_matches_brute_force():
    keys, lam = 10, 0.05
    brute = [0.0] * keys
    for j in range(20000):
        brute[j % keys] += math.exp(-lam * j) - math.exp(-lam * (j + 1))
    assert np.allclose(W.exponential_pmf(keys, lam), brute, atol=1e-12)


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
