"""Key distributions of the reference benchmark's key generator.

`Benchmark.next` (benchmark.go:202-244) draws the key of each command from
Bconfig.Distribution.  In the simulator the key of a command is a pure
function of (cluster, cid) so that both backends agree without shared RNG
state:

- "uniform"     rand.Intn(K)                      -> hash(cid) mod K
- "order"       counter = (counter+1) % K          -> cid mod K (cid is the
                (benchmark.go:205-207)                command's issue number, 1-based)
- "conflict"    key 0 if rand.Intn(100) < Conflicts, else the "order" key
                (benchmark.go:213-219)              (the order counter is cid, so it
                                                    also advances on conflict draws)
- "normal"      int(NormFloat64()*Sigma + Mu), then wrapped: while < 0 add K,
                while > K subtract K (benchmark.go:221-227)
- "zipfan"      rand.NewZipf(r, ZipfianS, ZipfianV, K).Uint64() (benchmark.go:99,229-230):
                P(k) proportional to (V + k)^-S over k in [0, K]
- "exponential" int(rand.ExpFloat64() / Lambda) (benchmark.go:232-233)

The last three become an inverse-CDF table (`Workload.key_cdf`) of the exact
probability mass of the reference's integer key.  The simulator's key space is
[0, keys): "normal" and "zipfan" return values in [0, K] inclusive in Go, so
they are restated with K = keys - 1; "exponential" is unbounded in Go and its
tail is folded modulo keys.  The moving-mean option (Bconfig.Move, Speed in
wall-clock milliseconds, benchmark.go:137-140) has no step-time equivalent and
is not modelled.  Keys are offsets from Bconfig.Min.
"""
import math

from . import abi

DISTRIBUTIONS = {"uniform": abi.DIST_UNIFORM, "order": abi.DIST_ORDER, "conflict": abi.DIST_CONFLICT,
                 "normal": abi.DIST_TABLE, "zipfan": abi.DIST_TABLE, "zipfian": abi.DIST_TABLE,
                 "exponential": abi.DIST_TABLE}

# Bconfig defaults (benchmark.go:53-71)
DEFAULTS = {"conflicts": 100, "mu": 0.0, "sigma": 60.0, "zipfian_s": 2.0, "zipfian_v": 1.0, "lam": 0.01}


def _phi(x, mu, sigma):
    return 0.5 * (1.0 + math.erf((x - mu) / (sigma * math.sqrt(2.0))))


def normal_pmf(keys, mu, sigma):
    """P(key = k), k in [0, keys), of benchmark.go:221-227 with K = keys - 1."""
    K = keys - 1
    p = [0.0] * keys
    if K == 0:
        return [1.0]
    lo = int(math.floor(mu - 40 * sigma)) - 2
    hi = int(math.ceil(mu + 40 * sigma)) + 2
    for j in range(lo, hi + 1):
        # int() truncates toward zero: j >= 1 from [j, j+1), 0 from (-1, 1), j <= -1 from (j-1, j]
        if j >= 1:
            m = _phi(j + 1, mu, sigma) - _phi(j, mu, sigma)
        elif j == 0:
            m = _phi(1, mu, sigma) - _phi(-1, mu, sigma)
        else:
            m = _phi(j, mu, sigma) - _phi(j - 1, mu, sigma)
        if m <= 0.0:
            continue
        k = j
        if k < 0:
            k += K * ((-k + K - 1) // K)
        if k > K:
            k -= K * ((k - K + K - 1) // K)
        p[k] += m
    return p


def zipf_pmf(keys, s, v):
    """P(key = k) of rand.NewZipf(s, v, imax=K) with K = keys - 1 (needs s > 1, v >= 1)."""
    if not (s > 1.0 and v >= 1.0):
        raise ValueError("zipfian needs s > 1 and v >= 1 (math/rand.NewZipf)")
    w = [(v + k) ** -s for k in range(keys)]
    t = sum(w)
    return [x / t for x in w]


def exponential_pmf(keys, lam):
    """P(int(Exp/lambda) mod keys = k) (benchmark.go:232-233, tail folded)."""
    if lam <= 0.0:
        raise ValueError("lambda must be > 0")
    a = math.exp(-lam)
    den = 1.0 - a ** keys
    return [(a ** k) * (1.0 - a) / den for k in range(keys)]


def key_cdf(pmf):
    """Inverse-CDF thresholds: key = #{k < keys-1 : u32 draw >= cdf[k]}."""
    out, c = [], 0.0
    tot = sum(pmf)
    for k in range(len(pmf) - 1):
        c += pmf[k] / tot
        out.append(min(0xFFFFFFFF, max(0, int(round(c * 4294967296.0)))))
    for k in range(1, len(out)):   # rounding must not break monotonicity
        out[k] = max(out[k], out[k - 1])
    return out


def table_pmf(name, keys, **kw):
    p = {**DEFAULTS, **kw}
    if name == "normal":
        return normal_pmf(keys, p["mu"], p["sigma"])
    if name in ("zipfan", "zipfian"):
        return zipf_pmf(keys, p["zipfian_s"], p["zipfian_v"])
    if name == "exponential":
        return exponential_pmf(keys, p["lam"])
    raise ValueError(f"not a table distribution: {name}")


def set_distribution(w, name, keys=None, **kw):
    """Fill `w` (abi.Workload) for Bconfig.Distribution `name`."""
    if name not in DISTRIBUTIONS:
        raise ValueError(f"unknown distribution {name}")   # benchmark.go:235-236 log.Fatalf
    w.distribution = DISTRIBUTIONS[name]
    w.conflicts = int(kw.get("conflicts", DEFAULTS["conflicts"])) if name == "conflict" else 0
    for i in range(abi.MAX_KEYS):
        w.key_cdf[i] = 0
    if w.distribution == abi.DIST_TABLE:
        if not keys or keys < 1 or keys > abi.MAX_KEYS:
            raise ValueError("table distributions need keys in [1, 64]")
        for i, c in enumerate(key_cdf(table_pmf(name, keys, **kw))):
            w.key_cdf[i] = c
    return w


def expected_pmf(w, keys):
    """Probability of each key in [0, keys) under the workload's distribution,
    ignoring locality (for tests and documentation)."""
    if w.distribution == abi.DIST_TABLE:
        edges = [0] + [w.key_cdf[i] for i in range(keys - 1)] + [4294967296]
        return [(edges[k + 1] - edges[k]) / 4294967296.0 for k in range(keys)]
    if w.distribution == abi.DIST_CONFLICT:
        c = w.conflicts / 100.0
        return [c + (1 - c) / keys if k == 0 else (1 - c) / keys for k in range(keys)]
    return [1.0 / keys] * keys
