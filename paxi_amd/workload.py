"""Key distributions of the reference benchmark's key generator.

`Benchmark.next` (benchmark.go:202-244) draws the key of each command from
Bconfig.Distribution.  In the simulator the key of a command is a pure
function of (cluster, cid) so that both backends agree without shared RNG
state:

- "uniform"     rand.Intn(K) + Min                -> hash(cid) mod K
- "order"       counter = (counter+1) % K; + Min   -> cid mod K (cid is the
                (benchmark.go:205-207)                command's issue number, 1-based)
- "conflict"    the literal key 0 if rand.Intn(100) < Conflicts, else the
                "order" key (benchmark.go:213-219)  (the order counter is cid, so it
                                                    also advances on conflict draws)
- "normal"      int(NormFloat64()*Sigma + Mu), then wrapped: while < 0 add K,
                while > K subtract K (benchmark.go:221-227)
- "zipfan"      rand.NewZipf(r, ZipfianS, ZipfianV, K).Uint64() (benchmark.go:99,229-230):
                P(k) proportional to (V + k)^-S over k in [0, K]
- "exponential" int(rand.ExpFloat64() / Lambda) (benchmark.go:232-233)

Key indices and key values.  Go adds Bconfig.Min to the "order" / "uniform"
keys and to conflict's counter key, but not to conflict's literal key 0 nor to
the table distributions' keys.  The simulator keeps key *indices* in
[0, keys) and maps them to the values the Database sees (`key_value`): Min + k
for "order"/"uniform"/"conflict" over a key space of Bconfig.K = key_space
indices; conflict's literal 0 is index key_space when Min != 0 (its own key,
as in Go); the table distributions' index is the value.

The last three become an inverse-CDF table (`Workload.key_cdf`) of the exact
probability mass of the reference's integer key.  "normal" and "zipfan" return
values in [0, K] inclusive in Go, so they are restated with K = keys - 1.
"exponential" is unbounded in Go: its table holds the exact mass of keys
[0, keys), and `key_tail` marks the draws beyond them, which are not folded
back - the replica that needs such a key raises UNFAITHFUL (the key space is a
bound of the model, like the log window).

Bconfig.Move (benchmark.go:137-140) moves "normal"'s Mu on a timer:
`Mu = float64(int(Mu+1) % K)` every Speed ms.  The simulator's generator clock
is the cluster's issue count (cid - 1 counts the commands issued before this
one, workers in turn): Mu moves once per `move_every` issued commands, the
analogue of Speed ms at a rate of move_every / Speed commands per ms.  The Mu
sequence is finite up to a cycle (after the first move Mu is an integer in
(-K, K)), so every Mu it visits gets its own table (`move_cdf`).
"""
import ctypes as C
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
    """P(int(Exp/lambda) = k) for k in [0, keys) (benchmark.go:232-233); the
    rest of the mass, a^keys, lies beyond the key space (not folded)."""
    if lam <= 0.0:
        raise ValueError("lambda must be > 0")
    a = math.exp(-lam)
    return [(a ** k) * (1.0 - a) for k in range(keys)]


def _u32(c):
    return min(0xFFFFFFFF, max(0, int(round(c * 4294967296.0))))


def key_cdf(pmf, normalise=True):
    """Inverse-CDF thresholds: key = #{k < keys-1 : u32 draw >= cdf[k]}.  With
    normalise=False the pmf's total may be below 1 (a tail beyond the keys)."""
    out, c = [], 0.0
    tot = sum(pmf) if normalise else 1.0
    for k in range(len(pmf) - 1):
        c += pmf[k] / tot
        out.append(_u32(c))
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


def _go_mod(a, k):
    """Go's % on ints: truncated division, the result has the dividend's sign."""
    r = abs(a) % k
    return r if a >= 0 else -r


def mu_sequence(mu0, K):
    """The Mu values of Bconfig.Move (benchmark.go:138: Mu = float64(int(Mu+1) % K)):
    (mus, loop) with mus[e] the Mu after e moves, and mus[e] = mus[loop + (e-loop) %
    (len(mus)-loop)] for e >= len(mus)."""
    if K < 1:
        raise ValueError("moving Mu needs K >= 1 (Go's % by zero panics)")
    mus, seen = [float(mu0)], {}
    while True:
        m = float(_go_mod(int(mus[-1] + 1.0), K))   # int() truncates toward zero, as Go's conversion
        if m in seen:
            return mus, seen[m]
        seen[m] = len(mus)
        mus.append(m)


def set_distribution(w, name, keys=None, key_space=0, move_every=0, **kw):
    """Fill `w` (abi.Workload) for Bconfig.Distribution `name`.  key_space is
    Bconfig.K of "order"/"uniform"/"conflict" (0 = keys); move_every > 0 moves
    "normal"'s Mu once per that many issued commands (Bconfig.Move)."""
    if name not in DISTRIBUTIONS:
        raise ValueError(f"unknown distribution {name}")   # benchmark.go:235-236 log.Fatalf
    w.distribution = DISTRIBUTIONS[name]
    w.conflicts = int(kw.get("conflicts", DEFAULTS["conflicts"])) if name == "conflict" else 0
    w.key_space = key_space
    w.key_tail = 0
    w.move_every = w.move_tables = w.move_loop = 0
    w.move_cdf = None
    w._move_buf = None
    for i in range(abi.MAX_KEYS):
        w.key_cdf[i] = 0
    if name == "conflict" and getattr(w, "key_min", 0) and keys and (key_space or keys) >= keys:
        # the native check_keys refuses it too: Go's literal key 0 needs an index of its own
        raise ValueError("conflict with key_min != 0 needs key_space < keys (literal key 0 has its own index)")
    if w.distribution != abi.DIST_TABLE:
        if move_every:
            raise ValueError("Move applies to the normal distribution")
        return w
    if not keys or keys < 1 or keys > abi.MAX_KEYS:
        raise ValueError("table distributions need keys in [1, 64]")
    if name == "exponential":
        pmf = table_pmf(name, keys, **kw)
        for i, c in enumerate(key_cdf(pmf, normalise=False)):
            w.key_cdf[i] = c
        w.key_tail = _u32(sum(pmf))            # draws at or above: beyond the key space
    else:
        for i, c in enumerate(key_cdf(table_pmf(name, keys, **kw))):
            w.key_cdf[i] = c
    if move_every:
        if name != "normal":
            raise ValueError("Move applies to the normal distribution (benchmark.go:137-140)")
        p = {**DEFAULTS, **kw}
        mus, loop = mu_sequence(p["mu"], keys - 1)
        buf = (C.c_uint32 * (len(mus) * abi.MAX_KEYS))()
        for e, mu in enumerate(mus):
            for i, c in enumerate(key_cdf(normal_pmf(keys, mu, p["sigma"]))):
                buf[e * abi.MAX_KEYS + i] = c
        w.move_every, w.move_tables, w.move_loop = move_every, len(mus), loop
        w._move_buf = buf                      # keeps the tables alive while w is
        w.move_cdf = C.cast(buf, C.POINTER(C.c_uint32))
    return w


def expected_pmf(w, keys, table=None):
    """Probability of each key index in [0, keys) under the workload's
    distribution, ignoring locality (for tests and documentation); with
    moving Mu, of table `table`.  For "exponential" the masses sum to less
    than 1 (the rest is beyond the key space)."""
    if w.distribution == abi.DIST_TABLE:
        if table is not None:
            cdf = [w.move_cdf[table * abi.MAX_KEYS + i] for i in range(keys - 1)]
        else:
            cdf = [w.key_cdf[i] for i in range(keys - 1)]
        top = w.key_tail if (w.key_tail and table is None) else 4294967296
        edges = [0] + cdf + [top]
        return [(edges[k + 1] - edges[k]) / 4294967296.0 for k in range(keys)]
    ks = w.key_space or keys
    if w.distribution == abi.DIST_CONFLICT:
        if w.key_min and ks >= keys:
            raise ValueError("conflict with key_min != 0 needs key_space < keys (literal key 0 has its own index)")
        c = w.conflicts / 100.0
        p = [(1 - c) / ks if k < ks else 0.0 for k in range(keys)]
        p[ks if w.key_min else 0] += c
        return p
    return [1.0 / ks if k < ks else 0.0 for k in range(keys)]


def key_value(w, keys, k):
    """The key value the reference's Database sees for key index k (Command.Key)."""
    if k >= keys:
        raise ValueError(f"key index {k} lies beyond the key space (an exponential tail draw)")
    if w.distribution == abi.DIST_CONFLICT and w.key_min and (w.key_space or keys) >= keys:
        raise ValueError("conflict with key_min != 0 needs key_space < keys (literal key 0 has its own index)")
    if w.distribution == abi.DIST_TABLE:
        return k
    if w.distribution == abi.DIST_CONFLICT and w.key_min and k == (w.key_space or keys):
        return 0
    return w.key_min + k


def key_index(w, keys, v):
    """Inverse of key_value."""
    for k in range(keys):
        try:
            if key_value(w, keys, k) == v:
                return k
        except ValueError:
            break
    raise ValueError(f"key {v} is not in the workload's key space")
