"""Multi-GPU orchestration: one process per GPU, clusters sharded by range.

Clusters never exchange messages, so the data path has no collective.  Each
rank simulates the global cluster range [rank*C, (rank+1)*C) — the PRNG is keyed
by the global cluster id, so a cluster's trajectory does not
depend on the number of ranks — and torch.distributed all-reduces only the
statistics (sum) and the elapsed time (max).  With backend "nccl" that is RCCL
over xGMI on MI355X; tests use "gloo" on the CPU.
"""
import os

# order of the per-rank counter vector that gets all-reduced
FLAG_NAMES = ("WOVF", "GHOST", "MBOX_OVF", "PEND_OVF", "UNFAITHFUL", "POISON", "BALLOT_OVF", "HIST_OVF")
COUNTERS = ("delivered_total", "commits", "replies", "dropped", "client_requests", "alg_bytes",
            "violations", "agree_compared", "agree_missed", "active", "active_start") + \
    tuple("flag_" + n for n in FLAG_NAMES)


def env_rank():
    """(rank, world, local_rank) from the torchrun environment (defaults: single process)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard(clusters_per_rank, rank):
    """Global cluster range of one rank under weak scaling: (cluster_base, count)."""
    return rank * clusters_per_rank, clusters_per_rank


def reduce_counters_abi(pd, values, elapsed):
    """The same reduction through the C-ABI (paxisim_dist_allreduce, RCCL):
    integer sums and float maxes over every rank of the communicator `pd`."""
    sums, maxes = pd.allreduce([[int(values.get(k, 0)) for k in COUNTERS]], [[float(e) for e in elapsed]])
    return dict(zip(COUNTERS, [float(v) for v in sums])), maxes


def reduce_counters(values, elapsed, device=None, group=None):
    """Sum `values` (dict over COUNTERS) and max `elapsed` (list of floats) over
    all ranks.  Returns (summed dict, maxed list).  No-op without a process group."""
    import torch
    import torch.distributed as dist
    vec = torch.tensor([float(values.get(k, 0)) for k in COUNTERS], dtype=torch.float64, device=device)
    tim = torch.tensor([float(e) for e in elapsed], dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(vec, op=dist.ReduceOp.SUM, group=group)
        dist.all_reduce(tim, op=dist.ReduceOp.MAX, group=group)
    return dict(zip(COUNTERS, vec.tolist())), tim.tolist()


def stats_counters(delta, alg_bytes=0, violations=0, flagged=None, **extra):
    """Counter dict from a stats delta (bench.stats_delta), scan results and
    extra integer counters (agree_compared, agree_missed, active, active_start)."""
    flagged = flagged or [0] * 8
    d = {"delivered_total": delta["delivered_total"], "commits": delta["commits"], "replies": delta["replies"],
         "dropped": delta["dropped"], "client_requests": delta["client_requests"], "alg_bytes": alg_bytes,
         "violations": violations}
    d.update(extra)
    d.update({"flag_" + n: flagged[i] for i, n in enumerate(FLAG_NAMES)})
    return d


# ---- sharding invariance (per-cluster state at G=8 equals G=1) ----
DIGEST_CLUSTERS = 256


def digest_range(clusters_per_rank):
    """Local clusters each rank digests: [C/2, C/2 + 256) (clipped to the shard)."""
    lo = clusters_per_rank // 2
    return lo, max(0, min(DIGEST_CLUSTERS, clusters_per_rank - lo))


def state_digest(sim, lo, n):
    """SHA-256 (first 16 hex digits) of the replica states of local clusters
    [lo, lo+n) as paxisim_read_state returns them: equal digests, equal states."""
    import hashlib
    if n == 0:
        return "0" * 16
    return hashlib.sha256(bytes(sim.read_state(lo, n))).hexdigest()[:16]


def gather_digests(digest, world):
    """{rank: digest} on every rank (torch.distributed all_gather_object)."""
    if world == 1:
        return {0: digest}
    import torch.distributed as dist
    out = [None] * world
    dist.all_gather_object(out, digest)
    return {r: d for r, d in enumerate(out)}
