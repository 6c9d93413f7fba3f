"""Lane imbalance of the serial step kernel, and what re-binning clusters into
waves could recover (round-3 verdict item 3), measured offline on the oracle.

A wave of the serial kernel runs replica r's replica-step for its 64 clusters
together, so each (step, replica) costs about as many merge trips as its
busiest lane needs.  This runs a BASELINE config's clusters on the CPU oracle
from step `start` for `steps` steps, takes the exact number of records every
(cluster, replica) handles at every step, and prices assignments of the live
clusters to waves of 64 by cost = sum over steps, replicas and waves of the
largest lane count, against the mean (sum / 64):
  random       - the order compaction leaves (no re-binning)
  load         - sorted by the previous half-window's message count (the proxy
                 the verdict names: last launch's delivered count)
  phase k      - sorted by the convoy phase: the step (mod k) at which the
                 cluster's leader was busiest in the previous half-window
  phase k (same window) - the same, measured on the priced window itself (a bound)
  busiest_first - no re-binning; every lane runs its replicas busiest first
                 (the serial kernel's PXS_BUSY_FIRST order)
  lane_total_bound - lanes that advance through their replicas independently
The oracle is the checker here, not the thing measured.
usage: python tools/imbalance.py <config> <clusters> <start> <steps> [out.json]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import bench  # noqa: E402
import oracle_lib as ol  # noqa: E402


def counts(cfg_id, C, start, T):
    a = argparse.Namespace(window=None, mbox=None, kv=1, history=512, clusters=C, sim_steps=None, warmup=5,
                           steps=20, crash_step=None, fz=1)
    for k, v in bench.DEFAULTS[cfg_id].items():
        if getattr(a, k, None) is None:
            setattr(a, k, v)
    a.crash_step = a.warmup * a.sim_steps
    cfg, wl, fp, faults, _ = bench.workload(cfg_id, C, 0, 0, a)
    o = ol.OracleSim(cfg, wl, fp, faults)
    o.step(start, threads=min(8, os.cpu_count() or 1))
    N = sum(cfg.npz[i] for i in range(cfg.n_zones))

    def deliv():
        return np.array([sum(s.delivered) + s.client_requests for s in o.read_state()]).reshape(C, N)
    prev, M = deliv(), np.zeros((T, C, N), dtype=np.int32)
    for t in range(T):
        o.step(1)
        cur = deliv()
        M[t], prev = cur - prev, cur
    o.close()
    return M


def main():
    cfg_id, C, start, T = (int(x) for x in sys.argv[1:5])
    M = counts(cfg_id, C, start, T)
    live = M.sum(axis=(0, 2)) > 0
    Ml = M[:, live, :]
    L = Ml.shape[1] // 64 * 64
    Ml = Ml[:, :L, :]
    h = T // 2
    rng = np.random.default_rng(0)

    def cost(perm, lo, hi):
        X = Ml[lo:hi][:, perm, :].reshape(hi - lo, L // 64, 64, -1)
        return float(X.max(axis=2).sum() / (Ml[lo:hi].sum() / 64.0))

    res = {"config": cfg_id, "clusters": C, "live": int(L), "window": [start, start + T],
           "metric": "sum over steps, replicas and waves of the largest lane's records / the mean lane's (1 = no imbalance)",
           "priced_on": [start + h, start + T]}
    res["random"] = cost(rng.permutation(L), h, T)
    res["load"] = cost(np.argsort(Ml[:h].sum(axis=(0, 2)), kind="stable"), h, T)
    lead = Ml[:, :, :].sum(axis=2) if cfg_id == 5 else Ml[:, :, 0]
    for k in (2, 3, 4, 6):
        for name, (lo, hi) in (("phase%d" % k, (0, h)), ("phase%d_same_window" % k, (h, T))):
            ph = np.zeros((L, k))
            for t in range(lo, hi):
                ph[:, (start + t) % k] += lead[t]
            res[name] = cost(np.lexsort((ph.sum(axis=1), np.argmax(ph, axis=1))), h, T)
    # what compaction implements (phase binning): classes by
    # residue, arbitrary order inside a class; and with each class split into
    # load buckets (quantiles of the previous half-window's records)
    ph = np.zeros((L, 3))
    for t in range(0, h):
        ph[:, (start + t) % 3] += lead[t]
    cls, load = np.argmax(ph, axis=1), Ml[:h].sum(axis=(0, 2))
    shuf = rng.permutation(L)
    res["phase3_binned"] = cost(shuf[np.argsort(cls[shuf], kind="stable")], h, T)
    for nb in (2, 3, 4):
        edges = np.quantile(load, np.linspace(0, 1, nb + 1)[1:-1])
        bucket = np.searchsorted(edges, load, side="right")
        key = cls * nb + bucket
        res["phase3_binned_%d_load_buckets" % nb] = cost(shuf[np.argsort(key[shuf], kind="stable")], h, T)
    # replica order per lane: each lane runs its replicas busiest first (the
    # step's counts are known before any replica runs), so the k-th replica-step
    # of every lane in a wave is its k-th busiest; and the bound where lanes
    # advance through their replicas independently (no shared replica index)
    Xp = Ml[h:T].reshape(T - h, L // 64, 64, -1)
    res["busiest_first"] = float((-np.sort(-Xp, axis=3)).max(axis=2).sum() / (Ml[h:T].sum() / 64.0))
    res["lane_total_bound"] = float(Xp.sum(axis=3).max(axis=2).sum() / (Ml[h:T].sum() / 64.0))
    # Cluster pools (round-5 verdict item 3).  A workgroup of `lanes` lanes
    # (lanes / 64 waves) owns 256 clusters in the binned order; at each
    # (step, replica r) the 256 clusters' replica-r inboxes are a pool: a lane
    # takes the next pending cluster whenever it has drained one (greedy list
    # scheduling, `switch` trips per cluster taken: its registers and first
    # record).  The workgroup's waves share the pool, so they meet at a barrier
    # per (step, replica): a phase holds all of its waves for its slowest
    # wave's trips.  slot_time = sum over phases of waves x the slowest wave,
    # over the mean-lane trips (the static kernel: each wave alone, no barrier,
    # = phase3_binned).  The LDS image is per cluster (about 17.3 KB per 64), so
    # a 256-cluster workgroup takes 69 KB and a CU holds 2 of them: 2 x waves
    # per CU, against 8 today.  rate_vs_static = (waves per CU / 8) x
    # (static cost / slot_time): latency-bound waves each run at their own pace.
    order = shuf[np.argsort(cls[shuf], kind="stable")]
    Xb = Ml[h:T][:, order, :]
    Lg = L // 256 * 256
    static = res["phase3_binned"]

    def pool_cost(lanes, switch):
        tot = 0.0
        for t in range(T - h):
            for g in range(0, Lg, 256):
                for r in range(Xb.shape[2]):
                    free = np.zeros(lanes)
                    for v in Xb[t, g:g + 256, r]:         # cluster order: the next pending one
                        k = int(np.argmin(free))
                        free[k] += v + (switch if v else 0)
                    tot += (lanes // 64) * free.reshape(lanes // 64, 64).max(axis=1).max()
        return float(tot / (Xb[:, :Lg].sum() / 64.0))

    # The same pool with one barrier per step instead of per (step, replica):
    # replica-steps of one step are independent, so a wave takes batches of up
    # to 64 pending non-empty (cluster, r) items of the lowest pending r, its
    # lanes coherent on r; a batch costs its largest item (+ switch per item
    # taken, once per batch: the lanes switch together), batches go to the
    # least-loaded of the 4 waves, and a step holds all 4 for its slowest.
    def step_pool_cost(switch):
        tot = 0.0
        for t in range(T - h):
            for g in range(0, Lg, 256):
                load = np.zeros(4)
                for r in range(Xb.shape[2]):
                    items = Xb[t, g:g + 256, r]
                    items = items[items > 0]
                    for b in range(0, len(items), 64):
                        k = int(np.argmin(load))
                        load[k] += items[b:b + 64].max() + switch
                tot += 4 * load.max()
        return float(tot / (Xb[:, :Lg].sum() / 64.0))

    res["pool"] = {"metric": "slot_time (see tools/imbalance.py) and rate against the static binned kernel",
                   "static_binned_cost": static}
    for lanes in (256, 128, 64):
        for sw in (0, 1, 2):
            st_ = pool_cost(lanes, sw)
            res["pool"][f"{lanes}_lanes_switch{sw}"] = {"slot_time": st_,
                                                        "rate_vs_static": (2 * lanes / 64) / 8 * static / st_}
    for sw in (0, 1, 2):
        st_ = step_pool_cost(sw)
        res["pool"][f"step_barrier_256_lanes_switch{sw}"] = {"slot_time": st_, "rate_vs_static": static / st_}
    x = lead.astype(float) - lead.mean(axis=0)
    res["leader_autocorrelation"] = {str(g): float((x[g:] * x[:-g]).sum() / (x * x).sum()) for g in range(1, 7)}
    out = json.dumps(res, indent=1)
    print(out)
    if len(sys.argv) > 5:
        open(sys.argv[5], "w").write(out + "\n")


if __name__ == "__main__":
    main()
