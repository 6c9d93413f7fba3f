"""Records per non-empty mailbox box (one source's records to one replica for
one step), measured on the oracle: how many of a lane's record reads a
lane-major record layout would serve from a line already fetched.  Round 5
(DESIGN.md §5.7): config 2 has 8.0 records per box, config 5 1.45.  The
oracle is the checker here, not the thing measured.

  python tools/box_hist.py <config> <clusters> <start> <steps>
"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import bench  # noqa: E402
import oracle_lib as ol  # noqa: E402


def main():
    cfg_id, C, start, T = (int(x) for x in sys.argv[1:5])
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
    h, recs = collections.Counter(), 0
    for _ in range(T):
        for c in range(C):
            for r in range(N):
                for n in collections.Counter(x[0] for x in o.read_inbox(c, r)).values():   # by source
                    h[n] += 1
                    recs += n
        o.step(1)
    o.close()
    boxes = max(1, sum(h.values()))
    print("config", cfg_id, "boxes", boxes, "records", recs, "records/box %.2f" % (recs / boxes))
    print("hist", sorted(h.items())[:12])
    print("records beyond the first in their box: %.3f" % ((recs - boxes) / max(1, recs)))


if __name__ == "__main__":
    main()
