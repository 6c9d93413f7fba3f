"""Capture a cluster's message trace as Paxi gob streams, or replay one.

    python tools/trace_cli.py capture --config 2 --cluster 3 --steps 300 [--clusters 64] --out DIR
    python tools/trace_cli.py replay DIR

`capture` runs a BASELINE config (bench.py's workloads) on the GPU, records the
chosen cluster's inbox step by step and writes DIR/<src>-<dst>.gob (the bytes a
Paxi sender's gob.Encoder writes on that TCP connection, transport.go:108),
DIR/schedule.json (delivery steps, the client's HTTP requests), and
DIR/run.json (the configuration and the captured replicas' final state).
`replay` rebuilds that configuration for the one cluster, decodes the streams
(paxi_amd/trace.py) and delivers them into a run whose links are all dropped,
then compares each replica's final state with the captured one.
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from paxi_amd import abi, trace  # noqa: E402

# replica state compared after a replay: everything but dropped and replies
# (the replay drops every send and has no client workers of its own)
KEEP = lambda t: t[:11] + t[12:14] + t[15:]


def to_dict(s):
    out = {}
    for name, ty in s._fields_:
        v = getattr(s, name)
        if name == "move_cdf":          # Workload's moving-Mu tables: the pointed-to thresholds
            out[name] = [v[i] for i in range(s.move_tables * abi.MAX_KEYS)] if v else None
        else:
            out[name] = list(v) if isinstance(v, C.Array) else v
    return out


def from_dict(cls, d):
    s = cls()
    for name, ty in s._fields_:
        if name not in d:
            continue
        if name == "move_cdf":
            if d[name]:
                s._move_buf = (C.c_uint32 * len(d[name]))(*d[name])
                s.move_cdf = C.cast(s._move_buf, C.POINTER(C.c_uint32))
        elif issubclass(ty, C.Array):
            arr = getattr(s, name)
            for i, x in enumerate(d[name]):
                arr[i] = x
        else:
            setattr(s, name, d[name])
    return s


def capture(args, backend=None):
    import bench
    from paxi_amd.sim import Simulation
    backend = backend or Simulation
    d = bench.DEFAULTS[args.config]
    ns = argparse.Namespace(window=d["window"], mbox=d["mbox"], history=512, kv=1, crash_step=args.crash_step)
    cfg, wl, fp, faults, desc = bench.workload(args.config, args.clusters, 0, 0, ns)
    sim = backend(cfg, wl, fp, faults)
    tr = trace.capture(sim, args.cluster, args.steps)
    streams, sched = trace.export(sim, args.cluster, tr, outdir=args.out)
    state = [list(s.as_tuple()[:8]) + [list(s.as_tuple()[8])] + list(s.as_tuple()[9:])
             for s in sim.read_state(args.cluster, 1)]
    run = {"workload": desc["workload"], "cluster": args.cluster, "config": to_dict(cfg), "workload_params": to_dict(wl),
           "faults": [to_dict(f) for f in faults], "state": state}
    with open(os.path.join(args.out, "run.json"), "w") as f:
        json.dump(run, f)
    print(f"captured cluster {args.cluster}: {len(tr['msgs'])} messages on {len(streams)} links, steps "
          f"[{tr['t0']}, {tr['t0'] + tr['steps']}) -> {args.out}")
    return run


def replay(args, backend=None):
    from paxi_amd.sim import Simulation
    backend = backend or Simulation
    with open(os.path.join(args.dir, "run.json")) as f:
        run = json.load(f)
    cfg = from_dict(abi.Config, run["config"])
    cfg.clusters, cfg.cluster_base = 1, run["cluster"]
    wl = from_dict(abi.Workload, run["workload_params"])
    faults = trace.replay_setup(wl, abi.n_replicas(cfg))
    # a captured Crash discards inboxes at Recv (socket.go:111-118): it is replayed too
    faults += [from_dict(abi.Fault, f) for f in run["faults"] if f["kind"] == abi.FAULT_CRASH]
    sim = backend(cfg, wl, None, faults)
    streams, sched = trace.load_dir(args.dir)
    tr = trace.import_streams(sim, 0, streams, sched)
    trace.replay(sim, 0, tr)
    got = [KEEP(s.as_tuple()) for s in sim.read_state(0, 1)]
    want = [KEEP(tuple(r[:8]) + (tuple(r[8]),) + tuple(r[9:])) for r in run["state"]]
    ok = got == want
    print(f"replayed {len(tr['msgs'])} messages into cluster {run['cluster']}: "
          f"{'every replica matches the capture' if ok else 'MISMATCH'}")
    return ok


def main(argv=None):
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    c = sub.add_parser("capture")
    c.add_argument("--config", type=int, default=2, choices=[2, 3, 4, 5])
    c.add_argument("--cluster", type=int, default=0)
    c.add_argument("--clusters", type=int, default=64)
    c.add_argument("--steps", type=int, default=300)
    c.add_argument("--crash-step", type=int, default=100)
    c.add_argument("--out", required=True)
    r = sub.add_parser("replay")
    r.add_argument("dir")
    args = ap.parse_args(argv)
    if args.cmd == "capture":
        capture(args)
        return 0
    return 0 if replay(args) else 1


if __name__ == "__main__":
    sys.exit(main())
