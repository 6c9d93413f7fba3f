"""Runner for the G1-G14 scripted one-cluster traces (tests/golden/kats.json
"gtraces", derived by hand from the Go source in tests/golden/make_kats.py).

The same runner drives either backend: the CPU oracle (tests/oracle_lib.py)
or the HIP library (paxi_amd.sim.Simulation).  A trace is
  config    npz / max_delay / thrifty / ephemeral_leader / seed
  workload  outstanding workers, max requests, target replica per worker
  faults    [kind, src, dst, param, step_from, step_to] scripted socket faults
  inject    [step, replica, cid]: a client request handled at `step`
  checkpoints  replica fields expected after `after` steps
  expect    every replica's final state, executed commands, message counts
  log       optional read_log window of one replica
  totals    optional cluster-wide counters
"""
import json
import os

from paxi_amd import abi

KATS = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "kats.json")))
GTRACES = KATS["gtraces"]
NAME_TO_MSG = {v: k for k, v in abi.MSG_NAMES.items()}


def build(tr, seed=None):
    c = tr["config"]
    cfg = abi.make_config(npz=c["npz"], clusters=1, seed=c.get("seed", 1) if seed is None else seed,
                          window=16, mbox_cap=16, max_delay=c["max_delay"], thrifty=c.get("thrifty", 0),
                          ephemeral_leader=c.get("ephemeral_leader", 0))
    w = tr["workload"]
    wl = abi.make_workload(outstanding=w["outstanding"], max_requests=w["max_requests"], target=w["target"])
    faults = [abi.make_fault(k, s, d, p, step_from=a, step_to=b) for k, s, d, p, a, b in tr["faults"]]
    return cfg, wl, faults


def _replica_view(r):
    return {"ballot": r.ballot, "slot": r.slot, "execute": r.execute, "active": r.active,
            "p1_acks": r.p1_acks, "npending": r.npending,
            "delivered": {abi.MSG_NAMES[i]: r.delivered[i] for i in range(abi.NMSG) if r.delivered[i]},
            "client_requests": r.client_requests, "sent": r.sent, "dropped": r.dropped,
            "discarded": r.discarded, "commits": r.commits, "replies": r.replies, "flags": r.flags}


def run(sim, tr, exec_log=None):
    """Step `sim` through the trace, checking checkpoints; return a list of
    mismatch strings (empty = the trace's hand-derived answer holds)."""
    errs = []
    injects = sorted(tr["inject"])
    cps = {cp["after"]: cp for cp in tr["checkpoints"]}
    t = 0
    while t < tr["steps"]:
        for step, r, cid in injects:
            if step == t:
                sim.inject(0, r, cid)
        sim.step(1)
        t += 1
        if t in cps:
            st = sim.read_state()
            for r, want in cps[t]["replicas"].items():
                got = _replica_view(st[int(r)])
                for k, v in want.items():
                    if got[k] != v:
                        errs.append(f"after {t} replica {r} {k}: got {got[k]} want {v}")
    st = sim.read_state()
    for r, want in enumerate(tr["expect"]):
        got = _replica_view(st[r])
        for k, v in want.items():
            if k == "executed":
                continue
            if got[k] != v:
                errs.append(f"final replica {r} {k}: got {got[k]} want {v}")
        if exec_log is not None:
            ex = exec_log(sim, r)
            if ex != want["executed"]:
                errs.append(f"final replica {r} executed: got {ex} want {want['executed']}")
    if "log" in tr:
        lg = tr["log"]
        ents = sim.read_log(0, lg["replica"], lg["slot_lo"], len(lg["entries"]))
        for e, want in zip(ents, lg["entries"]):
            got = {"slot": e.slot, "flags": e.flags, "ballot": e.ballot, "cmd": e.cmd, "acks": e.acks,
                   "request": e.request}
            if got != want:
                errs.append(f"log slot {want['slot']}: got {got} want {want}")
    if "totals" in tr:
        s = sim.stats()
        got = {"delivered_total": s.delivered_total, "sent": s.sent, "dropped": s.dropped,
               "commits": s.commits, "replies": s.replies}
        for k, v in tr["totals"].items():
            if got[k] != v:
                errs.append(f"totals {k}: got {got[k]} want {v}")
    return errs


def seeds_for(tr):
    """Seeds a trace is checked under: its own only if its outcome depends on
    the PRNG (G2's flaky draws), else several, since a serialised trace must
    not depend on the merge order."""
    if tr.get("seed_dependent"):
        return [tr["config"].get("seed", 1)]
    return [1, 7, 42, 1234]
