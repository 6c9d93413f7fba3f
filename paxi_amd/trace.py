"""Message traces in the reference's wire format: capture, gob export, gob
import and replay.

A Paxi deployment on the TCP transport carries every replica-to-replica
message as a gob stream, one `gob.Encoder` per connection
(transport.go:99-116) and one `gob.Decoder` per accepted connection
(transport.go:146-165); the types travel under their gob.Register names
(message.go:8-17 and each protocol's msg.go).  Here:

- `capture(sim, cluster, steps)` steps a simulation one step at a time and
  records, before each step, every replica's inbox (paxisim_read_inbox): what
  each link delivers, in link (FIFO) order, plus the client's HTTP requests;
- `export(trace)` turns each directed link's messages into the bytes a Paxi
  sender's encoder writes on that connection (`gob.Encoder.Encode(&m)` with
  m an `interface{}`, paxi_amd/gob.py) and keeps the client requests, which
  travel over HTTP, and the delivery steps beside them;
- `import_streams(...)` decodes such streams back into simulator records;
- `replay(sim, cluster, trace)` delivers a trace into a simulation
  (paxisim_deliver): run with every link dropped and no client workers of its
  own, each replica then receives exactly the trace's messages at the trace's
  steps, so a replayed cluster retraces the captured one.

Messages map to Paxi values as follows (a ballot is the 64-bit
`n << 32 | zone << 16 | node`, an ID is "zone.node"):
  Request  paxi.Request{Command, NodeID = forwarder}          (node.go:165-172)
  Reply    paxi.Reply{Command, Value}                          (node.go:83-97; Value = Execute's result,
           paxos.go:352-362, as a write's value: Uvarint(cid) in 10 bytes, nil = 0)
  P1a..P3  paxos.P1a{Ballot} / P1b{Ballot, ID, Log} / P2a{Ballot, Slot, Command} /
           P2b{Ballot, ID, Slot} / P3{Ballot, Slot, Command}   (paxos/msg.go:19-70)
  ABD      abd.Get{ID, CID, Key} / GetReply{ID, CID, Key, Value, Version} /
           Set{...} / SetReply{ID, CID, Key}                   (abd/msg.go:16-46)
  WPaxos   wpaxos.Prepare{Key, P1a} / Promise{Key, P1b} / Accept{Key, P2a} /
           Accepted{Key, P2b} / Commit{Key, P3} / LeaderChange{Key, To, From, Ballot}
           (M2Paxos and KPaxos: the same shapes in packages m2paxos and kpaxos)
A Command is {Key = Bconfig.Min + key, Value = Uvarint(cid) in a 10-byte buffer
for a write (client/client.go:42-45) or nil for a read, ClientID "", CommandID
= cid}; the simulator derives key and kind from the command id
(paxisim_commands), so an imported command must agree with them.  Not carried
(the simulator has no such state): a Request's Timestamp and Properties, a
Reply's Properties / Err.
  EPaxos   epaxos.PreAccept / PreAcceptReply / Accept / AcceptReply / Commit (epaxos/msg.go:18-65)
"""
from __future__ import annotations

import json
import os

from . import abi, gob
from . import workload as _wl

T_REQUEST, T_REPLY, T_P1A, T_P1B, T_P1B_ENTRY, T_P2A, T_P2B, T_P3 = 1, 2, 3, 4, 5, 6, 7, 8
T_GET, T_GETREPLY, T_SET, T_SETREPLY, T_LEADERCHG = 9, 10, 11, 12, 13
T_PREACCEPT, T_PREACCEPTREPLY, T_ACCEPT, T_ACCEPTREPLY, T_COMMIT = 14, 15, 16, 17, 18

P = gob.PKG
PAXOS_NAMES = {T_P1A: f"{P}/paxos.P1a", T_P1B: f"{P}/paxos.P1b", T_P2A: f"{P}/paxos.P2a",
               T_P2B: f"{P}/paxos.P2b", T_P3: f"{P}/paxos.P3"}
_KEYED = {T_P1A: "Prepare", T_P1B: "Promise", T_P2A: "Accept", T_P2B: "Accepted", T_P3: "Commit",
          T_LEADERCHG: "LeaderChange"}
# the per-key protocols' wrappers, one package each (wpaxos/, m2paxos/, kpaxos/ msg.go)
KEYED_NAMES = {proto: {t: f"{P}/{pkg}.{n}" for t, n in _KEYED.items()}
               for proto, pkg in ((abi.WPAXOS, "wpaxos"), (abi.M2PAXOS, "m2paxos"), (abi.KPAXOS, "kpaxos"))}
WPAXOS_NAMES = KEYED_NAMES[abi.WPAXOS]
ABD_NAMES = {T_GET: f"{P}/abd.Get", T_GETREPLY: f"{P}/abd.GetReply", T_SET: f"{P}/abd.Set",
             T_SETREPLY: f"{P}/abd.SetReply"}
EPAXOS_NAMES = {T_PREACCEPT: f"{P}/epaxos.PreAccept", T_PREACCEPTREPLY: f"{P}/epaxos.PreAcceptReply",
                T_ACCEPT: f"{P}/epaxos.Accept", T_ACCEPTREPLY: f"{P}/epaxos.AcceptReply", T_COMMIT: f"{P}/epaxos.Commit"}
NAME_TYPE = {v: k for d in (PAXOS_NAMES, ABD_NAMES, EPAXOS_NAMES, *KEYED_NAMES.values()) for k, v in d.items()}
NAME_TYPE[f"{P}.Request"] = T_REQUEST
NAME_TYPE[f"{P}.Reply"] = T_REPLY


class TraceError(ValueError):
    pass


class Topology:
    """Replica index <-> ID "z.n" and compressed <-> 64-bit ballots (id.go, ballot.go:15-17)."""

    def __init__(self, cfg):
        self.ids = []
        for z in range(cfg.n_zones):
            for k in range(cfg.npz[z]):
                self.ids.append((z + 1, k + 1))
        self.N = len(self.ids)
        self.index = {f"{z}.{n}": r for r, (z, n) in enumerate(self.ids)}

    def id(self, r):
        z, n = self.ids[r]
        return f"{z}.{n}"

    def replica(self, ident):
        if ident not in self.index:
            raise TraceError(f"unknown replica ID {ident!r}")
        return self.index[ident]

    def ballot64(self, b):
        if b == 0:
            return 0
        z, n = self.ids[b & 15]
        return ((b >> 4) << 32) | (z << 16) | n

    def ep_ballot64(self, b):
        """EPaxos ballots are NewBallot(0, owner) (epaxos/replica.go:114), kept as 1 + owner index."""
        if b == 0:
            return 0
        z, n = self.ids[b - 1]
        return (z << 16) | n

    def ep_ballot32(self, b):
        if b == 0:
            return 0
        if b >> 32:
            raise TraceError("EPaxos ballots carry n = 0 here")
        return 1 + self.replica(f"{(b >> 16) & 0xFFFF}.{b & 0xFFFF}")

    def ballot32(self, b):
        if b == 0:
            return 0
        n, z, node = b >> 32, (b >> 16) & 0xFFFF, b & 0xFFFF
        r = self.replica(f"{z}.{node}")
        if n >= 1 << 27:
            raise TraceError("ballot counter beyond the simulator's 27 bits")
        return (n << 4) | r


def uvarint10(v: int) -> bytes:
    """binary.PutUvarint into make([]byte, binary.MaxVarintLen64) (client/client.go:42-45)."""
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out) + bytes(10 - len(out))


def read_uvarint(b: bytes) -> int:
    v, s = 0, 0
    for c in b:
        v |= (c & 0x7F) << s
        if c < 0x80:
            return v
        s += 7
    raise TraceError("truncated uvarint")


class Codec:
    """Records of one cluster <-> Paxi message values."""

    def __init__(self, sim, cluster):
        self.sim, self.cluster, self.cfg = sim, cluster, sim.cfg
        self.top = Topology(sim.cfg)
        self.kval = self._key_value                                       # key index <-> Command.Key
        self.kidx = lambda v: _wl.key_index(sim.wl, sim.cfg.keys, v)
        self.proto = sim.cfg.protocol
        self._cmd = {}

    def _key_value(self, k):
        # an exponential tail draw (index == keys) names a key the simulator
        # has no state for; the replicas raised UNFAITHFUL
        if k >= self.cfg.keys:
            raise TraceError(f"key index {k} lies beyond the key space (an exponential tail draw): "
                             "the simulator flags such commands UNFAITHFUL and cannot export them")
        return _wl.key_value(self.sim.wl, self.cfg.keys, k)

    def _commands(self, cids):
        todo = sorted({c for c in cids if c and c not in self._cmd})
        if todo:
            for c, kw in zip(todo, self.sim.commands(self.cluster, todo)):
                self._cmd[c] = kw

    def command(self, cid):
        key, write = self._cmd[cid]
        return {"Key": self.kval(key), "Value": uvarint10(cid) if write else None, "ClientID": "",
                "CommandID": cid}

    def check_command(self, c):
        cid = c["CommandID"]
        if not (1 <= cid < (1 << 27)):
            raise TraceError(f"command id {cid} outside the simulator's 27 bits")
        self._commands([cid])
        key, write = self._cmd[cid]
        if c["Key"] != self.kval(key) or (c["Value"] is not None) != write or \
                (write and read_uvarint(c["Value"]) != cid):
            raise TraceError(f"command {c} is not the simulator's command {cid}")
        return cid

    # records (one message: a header record and its payload records) -> (name, value)
    def to_go(self, src, recs):
        hdr, b, s, cid = recs[0][1:]
        if self.proto != abi.EPAXOS:
            self._commands([r[4] for r in recs])
        elif (hdr & 0xFF) in (T_PREACCEPT, T_COMMIT):
            self._commands([cid])
        t, key = hdr & 0xFF, hdr >> 16
        top = self.top
        if t == T_REQUEST:
            return f"{P}.Request", {"Command": self.command(cid), "NodeID": top.id(src)}
        if t == T_REPLY:
            return f"{P}.Reply", {"Command": self.command(cid), "Value": uvarint10(b) if b else None}
        if self.proto == abi.EPAXOS:
            return self._ep_to_go(src, t, b, s, cid, [w for r in recs[1:] for w in r[1:]])
        if self.proto == abi.ABD:
            k = self.kval((hdr >> 8) & 0xFF)
            v = {"ID": top.id(src), "CID": b, "Key": k}
            if t in (T_GETREPLY, T_SET):                    # {opid, version, value}
                v["Version"] = s
                v["Value"] = uvarint10(cid) if cid else None
            return ABD_NAMES[t], v
        if t == T_P1A:
            v = {"Ballot": top.ballot64(b)}
        elif t == T_P1B:
            log = {}
            for e in recs[1:]:
                log[e[3]] = {"Command": self.command(e[4]), "Ballot": top.ballot64(e[2])}
            v = {"Ballot": top.ballot64(b), "ID": top.id(src), "Log": log}   # make(map...) in HandleP1a: never nil
        elif t in (T_P2A, T_P3):
            v = {"Ballot": top.ballot64(b), "Slot": s, "Command": self.command(cid)}
        elif t == T_P2B:
            v = {"Ballot": top.ballot64(b), "ID": top.id(src), "Slot": s}
        elif t == T_LEADERCHG and self.proto in abi.PER_KEY:
            return KEYED_NAMES[self.proto][t], {"Key": self.kval(key), "To": top.id(s), "From": top.id(cid),
                                                "Ballot": top.ballot64(b)}
        else:
            raise TraceError(f"message type {t} has no Paxi wire form here")
        if self.proto in abi.PER_KEY:
            inner = {T_P1A: "P1a", T_P1B: "P1b", T_P2A: "P2a", T_P2B: "P2b", T_P3: "P3"}[t]
            return KEYED_NAMES[self.proto][t], {"Key": self.kval(key), inner: v}
        return PAXOS_NAMES[t], v

    # EPaxos (epaxos/msg.go:18-65): header {type | n << 8, ballot, slot, w3} + payload words
    # PreAccept w3 = cmd, [seq, Dep[N]]; PreAcceptReply w3 = seq, [Dep[N], Committed[N]];
    # Accept w3 = seq, [Dep[N]]; AcceptReply; Commit w3 = cmd, [seq, Dep[N]].  A Dep map holds
    # the positive entries only (attributes / merge add an id only above the zero default,
    # epaxos/replica.go:60-70, instance.go:29-40); Committed holds every id (-1 = none, replica.go:44).
    def _ep_to_go(self, src, t, b, s, w3, pay):
        top, N = self.top, self.top.N
        i32 = lambda u: u - (1 << 32) if u >= 1 << 31 else u
        deps = lambda ws: {top.id(k): i32(ws[k]) for k in range(N) if i32(ws[k]) > 0}
        v = {"Ballot": top.ep_ballot64(b), "Replica": top.id(src), "Slot": s}
        if t in (T_PREACCEPT, T_COMMIT):
            v.update({"Command": self.command(w3), "Seq": i32(pay[0]), "Dep": deps(pay[1:1 + N])})
        elif t == T_PREACCEPTREPLY:
            v.update({"Seq": i32(w3), "Dep": deps(pay[:N]),
                      "Committed": {top.id(k): i32(pay[N + k]) for k in range(N)}})
        elif t == T_ACCEPT:
            v.update({"Seq": i32(w3), "Dep": deps(pay[:N])})
        elif t != T_ACCEPTREPLY:
            raise TraceError(f"message type {t} has no EPaxos wire form")
        return EPAXOS_NAMES[t], v

    def _ep_from_go(self, src, t, v):
        top, N = self.top, self.top.N
        u32 = lambda x: x & 0xFFFFFFFF
        dep = lambda m: [u32((m or {}).get(top.id(k), 0)) for k in range(N)]
        b, s = top.ep_ballot32(v["Ballot"]), v["Slot"]
        if t in (T_PREACCEPT, T_COMMIT):
            w3, pay = self.check_command(v["Command"]), [u32(v["Seq"])] + dep(v["Dep"])
        elif t == T_PREACCEPTREPLY:
            com = v.get("Committed") or {}
            if len(com) != N:
                raise TraceError("PreAcceptReply.Committed must name every replica")
            w3, pay = u32(v["Seq"]), dep(v["Dep"]) + [u32(com[top.id(k)]) for k in range(N)]
        elif t == T_ACCEPT:
            w3, pay = u32(v["Seq"]), dep(v["Dep"])
        else:
            w3, pay = 0, []
        n = (len(pay) + 3) // 4
        pay = pay + [0] * (4 * n - len(pay))
        return [(src, t | (n << 8), b, s, w3)] + [(src, *pay[4 * k:4 * k + 4]) for k in range(n)]

    # (name, value) -> records
    def from_go(self, src, name, v):
        t = NAME_TYPE.get(name)
        if t is None:
            raise TraceError(f"no simulator form for {name}")
        top = self.top
        if t == T_REQUEST:
            return [(src, T_REQUEST, 0, 0, self.check_command(v["Command"]))]
        if t == T_REPLY:
            val = v.get("Value")
            return [(src, T_REPLY, read_uvarint(val) if val else 0, 0, self.check_command(v["Command"]))]
        if self.proto == abi.EPAXOS:
            if name not in EPAXOS_NAMES.values():
                raise TraceError(f"{name} is not an EPaxos message")
            return self._ep_from_go(src, t, v)
        if t in (T_GET, T_GETREPLY, T_SET, T_SETREPLY):
            k = self.kidx(v["Key"])
            val = v.get("Value")
            return [(src, t | (k << 8), v["CID"], v.get("Version", 0) if t in (T_GETREPLY, T_SET) else 0,
                     read_uvarint(val) if val else 0)]
        key = 0
        if self.proto in abi.PER_KEY:
            if name not in KEYED_NAMES[self.proto].values():
                raise TraceError(f"{name} is not a message of this protocol")
            key = self.kidx(v["Key"])
            if t == T_LEADERCHG:
                return [(src, t | (key << 16), top.ballot32(v["Ballot"]), top.replica(v["To"]),
                         top.replica(v["From"]))]
            v = v[{T_P1A: "P1a", T_P1B: "P1b", T_P2A: "P2a", T_P2B: "P2b", T_P3: "P3"}[t]]
        kt = key << 16
        if t == T_P1A:
            return [(src, T_P1A | kt, top.ballot32(v["Ballot"]), 0, 0)]
        if t == T_P1B:
            log = v.get("Log") or {}
            out = [(src, T_P1B | (len(log) << 8) | kt, top.ballot32(v["Ballot"]), 0, 0)]
            for slot in sorted(log):                     # uncommitted slots in ascending order
                cb = log[slot]
                out.append((src, T_P1B_ENTRY, top.ballot32(cb["Ballot"]), slot, self.check_command(cb["Command"])))
            return out
        if t in (T_P2A, T_P3):
            return [(src, t | kt, top.ballot32(v["Ballot"]), v["Slot"], self.check_command(v["Command"]))]
        if t == T_P2B:
            return [(src, T_P2B | kt, top.ballot32(v["Ballot"]), v["Slot"], 0)]
        raise TraceError(f"no simulator form for {name}")


def _split(recs):
    """Records of one source (FIFO) -> messages (a header and its payload records)."""
    out, i = [], 0
    while i < len(recs):
        h = recs[i][1]
        t = h & 0xFF
        n = 1 + (((h >> 8) & 0xFF) if t == T_P1B or 14 <= t <= 18 else 0)
        out.append(recs[i:i + n])
        i += n
    return out


def capture(sim, cluster, steps):
    """Step `sim` `steps` times, recording before each step what every replica
    receives.  Returns {"N", "t0", "steps", "msgs": [(step, src, dst, [records])]},
    in delivery order per link."""
    N = sim.N
    out = []
    t0 = sim.stats().steps
    wl = sim.wl
    for k in range(steps):
        t = t0 + k
        for dst in range(N):
            recs = sim.read_inbox(cluster, dst)
            by_src = {}
            for r in recs:
                by_src.setdefault(r[0], []).append(r)
            # a worker starting at this step (paxisim_workload.start_step) sends its first
            # request during the step, behind the ones already queued: not in the inbox yet
            for w in range(wl.outstanding):
                if t > 0 and wl.start_step[w] == t and wl.target[w] == dst:
                    by_src.setdefault(N, []).append((N, T_REQUEST, 0, 0, 1 + w))
            for src in sorted(by_src):
                for m in _split(by_src[src]):
                    out.append((t, src, dst, m))
        sim.step(1)
    return {"N": N, "t0": t0, "steps": steps, "msgs": out}


def export(sim, cluster, trace, outdir=None):
    """Per-link gob streams of a captured trace: {(src, dst): bytes} as a Paxi
    sender's encoder writes them, plus the schedule {"links": {"src->dst":
    [steps]}, "client": [(step, dst, cid)]}.  Every sending replica is its own
    Go process with its own type-id counter (encoding/gob's registry is per
    process), so one registry per source replica is shared by that replica's
    outgoing links.  With outdir, writes <src>-<dst>.gob files and
    schedule.json there."""
    codec = Codec(sim, cluster)
    regs = {}
    enc, sched, client = {}, {}, []
    N = trace["N"]
    for (t, src, dst, recs) in trace["msgs"]:
        if src == N:                                          # the HTTP path (http.go:99), not gob
            client.append((t, dst, recs[0][4]))
            continue
        name, v = codec.to_go(src, recs)
        if (src, dst) not in enc:
            enc[(src, dst)] = gob.Encoder(regs.setdefault(src, gob.TypeIds()))
        e = enc[(src, dst)]
        e.encode_interface(name, v)
        sched.setdefault(f"{src}->{dst}", []).append(t)
    streams = {k: e.getvalue() for k, e in enc.items()}
    schedule = {"N": N, "t0": trace["t0"], "steps": trace["steps"], "links": sched, "client": client,
                "ids": [codec.top.id(r) for r in range(N)]}
    if outdir:
        os.makedirs(outdir, exist_ok=True)
        for (src, dst), b in streams.items():
            with open(os.path.join(outdir, f"{src}-{dst}.gob"), "wb") as f:
                f.write(b)
        with open(os.path.join(outdir, "schedule.json"), "w") as f:
            json.dump(schedule, f)
    return streams, schedule


def import_streams(sim, cluster, streams, schedule):
    """Decode per-link gob streams into a trace (the inverse of export)."""
    codec = Codec(sim, cluster)
    N = schedule["N"]
    msgs = []
    for (src, dst), data in sorted(streams.items()):
        steps = schedule["links"][f"{src}->{dst}"]
        vals = list(gob.Decoder(data))
        if len(vals) != len(steps):
            raise TraceError(f"link {src}->{dst}: {len(vals)} messages, {len(steps)} steps")
        for t, (name, v) in zip(steps, vals):
            msgs.append((t, src, dst, [tuple(r) for r in codec.from_go(src, name, v)]))
    for (t, dst, cid) in schedule["client"]:
        msgs.append((t, N, dst, [(N, T_REQUEST, 0, 0, cid)]))
    return {"N": N, "t0": schedule["t0"], "steps": schedule["steps"], "msgs": msgs}


def load_dir(path):
    with open(os.path.join(path, "schedule.json")) as f:
        schedule = json.load(f)
    schedule["client"] = [tuple(c) for c in schedule["client"]]
    streams = {}
    for name in os.listdir(path):
        if name.endswith(".gob"):
            src, dst = (int(x) for x in name[:-4].split("-"))
            with open(os.path.join(path, name), "rb") as f:
                streams[(src, dst)] = f.read()
    return streams, schedule


def replay(sim, cluster, trace):
    """Deliver a trace into `sim` step by step: before step t, each (dst, src)
    gets the trace's records for step t, in link order.  The caller runs sim
    with every replica-to-replica link dropped and no client workers of its
    own (replay_config), so the replicas see exactly the trace."""
    by_step = {}
    for (t, src, dst, recs) in trace["msgs"]:
        by_step.setdefault(t, []).append((src, dst, recs))
    t0 = sim.stats().steps
    if t0 != trace["t0"]:
        raise TraceError(f"simulation at step {t0}, trace starts at {trace['t0']}")
    for k in range(trace["steps"]):
        per = {}
        for (src, dst, recs) in by_step.get(t0 + k, []):
            per.setdefault((dst, src), []).extend(recs)
        for (dst, src), recs in sorted(per.items()):
            sim.deliver(cluster, dst, src, recs)
        sim.step(1)


def replay_setup(wl, n_replicas, far=1 << 26):
    """Workload and scripted faults for a replay run: workers that never start
    (start_step far in the future) and every replica-to-replica link dropped
    for good (sends are counted and go nowhere), so only the replayed records
    move.  A Crash of the captured run is not in its trace (a crashed replica
    discards its inbox at Recv, socket.go:111-118): add it to the replay too."""
    for w in range(wl.outstanding):
        wl.start_step[w] = far
    return [abi.make_fault(abi.FAULT_DROP, r) for r in range(n_replicas)]
