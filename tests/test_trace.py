"""Message traces in Paxi's wire format (paxi_amd/gob.py, paxi_amd/trace.py):
the gob primitives against encoding/gob's documented examples, gob round
trips of every Paxi message type, capture -> gob export -> import -> replay
on the oracle (CPU) and on the HIP path (-m gpu), and GPU-vs-oracle parity
of the inbox reads the capture is built on."""
import json
import os

import pytest

from paxi_amd import abi, gob, trace
from oracle_lib import OracleSim

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "gob_kats.json")


def kats():
    with open(GOLD) as f:
        return json.load(f)


def test_gob_primitives_match_documentation():
    k = kats()
    for v, h in k["uint"]:
        assert gob.enc_uint(v).hex() == h
        assert gob.Reader(bytes.fromhex(h)).uint() == v
    for v, h in k["int"]:
        assert gob.enc_int(v).hex() == h
        assert gob.Reader(bytes.fromhex(h)).int() == v
    for v, h in k["string"]:
        assert gob.enc_bytes(v.encode()).hex() == h
    for v, h in k["float"]:
        assert gob.enc_float(v).hex() == h
        assert gob._float(gob.Reader(bytes.fromhex(h)).uint()) == v


def test_gob_point_example():
    """Point{22, 33} in a fresh process, byte for byte as the documentation gives it."""
    assert gob.encode_point_example(22, 33).hex() == kats()["point_22_33"]


P = gob.PKG
CMD_W = {"Key": 7, "Value": trace.uvarint10(300), "ClientID": "", "CommandID": 300}
CMD_R = {"Key": 3, "Value": None, "ClientID": "", "CommandID": 5}
SAMPLES = [
    (f"{P}.Request", {"Command": CMD_W, "Properties": None, "Timestamp": 0, "NodeID": "1.2"}),
    (f"{P}.Reply", {"Command": CMD_R, "Value": None, "Properties": None, "Timestamp": 0, "Err": None}),
    (f"{P}/paxos.P1a", {"Ballot": (3 << 32) | (1 << 16) | 2}),
    (f"{P}/paxos.P1b", {"Ballot": 4295032833, "ID": "1.3", "Log": {}}),
    (f"{P}/paxos.P1b", {"Ballot": 4295032833, "ID": "1.3",
                        "Log": {4: {"Command": CMD_W, "Ballot": 4295032833}, 2: {"Command": CMD_R, "Ballot": 7}}}),
    (f"{P}/paxos.P2a", {"Ballot": 4295032833, "Slot": 0, "Command": CMD_W}),
    (f"{P}/paxos.P2b", {"Ballot": 4295032833, "ID": "1.2", "Slot": 9}),
    (f"{P}/paxos.P3", {"Ballot": 0, "Slot": 1 << 20, "Command": CMD_R}),
    (f"{P}/abd.Get", {"ID": "1.1", "CID": 3, "Key": 0}),
    (f"{P}/abd.GetReply", {"ID": "1.2", "CID": 3, "Key": 2, "Value": trace.uvarint10(1 << 40), "Version": 4}),
    (f"{P}/abd.Set", {"ID": "1.1", "CID": 3, "Key": 2, "Value": None, "Version": 0}),
    (f"{P}/abd.SetReply", {"ID": "1.4", "CID": 99, "Key": 1}),
    (f"{P}/wpaxos.Prepare", {"Key": 5, "P1a": {"Ballot": 8590065667}}),
    (f"{P}/wpaxos.Promise", {"Key": 5, "P1b": {"Ballot": 8590065667, "ID": "2.3", "Log": {}}}),
    (f"{P}/wpaxos.Accept", {"Key": 5, "P2a": {"Ballot": 8590065667, "Slot": 2, "Command": CMD_R}}),
    (f"{P}/wpaxos.Accepted", {"Key": 0, "P2b": {"Ballot": 8590065667, "ID": "3.1", "Slot": 2}}),
    (f"{P}/wpaxos.Commit", {"Key": 5, "P3": {"Ballot": 8590065667, "Slot": 2, "Command": CMD_W}}),
    (f"{P}/wpaxos.LeaderChange", {"Key": 5, "To": "2.1", "From": "1.1", "Ballot": 8590065667}),
    (f"{P}/epaxos.PreAccept", {"Ballot": 65537, "Replica": "1.1", "Slot": 3, "Command": CMD_W, "Seq": 4,
                               "Dep": {"1.2": 2, "2.1": 7}}),
    (f"{P}/epaxos.PreAcceptReply", {"Ballot": 65537, "Replica": "1.2", "Slot": 3, "Seq": 5, "Dep": {},
                                    "Committed": {"1.1": 2, "1.2": -1, "2.1": 0}}),
    (f"{P}/epaxos.Accept", {"Ballot": 65537, "Replica": "1.1", "Slot": 3, "Seq": 5, "Dep": {"1.2": 2}}),
    (f"{P}/epaxos.AcceptReply", {"Ballot": 65537, "Replica": "2.1", "Slot": 3}),
    (f"{P}/epaxos.Commit", {"Ballot": 65537, "Replica": "1.1", "Slot": 3, "Command": CMD_R, "Seq": 5,
                            "Dep": {"1.2": 2}}),
]


def test_gob_roundtrip_every_message_type():
    """Every registered type through one encoder (one connection): each decodes
    to what was sent, zero fields included, and type definitions go out once."""
    e = gob.Encoder()
    sizes = []
    for name, v in SAMPLES + SAMPLES:
        sizes.append(len(e.encode_interface(name, v)))
    got = list(gob.Decoder(e.getvalue()))
    assert got == SAMPLES + SAMPLES
    first, again = sizes[:len(SAMPLES)], sizes[len(SAMPLES):]
    assert all(b <= a for a, b in zip(first, again)) and sum(again) < sum(first)


def test_gob_type_ids_follow_a_fresh_process():
    """P2a first: P2a takes 65 before its fields, Command 66 (a struct takes its
    id before its fields are built); definitions precede the first value."""
    reg = gob.TypeIds()
    e = gob.Encoder(reg)
    data = e.encode_interface(f"{P}/paxos.P2a", SAMPLES[5][1])
    assert reg.id_of(gob.P2A) == 65 and reg.id_of(gob.COMMAND) == 66
    r = gob.Reader(data)
    n1 = r.uint()
    m1 = gob.Reader(r.take(n1))
    assert m1.int() == gob.INTERFACE and m1.uint() == 0
    assert m1.take(m1.uint()).decode() == f"{P}/paxos.P2a"
    assert m1.int() == -65                           # P2a's definition continues the first message
    n2 = r.uint()
    assert gob.Reader(r.take(n2)).int() == -66       # Command's in a message of its own
    n3 = r.uint()
    assert gob.Reader(r.take(n3)).int() == 65        # then the value
    assert r.left() == 0
    # a P1b afterwards: its map type takes its id after CommandBallot
    e.encode_interface(f"{P}/paxos.P1b", SAMPLES[4][1])
    assert reg.id_of(gob.COMMAND_BALLOT) == 68 and reg.id_of(gob.P1B) == 67
    assert reg.id_of(gob.P1B.fields[2][1]) == 69


def test_gob_decoder_accepts_inline_definitions():
    """doc.go's grammar also allows an interface's later type definitions
    delimited inside the same message (decodeTypeSequence skips their count)."""
    e = gob.Encoder()
    e.encode_interface(f"{P}/paxos.P2a", SAMPLES[5][1])
    r = gob.Reader(e.getvalue())
    msgs = []
    while r.left():
        msgs.append(r.take(r.uint()))
    inline = msgs[0] + gob.enc_uint(len(msgs[1])) + msgs[1] + gob.enc_uint(len(msgs[2])) + msgs[2]
    assert list(gob.Decoder(gob.enc_uint(len(inline)) + inline)) == [SAMPLES[5]]


def test_gob_rejects_garbage():
    with pytest.raises(gob.GobError):
        list(gob.Decoder(b"\x05\x10\x00\x03abc"))
    with pytest.raises(gob.GobError):
        gob.Encoder().encode_interface("main.Unregistered", {})


# ---- capture / export / import / replay -------------------------------------
def paxos_case(clusters=6, base=0, fp=True):
    cfg = abi.make_config(npz=[5], clusters=clusters, cluster_base=base, seed=11, window=16, mbox_cap=16,
                          max_delay=3, kv=1)
    wl = abi.make_workload(outstanding=4, target=[0, 0, 1, 2], write_ppm=600_000, keys=8)
    f = abi.make_fault_process(drop_ppm=8000, drop_len=10, slow_ppm=8000, slow_len=10, slow_min=1,
                               slow_max=3) if fp else None
    return cfg, wl, f


def wpaxos_case(clusters=4, base=0):
    cfg = abi.make_config(protocol=abi.WPAXOS, npz=[3, 3, 3], keys=6, fz=0, adaptive=1, policy_threshold=2,
                          clusters=clusters, cluster_base=base, seed=5, window=16, mbox_cap=24, max_delay=0)
    wl = abi.make_workload(outstanding=9, target=list(range(9)), locality_ppm=700_000, write_ppm=500_000,
                           key_min=1000)
    return cfg, wl, None


def abd_case(clusters=4, base=0):
    cfg = abi.make_config(protocol=abi.ABD, npz=[5], clusters=clusters, cluster_base=base, seed=3, keys=4,
                          mbox_cap=16, max_delay=2, history=64)
    wl = abi.make_workload(outstanding=3, target=[0, 1, 2], write_ppm=500_000)
    return cfg, wl, None


def perkey_case(proto):
    def mk(clusters=4, base=0):
        cfg = abi.make_config(protocol=proto, npz=[3, 3, 3], keys=16, clusters=clusters, cluster_base=base,
                              seed=9, window=16, mbox_cap=24, max_delay=0)
        wl = abi.make_workload(outstanding=9, target=list(range(9)), locality_ppm=700_000, key_min=192,
                               write_ppm=500_000)
        return cfg, wl, None
    return mk


def epaxos_case(clusters=4, base=0):
    cfg = abi.make_config(protocol=abi.EPAXOS, npz=[2, 2, 1], clusters=clusters, cluster_base=base, seed=11, keys=4,
                          window=32, mbox_cap=32, max_delay=2)
    wl = abi.make_workload(outstanding=5, target=list(range(5)), write_ppm=700_000)
    fp = abi.make_fault_process(drop_ppm=1500, drop_len=10, slow_ppm=3000, slow_len=20, slow_min=1, slow_max=2)
    return cfg, wl, fp


CASES = {"paxos": paxos_case, "wpaxos": wpaxos_case, "abd": abd_case, "m2paxos": perkey_case(abi.M2PAXOS),
         "kpaxos": perkey_case(abi.KPAXOS), "epaxos": epaxos_case}
KEEP = lambda t: t[:11] + t[12:14] + t[15:]   # replica state minus dropped and replies (the replay drops every send)


def replay_from_zero(backend, case, cluster=3, steps=150, tmpdir=None):
    mk = CASES[case]
    cfg, wl, fp = mk()
    a = backend(cfg, wl, fp)
    tr = trace.capture(a, cluster, steps)
    streams, sched = trace.export(a, cluster, tr, outdir=tmpdir)
    if tmpdir:
        streams, sched = trace.load_dir(tmpdir)
    tr2 = trace.import_streams(a, cluster, streams, sched)
    key = lambda m: (m[0], m[1], m[2], m[3])
    assert sorted(tr2["msgs"], key=key) == sorted(tr["msgs"], key=key)
    cfg2, wl2, _ = mk(clusters=1, base=cluster)
    faults = trace.replay_setup(wl2, abi.n_replicas(cfg2))
    b = backend(cfg2, wl2, None, faults)
    trace.replay(b, 0, tr2)
    sa = [KEEP(s.as_tuple()) for s in a.read_state(cluster, 1)]
    sb = [KEEP(s.as_tuple()) for s in b.read_state(0, 1)]
    return a, b, tr, streams, sa, sb


@pytest.mark.parametrize("case", ["paxos", "wpaxos", "abd", "m2paxos", "kpaxos", "epaxos"])
def test_replay_oracle(case, tmp_path):
    a, b, tr, streams, sa, sb = replay_from_zero(OracleSim, case, tmpdir=str(tmp_path))
    assert len(tr["msgs"]) > 100 and len(streams) >= 4
    assert sa == sb
    if case not in ("abd",):
        ia = [i.as_tuple() for i in a.read_instances(3, 1)]
        ib = [i.as_tuple() for i in b.read_instances(0, 1)]
        assert ia == ib


def test_trace_stream_per_link_is_fifo():
    """Each link's stream decodes in the order its messages were delivered."""
    cfg, wl, fp = paxos_case()
    a = OracleSim(cfg, wl, fp)
    tr = trace.capture(a, 2, 60)
    streams, sched = trace.export(a, 2, tr)
    codec = trace.Codec(a, 2)
    for (src, dst), data in streams.items():
        want = [codec.to_go(s, recs) for (t, s, d, recs) in tr["msgs"] if (s, d) == (src, dst)]
        assert list(gob.Decoder(data)) == [(n, gob.full(gob.REGISTERED[n], v)) for n, v in want]
        assert sched["links"][f"{src}->{dst}"] == sorted(sched["links"][f"{src}->{dst}"])


def test_type_ids_are_per_sending_replica():
    """Each replica is its own Go process: the first type a sender defines takes
    id 65 in that sender's first stream, whatever other senders defined first."""
    cfg, wl, fp = paxos_case()
    a = OracleSim(cfg, wl, fp)
    tr = trace.capture(a, 2, 60)
    streams, _ = trace.export(a, 2, tr)
    first_link = {}
    for (t, s, d, recs) in tr["msgs"]:
        if s < tr["N"]:
            first_link.setdefault(s, (s, d))
    assert len(first_link) >= 2
    for src, link in first_link.items():
        r = gob.Reader(streams[link])
        m = gob.Reader(r.take(r.uint()))
        assert m.int() == gob.INTERFACE and m.uint() == 0
        m.take(m.uint())                                  # the registered name
        assert m.int() == -65, f"sender {src}"


def test_keyed_protocols_use_their_own_package():
    """m2paxos.Accept and wpaxos.Accept are distinct registered Go types: each
    protocol exports its own, and imports refuse the other's."""
    cfg, wl, _ = CASES["m2paxos"]()
    a = OracleSim(cfg, wl)
    tr = trace.capture(a, 1, 40)
    streams, sched = trace.export(a, 1, tr)
    names = {n for data in streams.values() for n, _ in gob.Decoder(data)}
    assert names and all(n.startswith(f"{P}/m2paxos.") or n in (f"{P}.Request", f"{P}.Reply") for n in names)
    codec = trace.Codec(a, 1)
    with pytest.raises(trace.TraceError):
        codec.from_go(0, f"{P}/wpaxos.Prepare", {"Key": 192, "P1a": {"Ballot": 4295032833}})


def test_import_rejects_foreign_commands():
    cfg, wl, fp = paxos_case()
    a = OracleSim(cfg, wl, fp)
    codec = trace.Codec(a, 0)
    bad = dict(CMD_W)
    bad["CommandID"] = 5
    with pytest.raises(trace.TraceError):
        codec.from_go(1, f"{P}/paxos.P2a", {"Ballot": 4295032833, "Slot": 0, "Command": bad})
    with pytest.raises(trace.TraceError):
        codec.from_go(1, f"{P}/paxos.P2b", {"Ballot": (1 << 32) | (9 << 16) | 1, "ID": "1.2", "Slot": 0})


# ---- on the GPU --------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("case", ["paxos", "wpaxos", "abd"])
def test_read_inbox_parity_gpu(case):
    from paxi_amd.sim import Simulation
    cfg, wl, fp = CASES[case]()
    g, o = Simulation(cfg, wl, fp), OracleSim(cfg, wl, fp)
    for _ in range(6):
        for c in range(cfg.clusters):
            for r in range(abi.n_replicas(cfg)):
                assert g.read_inbox(c, r) == o.read_inbox(c, r)
        g.step(17)
        o.step(17)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["paxos", "wpaxos", "abd", "m2paxos", "kpaxos", "epaxos"])
def test_replay_gpu(case):
    """Capture on the GPU, gob export and import, replay on the GPU: the replayed
    cluster retraces the captured one, and both equal the oracle's."""
    from paxi_amd.sim import Simulation
    a, b, tr, streams, sa, sb = replay_from_zero(Simulation, case)
    assert sa == sb
    o = OracleSim(*CASES[case]())
    o.step(150)
    assert [KEEP(s.as_tuple()) for s in o.read_state(3, 1)] == sa
    cfg, wl, fp = CASES[case]()
    oa = OracleSim(cfg, wl, fp)
    otr = trace.capture(oa, 3, 150)
    ostreams, _ = trace.export(oa, 3, otr)
    assert ostreams == streams                    # the same bytes on every link


@pytest.mark.gpu
def test_deliver_into_frozen_cluster_gpu():
    """paxisim_deliver wakes a compacted (frozen) cluster like paxisim_inject does."""
    from paxi_amd.sim import Simulation
    cfg, wl, fp = paxos_case(clusters=130, fp=False)
    wl2 = abi.make_workload(outstanding=1, target=0, max_requests=2)
    g, o = Simulation(cfg, wl2, None), OracleSim(cfg, wl2, None)
    g.step(200)
    o.step(200)
    rec = [(5, trace.T_REQUEST, 0, 0, 77)]
    g.deliver(129, 0, 5, rec)
    o.deliver(129, 0, 5, rec)
    g.step(40)
    o.step(40)
    assert [s.as_tuple() for s in g.read_state()] == [s.as_tuple() for s in o.read_state()]


@pytest.mark.parametrize("config", [2, 4, 5])
def test_trace_cli_roundtrip_oracle(config, tmp_path):
    """tools/trace_cli.py: capture a BASELINE config's cluster to gob files, then
    replay them from the files alone (the oracle stands in for the GPU here)."""
    import argparse
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import trace_cli
    d = str(tmp_path)
    trace_cli.capture(argparse.Namespace(config=config, cluster=5, clusters=8, steps=120, crash_step=40, out=d),
                      backend=OracleSim)
    assert trace_cli.replay(argparse.Namespace(dir=d), backend=OracleSim)


@pytest.mark.gpu
@pytest.mark.parametrize("config", [2, 4, 5])
def test_trace_cli_roundtrip_gpu(config, tmp_path):
    """tools/trace_cli.py on the HIP path: capture and replay on the GPU."""
    import argparse
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import trace_cli
    d = str(tmp_path)
    trace_cli.capture(argparse.Namespace(config=config, cluster=5, clusters=70, steps=150, crash_step=40, out=d))
    assert trace_cli.replay(argparse.Namespace(dir=d))


def test_gob_omitted_float_and_complex_fields_decode_as_zero():
    """Go omits zero-valued fields on the wire and decodes them as 0.0 and 0i."""
    name = "example.Sample"
    t = gob.Struct("Sample", [("X", gob.INT), ("F", gob.FLOAT), ("Z", gob.COMPLEX)])
    gob.REGISTERED[name] = t
    try:
        e = gob.Encoder()
        e.encode_interface(name, {"X": 3, "F": 0.0, "Z": 0j})
        e.encode_interface(name, {"X": 0, "F": 17.0, "Z": complex(1.5, -2.0)})
        got = list(gob.Decoder(e.getvalue()))
        assert got == [(name, {"X": 3, "F": 0.0, "Z": 0j}), (name, {"X": 0, "F": 17.0, "Z": complex(1.5, -2.0)})]
        assert isinstance(got[0][1]["F"], float) and isinstance(got[0][1]["Z"], complex)
        assert gob.full(t, {"X": 3}) == {"X": 3, "F": 0.0, "Z": 0j}
    finally:
        del gob.REGISTERED[name]


def test_reply_value_travels_in_the_trace():
    """A forwarded request's Reply carries Execute's value (paxos.go:352-362)
    over the wire back to the forwarder, and import restores it."""
    cfg, wl, fp = paxos_case()
    wl.target[1] = 2                                          # a worker at a follower: its requests are forwarded
    a = OracleSim(cfg, wl, fp)
    tr = trace.capture(a, 1, 120)
    streams, sched = trace.export(a, 1, tr)
    vals = [v["Value"] for data in streams.values() for n, v in gob.Decoder(data) if n == f"{P}.Reply"]
    assert vals and any(x is not None for x in vals)
    back = trace.import_streams(a, 1, streams, sched)
    reps = [r for (t, s, d, recs) in back["msgs"] for r in recs if r[1] == trace.T_REPLY]
    assert any(r[2] for r in reps)


def test_export_refuses_exponential_tail_commands():
    """An exponential tail draw (key index == keys) has no Command.Key in the
    model: the codec raises TraceError, not a bare ValueError
    (ADVICE r4)."""
    cfg = abi.make_config(npz=[3], clusters=2, seed=4, keys=4, kv=1)
    wl = abi.make_workload(outstanding=2, target=0, write_ppm=500_000, distribution="exponential", keys=4, lam=0.1)
    a = OracleSim(cfg, wl)
    codec = trace.Codec(a, 0)
    tail = [c for c in range(1, 400) if a.command(0, c)[0] == 4]
    fine = [c for c in range(1, 400) if a.command(0, c)[0] < 4]
    assert tail and fine
    codec._commands([tail[0], fine[0]])
    assert codec.command(fine[0])["Key"] == a.command(0, fine[0])[0]
    with pytest.raises(trace.TraceError):
        codec.command(tail[0])
    a.close()
