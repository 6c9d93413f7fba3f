"""M2Paxos (m2paxos/replica.go, m2paxos/kpaxos.go) and KPaxos (kpaxos/replica.go):
per-key paxos.Paxos instances like WPaxos, with Majority quorums.  M2Paxos
steals leadership by the policy (always adaptive); KPaxos has a static leader
per key range (index(), kpaxos/replica.go:32-44: "z.1" for z = 1 + key/200).
Hand-derived known answers on the oracle; GPU parity under -m gpu."""
import pytest

from paxi_amd import abi
import oracle_lib as ol
from test_parity_wpaxos_gpu import run_and_compare


def cfg(proto, npz=(3, 3, 3), clusters=1, keys=1, **kw):
    kw.setdefault("window", 16)
    kw.setdefault("mbox_cap", 24)
    kw.setdefault("max_delay", 0)
    return abi.make_config(protocol=proto, npz=list(npz), clusters=clusters, keys=keys, seed=3, **kw)


@pytest.mark.parametrize("proto", [abi.M2PAXOS, abi.KPAXOS])
def test_single_write_is_one_paxos_round(proto):
    """One request at 1.1 for key 0: P1a broadcast, a Majority of P1bs (2 of
    3 with the self-ack), P2a, P2b, P3 — 10 socket messages, as Multi-Paxos."""
    o = ol.OracleSim(cfg(proto, npz=(3,)), abi.make_workload(outstanding=1, max_requests=1, target=[0]))
    o.step(12)
    st = o.stats().as_dict()
    assert st["delivered"] == {"P1a": 2, "P1b": 2, "P2a": 2, "P2b": 2, "P3": 2}
    assert st["commits"] == 1 and st["replies"] == 1
    leader = o.read_instances(0, 1)[0]
    assert leader.ballot == (1 << 32) | (1 << 16) | 1 and leader.active == 1 and leader.execute == 1


def test_m2paxos_phase1_on_majority_not_grid_row():
    """3 zones of 1 node, the P1b of 3.1 lost: WPaxos' Q1 (GridRow: an ack in
    every zone, wpaxos/kpaxos.go:15-20) never forms, M2Paxos' Majority (2 of 3
    with the self-ack, m2paxos/kpaxos.go:15-17) does and the write commits."""
    wl = abi.make_workload(outstanding=1, max_requests=1, target=[0])
    faults = [abi.make_fault(abi.FAULT_DROP, 2, 0, step_from=1, step_to=2)]   # the P1b 3.1 -> 1.1
    res = {}
    for proto in (abi.WPAXOS, abi.M2PAXOS):
        o = ol.OracleSim(cfg(proto, npz=(1, 1, 1)), wl, faults=faults)
        o.step(12)
        res[proto] = (o.stats().commits, o.read_instances(0, 1)[0].active)
    assert res[abi.M2PAXOS] == (1, 1) and res[abi.WPAXOS] == (0, 0)


def test_kpaxos_static_leaders_by_key_range():
    """Bconfig.Min = 190, 16 keys: values 190..199 are led by 1.1, 200..205 by
    2.1; requests elsewhere are forwarded there; nobody steals."""
    wl = abi.make_workload(outstanding=9, target=list(range(9)), key_min=190)
    o = ol.OracleSim(cfg(abi.KPAXOS, clusters=8, keys=16), wl)
    o.step(300)
    inst = o.read_instances()
    for c in range(8):
        for r in range(9):
            for k in range(16):
                i = inst[(c * 9 + r) * 16 + k]
                if i.active:
                    assert r == (0 if k < 10 else 3)
    st = o.stats().as_dict()
    assert "LeaderChange" not in st["delivered"] and st["delivered"]["Request"] > 0 and o.check() == 0


def test_kpaxos_leader_outside_configuration():
    """One zone: keys 200.. map to "2.1", which does not exist — the forward is
    a send to an unknown address (socket.go:86-88), dropped, never answered."""
    wl = abi.make_workload(outstanding=2, target=[0, 1], key_min=199, max_requests=30)
    o = ol.OracleSim(cfg(abi.KPAXOS, npz=(3,), clusters=4, keys=2), wl)
    o.step(200)
    st = o.stats().as_dict()
    assert st["dropped"] > 0 and st["replies"] < 2 * 30 * 4


@pytest.mark.gpu
@pytest.mark.parametrize("proto", [abi.M2PAXOS, abi.KPAXOS])
@pytest.mark.parametrize("faults", [False, True])
def test_gpu_parity(proto, faults):
    wl = abi.make_workload(outstanding=9, target=list(range(9)), locality_ppm=700_000, key_min=192)
    fp = abi.make_fault_process(drop_ppm=2000, drop_len=20, slow_ppm=2000, slow_len=20, slow_min=0,
                                slow_max=0) if faults else None
    sc = [abi.make_fault(abi.FAULT_CRASH, 3, step_from=100, step_to=180)] if faults else []
    st = run_and_compare(cfg(proto, clusters=150, keys=16), wl, fp, sc, chunks=(140, 161))
    assert st["commits"] > 0
