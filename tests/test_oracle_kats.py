"""Pin the CPU oracle against the reference's own KATs and hand-derived ones
(tests/golden/kats.json; see tests/golden/make_kats.py for provenance)."""
import itertools
import json
import os

import pytest

from paxi_amd import abi
import oracle_lib as ol

KATS = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "kats.json")))


def test_ballot_test_go():
    k = KATS["ballot_test"]
    b = ol.new_ballot(k["start_n"], k["zone"], k["node"])
    for _ in range(k["nexts"]):
        b = ol.ballot_next(b, k["zone"], k["node"])
    assert b >> 32 == k["expect_n"]
    assert [(b >> 16) & 0xFFFF, b & 0xFFFF] == k["expect_id"]


@pytest.mark.parametrize("n,zone,node,val", KATS["ballot_values"])
def test_ballot_values(n, zone, node, val):
    assert ol.new_ballot(n, zone, node) == val


@pytest.mark.parametrize("n,need", [(int(k), v) for k, v in KATS["majority_min"].items()])
def test_majority_threshold(n, need):
    for size in range(n + 1):
        assert ol.quorum(abi.Q_MAJORITY, [n], (1 << size) - 1) == (size >= need)


@pytest.mark.parametrize("fz,q1min,q2min", KATS["fgrid_3x3_min"])
def test_fgrid_minimum_quorums(fz, q1min, q2min):
    npz = [3, 3, 3]
    if fz == 0:
        k1, k2 = abi.Q_GRID_ROW, abi.Q_GRID_COLUMN
    else:
        k1, k2 = abi.Q_FGRID_Q1, abi.Q_FGRID_Q2
    sizes1 = [bin(m).count("1") for m in range(1 << 9) if ol.quorum(k1, npz, m, fz)]
    sizes2 = [bin(m).count("1") for m in range(1 << 9) if ol.quorum(k2, npz, m, fz)]
    assert min(sizes1) == q1min and min(sizes2) == q2min
    # every phase-1 quorum intersects every phase-2 quorum (the FPaxos safety condition)
    q1s = [m for m in range(1 << 9) if ol.quorum(k1, npz, m, fz)]
    q2s = [m for m in range(1 << 9) if ol.quorum(k2, npz, m, fz)]
    assert all(a & b for a, b in itertools.product(q1s[::7], q2s[::7]))


@pytest.mark.parametrize("case", KATS["checker"], ids=[c["name"] for c in KATS["checker"]])
def test_checker_test_go(case):
    n = ol.linearizable([tuple(o) for o in case["ops"]])
    e = case["expect"]
    if e == "zero":
        assert n == 0
    elif e == "nonzero":
        assert n > 0
    else:
        assert n == e


def _config1(seed=1):
    k = KATS["config1"]
    cfg = abi.make_config(npz=k["npz"], clusters=1, seed=seed, window=32, mbox_cap=16, max_delay=0)
    wl = abi.make_workload(outstanding=1, max_requests=k["writes"], target=k["target"])
    return ol.OracleSim(cfg, wl), k


def test_config1_message_counts():
    sim, k = _config1()
    sim.step(k["writes"] * k["steps_per_request"] + 10)
    st = sim.stats()
    got = {abi.MSG_NAMES[i]: st.delivered[i] for i in range(abi.NMSG) if st.delivered[i]}
    assert got == k["delivered"]
    assert st.delivered_total == k["delivered_total"]
    assert st.commits == k["writes"] and st.replies == k["writes"]
    s = sim.read_state()
    leader = s[0]
    assert leader.ballot == k["leader_ballot"]
    assert leader.active == 1 and leader.slot == k["leader_slot"] and leader.execute == k["leader_execute"]
    assert all(r.execute == k["writes"] for r in s)
    assert len({r.digest for r in s}) == 1 and all(r.flags == 0 for r in s)
    logs = [sim.exec_log(0, r) for r in range(3)]
    assert logs[0] == logs[1] == logs[2] == list(range(1, k["writes"] + 1))
    assert sim.check() == 0


def test_config1_independent_of_seed():
    a, k = _config1(seed=1)
    b, _ = _config1(seed=12345)
    a.step(3010)
    b.step(3010)
    assert a.stats().delivered_total == b.stats().delivered_total == k["delivered_total"]


def test_inject_validates_arguments():
    sim, _ = _config1()
    with pytest.raises(RuntimeError):
        sim.inject(0, 3, 5)          # replica out of range
    with pytest.raises(RuntimeError):
        sim.inject(0, 0, 0)          # cid 0 is nil
    for k in range(16):
        sim.inject(0, 1, 100 + k)
    with pytest.raises(RuntimeError, match="mailbox full"):
        sim.inject(0, 1, 200)        # 1 worker request + 16 injected > mbox_cap 16
