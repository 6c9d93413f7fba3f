"""The benchmark's key generator on the GPU against the oracle (round-3
verdict item 1): Bconfig.Move's moving Mu for "normal" with the
Mu sequence crossing the wrap (benchmark.go:137-140, 221-227), the unbounded
"exponential" at K=16 without folding (232-233), and "conflict"'s literal key 0
with Min != 0 (213-214).  Two levels: the key function itself
(paxisim_commands against oracle_command over thousands of command ids), and
whole runs - Multi-Paxos and EPaxos executing into the Database, ABD, KPaxos
with its key-range leaders - compared replica by replica, Database by
Database, including the UNFAITHFUL flags a tail draw raises."""
import pytest

from paxi_amd import abi
import oracle_lib as ol

pytestmark = pytest.mark.gpu

WORKLOADS = {
    # Mu 5.5 -> 6 -> 0 (the wrap) -> 1 ... with K = 7, moving every 23 commands
    "normal_move": dict(distribution="normal", keys=8, mu=5.5, sigma=1.3, move_every=23),
    # a negative start: int() toward zero and Go's signed %, then the cycle
    "normal_move_neg": dict(distribution="normal", keys=8, mu=-2.5, sigma=0.8, move_every=5),
    "exponential16": dict(distribution="exponential", keys=16, lam=0.15),
    "conflict_min": dict(distribution="conflict", conflicts=35, key_min=100, key_space=8),
    "order_space": dict(distribution="order", key_space=5),
}
KEYS = {"normal_move": 8, "normal_move_neg": 8, "exponential16": 16, "conflict_min": 9, "order_space": 8}


@pytest.mark.parametrize("name", sorted(WORKLOADS))
def test_command_keys_match_oracle(name):
    from paxi_amd.sim import Simulation
    keys = KEYS[name]
    cfg = abi.make_config(protocol=abi.ABD, npz=[3], clusters=40, seed=11, keys=keys)
    wl = abi.make_workload(outstanding=3, target=[0, 1, 2], write_ppm=500_000, **WORKLOADS[name])
    g, o = Simulation(cfg, wl), ol.OracleSim(cfg, wl)
    cids = list(range(1, 3001))
    for c in (0, 7, 39):
        assert g.commands(c, cids) == [o.command(c, cid) for cid in cids]
    seen = {k for k, _ in g.commands(7, cids)}
    if name == "exponential16":
        assert keys in seen                                       # tail draws: beyond the key space
    if name == "conflict_min":
        assert 8 in seen                                          # the literal key 0
    g.close()
    o.close()


CASES = [
    (abi.PAXOS, (5,), "normal_move"), (abi.PAXOS, (5,), "exponential16"), (abi.PAXOS, (3,), "normal_move_neg"),
    (abi.EPAXOS, (3,), "exponential16"), (abi.ABD, (5,), "normal_move"), (abi.ABD, (3,), "exponential16"),
    (abi.ABD, (3,), "conflict_min"), (abi.KPAXOS, (3, 3), "conflict_min"), (abi.WPAXOS, (3, 3), "exponential16"),
]


@pytest.mark.parametrize("proto,npz,name", CASES)
def test_runs_match_oracle(proto, npz, name):
    from paxi_amd.sim import Simulation
    N, keys = sum(npz), KEYS[name]
    kw = dict(history=256) if proto == abi.ABD else dict(kv=1)
    cfg = abi.make_config(protocol=proto, npz=list(npz), clusters=130, seed=9, keys=keys, mbox_cap=32,
                          window=32 if proto == abi.EPAXOS else 16, **kw)
    wl = abi.make_workload(outstanding=N, target=list(range(N)), write_ppm=600_000, **WORKLOADS[name])
    fp = abi.make_fault_process(drop_ppm=1000, drop_len=10, slow_ppm=2000, slow_len=10, slow_min=1, slow_max=3)
    g, o = Simulation(cfg, wl, fp), ol.OracleSim(cfg, wl, fp)
    for _ in range(3):
        g.step(100)
        o.step(100)
        gs, os_ = [r.as_tuple() for r in g.read_state()], [r.as_tuple() for r in o.read_state()]
        assert gs == os_
    if proto in abi.PER_KEY:
        assert [i.as_tuple() for i in g.read_instances()] == [i.as_tuple() for i in o.read_instances()]
    if proto == abi.ABD:
        for c in range(0, 130, 13):
            assert g.history(c) == o.history(c)
    else:
        for c in range(0, 130, 11):
            for r in range(N):
                assert g.read_kv(c, r, keys) == o.read_kv(c, r, keys)
    unf = sum(1 for r in g.read_state() if r.flags & abi.F_UNFAITHFUL)
    if name == "exponential16":
        assert unf > 0                                            # tail keys are flagged, not folded
    assert sum(r.execute for r in g.read_state()) > 0
    g.close()
    o.close()
