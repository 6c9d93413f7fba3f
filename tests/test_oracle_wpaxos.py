"""CPU oracle: WPaxos (wpaxos/replica.go, wpaxos/kpaxos.go, policy.go) behaviour.

The reference ships no WPaxos test, so these are behavioural
properties of the restated handlers; bit-exact GPU parity against this oracle
is in test_parity_wpaxos_gpu.py.
"""
import pytest

from paxi_amd import abi
import oracle_lib as ol

N, Z = 9, 3


def wp_config(clusters=64, keys=8, seed=7, **kw):
    kw.setdefault("window", 16)
    kw.setdefault("mbox_cap", 24)
    kw.setdefault("max_delay", 0)
    kw.setdefault("policy_threshold", 3)
    return abi.make_config(protocol=abi.WPAXOS, npz=[3, 3, 3], keys=keys, clusters=clusters, seed=seed, **kw)


def leaders(o, clusters, keys):
    ins = o.read_instances()
    out = {}
    for c in range(clusters):
        for k in range(keys):
            out[c, k] = [r for r in range(N) if ins[(c * N + r) * keys + k].active]
    return out


def test_home_zone_leaders_under_full_locality():
    """Every key is requested only from its home zone (k mod 3): its leader ends up there."""
    cfg = wp_config(clusters=48)
    wl = abi.make_workload(outstanding=9, target=list(range(9)), locality_ppm=1_000_000)
    o = ol.OracleSim(cfg, wl)
    o.step(1500)
    st = o.stats().as_dict()
    assert st["commits"] > 0 and o.check() == 0
    assert st["flagged"][4] == 0 and st["flagged"][5] == 0      # no UNFAITHFUL, no POISON
    for (c, k), ls in leaders(o, 48, 8).items():
        assert len(ls) == 1 and ls[0] // 3 == k % Z, (c, k, ls)


def test_object_stealing_with_partial_locality():
    """70% locality: remote hits trigger LeaderChange + phase-1 steals (replica.go:55-63, 101-108)."""
    cfg = wp_config(clusters=64)
    wl = abi.make_workload(outstanding=9, target=list(range(9)), locality_ppm=700_000)
    o = ol.OracleSim(cfg, wl)
    o.step(2000)
    st = o.stats().as_dict()
    assert st["delivered"].get("LeaderChange", 0) > 0
    assert st["delivered"]["P1a"] > 64 * 8 * 8          # more phase-1s than one election per key
    assert o.check() == 0
    assert st["flagged"][4] == 0 and st["flagged"][5] == 0
    home = sum(1 for (c, k), ls in leaders(o, 64, 8).items() if ls and ls[0] // 3 == k % Z)
    assert home >= 0.6 * 64 * 8


def test_null_policy_never_migrates():
    cfg = wp_config(clusters=32, policy_threshold=0)
    wl = abi.make_workload(outstanding=9, target=list(range(9)), locality_ppm=500_000)
    o = ol.OracleSim(cfg, wl)
    o.step(800)
    st = o.stats().as_dict()
    assert "LeaderChange" not in st["delivered"] and st["commits"] > 0 and o.check() == 0


def test_non_adaptive_handles_locally():
    """-adaptive=false: every replica runs p.HandleRequest itself (replica.go:64-65): no
    policy, and proposers duel; pending requests still move via paxos.forward (paxos.go:371-376)."""
    cfg = wp_config(clusters=32, adaptive=0)
    wl = abi.make_workload(outstanding=9, target=list(range(9)), locality_ppm=700_000)
    o = ol.OracleSim(cfg, wl)
    o.step(800)
    st = o.stats().as_dict()
    assert "LeaderChange" not in st["delivered"]
    assert st["delivered"]["P1a"] > st["delivered"]["P2a"] / 4 and o.check() == 0


@pytest.mark.parametrize("fz", [0, 1, 2])
def test_fgrid_quorums_agree(fz):
    cfg = wp_config(clusters=32, fz=fz)
    wl = abi.make_workload(outstanding=9, target=list(range(9)), locality_ppm=700_000)
    fp = abi.make_fault_process(drop_ppm=2000, drop_len=20, slow_ppm=2000, slow_len=20, slow_min=1, slow_max=3)
    cfg.max_delay = 3
    o = ol.OracleSim(cfg, wl, fp)
    o.step(1000)
    st = o.stats().as_dict()
    # Under message loss the reference itself can diverge (see the KAT below), so
    # agreement is only required of most clusters here.
    assert st["commits"] > 0 and st["dropped"] > 0 and o.check() <= 3


def test_reference_gap_p1b_omits_committed_slots():
    """KAT for a divergence of the reference under loss, reproduced as Go would run it.

    HandleP1a (paxos/paxos.go:149-155) reports only *uncommitted* entries, and
    the new leader learns slot numbers only from P1b logs (update, 164-180).
    Seeded trace (cluster 26, seed 7, Grid quorums): link 3.2 -> 3.3 is in a
    drop window, so 3.3 never hears of key 2; 3.2 commits slot 0 = cmd 8 with
    everyone else.  At step 5 a request for key 2 reaches 3.3, whose fresh
    kpaxos runs phase 1 at ballot (1, 3.3); every P1b is empty, so 3.3 proposes
    cmd 18 at slot 0, acceptors re-create the executed slot (HandleP2a 240-258)
    and accept, zone 3 forms a GridColumn Q2, and 3.3 executes cmd 18 at slot 0
    while the other eight replicas executed cmd 8 there."""
    cfg = wp_config(clusters=1, cluster_base=26, max_delay=3)
    wl = abi.make_workload(outstanding=9, target=list(range(9)), locality_ppm=700_000)
    fp = abi.make_fault_process(drop_ppm=2000, drop_len=20, slow_ppm=2000, slow_len=20, slow_min=1, slow_max=3)
    o = ol.OracleSim(cfg, wl, fp)
    o.step(9)
    assert o.check() == 0
    o.step(1)
    assert o.check() == 1
    logs = [o.exec_log(0, r, key=2) for r in range(N)]
    assert logs[:8] == [[8]] * 8 and logs[8] == [18]
    ins = o.read_instances()
    leader = ins[8 * 8 + 2]
    assert leader.active == 1 and leader.ballot == (1 << 32) | (3 << 16) | 3


def test_per_key_exec_logs_agree():
    """Per key, every replica executed a prefix of one sequence (client.go:279-320 per key)."""
    cfg = wp_config(clusters=4, keys=4)
    wl = abi.make_workload(outstanding=6, target=[0, 3, 6, 1, 4, 7], locality_ppm=700_000)
    o = ol.OracleSim(cfg, wl)
    o.step(600)
    for c in range(4):
        for k in range(4):
            logs = [o.exec_log(c, r, key=k) for r in range(N)]
            longest = max(logs, key=len)
            assert len(longest) > 0
            for lg in logs:
                assert lg == longest[:len(lg)], (c, k)


@pytest.mark.parametrize("keys", [0, 33])
def test_key_range_rejected(keys):
    cfg = wp_config(clusters=1, keys=keys)
    with pytest.raises(RuntimeError):
        ol.OracleSim(cfg, abi.make_workload(outstanding=1))


def _policy_run(policy, clusters=48, steps=1200, **kw):
    cfg = wp_config(clusters=clusters, policy=policy, **kw)
    wl = abi.make_workload(outstanding=9, target=list(range(9)), locality_ppm=700_000)
    o = ol.OracleSim(cfg, wl)
    o.step(steps)
    return o, o.stats().as_dict(), o.read_instances()


@pytest.mark.parametrize("interval", [1, 10, 60])
def test_majority_policy_migrates_and_resets_per_interval(interval):
    """majority.Hit (policy.go:79-101): LeaderChanges happen, and every instance's
    interval started no later than now and is at most `interval` old unless idle."""
    o, st, ins = _policy_run(abi.POLICY_MAJORITY, policy_interval=interval)
    assert st["commits"] > 0 and st["flagged"][5] == 0
    assert st["delivered"]["LeaderChange"] > 0
    for s in ins:
        if s.exists:
            assert s.policy_state[1] <= 1200
    # shorter intervals decide more often
    if interval == 1:
        _, st60, _ = _policy_run(abi.POLICY_MAJORITY, policy_interval=60)
        assert st["delivered"]["LeaderChange"] > st60["delivered"]["LeaderChange"]


@pytest.mark.parametrize("alpha", [0.3, 0.7, 1.0])
def test_ema_policy_state(alpha):
    """ema.Hit (policy.go:111-130): s stays within [1, Z] and the settled zone is
    one of the zones; alpha = 1 follows the last requester's zone."""
    import struct
    o, st, ins = _policy_run(abi.POLICY_EMA, policy_alpha=alpha)
    assert st["commits"] > 0 and st["flagged"][5] == 0
    seen = 0
    for s in ins:
        if not s.exists:
            continue
        v = struct.unpack("<d", struct.pack("<II", s.policy_state[0], s.policy_state[1]))[0]
        assert v == 0.0 or 1.0 <= v <= Z
        assert s.policy_state[2] <= Z
        seen += v != 0.0
    assert seen > 0
    assert st["delivered"]["LeaderChange"] > 0


def test_policy_config_is_validated():
    wl = abi.make_workload(outstanding=9, target=list(range(9)))
    for kw in (dict(policy=3), dict(policy=abi.POLICY_MAJORITY, policy_interval=0),
               dict(policy=abi.POLICY_EMA, policy_alpha=0.0), dict(policy=abi.POLICY_EMA, policy_alpha=1.5)):
        with pytest.raises(RuntimeError):
            ol.OracleSim(wp_config(clusters=2, **kw), wl)
