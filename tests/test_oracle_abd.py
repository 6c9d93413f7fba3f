"""ABD (abd/replica.go) on the CPU oracle: message accounting and the
linearizability behaviour the reference's versioning implies."""
import pytest

from paxi_amd import abi
import oracle_lib as ol


def abd(clusters=64, outstanding=4, target=(0, 1, 2, 3), write_ppm=500_000, npz=(5,), fp=None, keys=16, seed=7,
        history=512):
    cfg = abi.make_config(protocol=abi.ABD, npz=list(npz), clusters=clusters, seed=seed, keys=keys, history=history)
    wl = abi.make_workload(outstanding=outstanding, target=list(target), write_ppm=write_ppm)
    return ol.OracleSim(cfg, wl, fp)


def test_messages_per_op():
    """No faults: every op is Get + GetReply + Set + SetReply to/from N-1 peers = 4(N-1)."""
    s = abd()
    s.step(200)
    st = s.stats()
    d = st.as_dict()["delivered"]
    # ops still in flight at the cut have partial counts: bound by completed ops
    assert d["Get"] >= 4 * st.commits and d["SetReply"] >= 4 * st.commits - 4 * 64 * 4
    assert st.commits == st.replies > 0


@pytest.mark.parametrize("case", ["single_worker", "single_coordinator", "read_only", "write_only"])
def test_linearizable_when_no_conflicting_writers(case):
    kw = {"single_worker": dict(outstanding=1, target=(0,)),
          "single_coordinator": dict(target=(0,)),
          "read_only": dict(write_ppm=0),
          "write_only": dict(write_ppm=1_000_000)}[case]
    s = abd(**kw)
    s.step(300)
    a, n = s.linearizable()
    assert n > 0 and a == 0


def test_concurrent_coordinators_expose_versioning():
    """Writers at different replicas can pick the same version (abd/replica.go:123,
    no writer-id tie-break): the checker sees anomalous reads."""
    s = abd(clusters=200)
    s.step(300)
    a, n = s.linearizable()
    assert n > 0 and a > 0


def test_history_is_bounded_and_flagged():
    s = abd(clusters=4, history=8)
    s.step(200)
    st = s.stats()
    assert st.flagged[7] > 0          # PAXISIM_F_HIST_OVF
    assert all(len(s.history(c)) <= 8 * 5 for c in range(4))
