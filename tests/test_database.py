"""The replicas' Database (db.go:53-134) under config.kv: Execute writes a
write's value (its command id) to its key and counts database.version; a
read writes nothing (put skips nil values, db.go:123-126).  Every replica
that executed the same log prefix holds the same Database."""
import pytest

from paxi_amd import abi
import oracle_lib as ol


def kv_cfg(proto=abi.PAXOS, npz=(3,), clusters=4, keys=4, **kw):
    return abi.make_config(protocol=proto, npz=list(npz), clusters=clusters, keys=keys, seed=5, kv=1, **kw)


def expected_db(o, cluster, log, keys):
    """Database after Execute of `log` in order (db.go:98-106, put 123-133)."""
    db, version = [0] * keys, 0
    for cid in log:
        k, w = o.command(cluster, cid)
        if w:
            db[k], version = cid, version + 1
    return db, version


@pytest.mark.parametrize("proto,npz", [(abi.PAXOS, (3,)), (abi.WPAXOS, (2, 2)), (abi.KPAXOS, (3,)),
                                       (abi.EPAXOS, (3,))])
def test_database_is_log_replayed(proto, npz):
    """Config-1 shape (sequential writes through one replica, 4 keys) and a
    mixed workload with faults: every replica's Database is its execution log
    replayed (per key for the per-key protocols, execution order for EPaxos)."""
    N, K = sum(npz), 4
    fp = abi.make_fault_process(drop_ppm=2000, drop_len=5, slow_ppm=5000, slow_len=10, slow_min=1, slow_max=2)
    for wl, f, steps in ((abi.make_workload(outstanding=1, max_requests=300, target=0), None, 3000),
                         (abi.make_workload(outstanding=N, target=list(range(N)), write_ppm=500_000,
                                            max_requests=40), fp, 1500)):
        o = ol.OracleSim(kv_cfg(proto, npz, clusters=3, max_delay=3, keys=K), wl, f)
        o.step(steps)
        s = o.read_state()
        for c in range(3):
            for r in range(N):
                if proto in abi.PER_KEY:
                    db, version = [0] * K, 0
                    for k in range(K):
                        d, v = expected_db(o, c, o.exec_log(c, r, k), K)
                        db[k], version = d[k], version + v
                else:
                    db, version = expected_db(o, c, o.exec_log(c, r), K)
                assert (o.read_kv(c, r, K), s[c * N + r].executed_writes) == (db, version)
        assert sum(r.executed_writes for r in s) > 0


def test_reads_do_not_write():
    o = ol.OracleSim(kv_cfg(clusters=2, max_delay=0),
                     abi.make_workload(outstanding=2, max_requests=50, target=0, write_ppm=300_000))
    o.step(400)
    s = o.read_state()
    assert all(0 < r.executed_writes < r.executions == 100 for r in s)


def test_kv_off_is_refused():
    o = ol.OracleSim(abi.make_config(npz=[3], clusters=1), abi.make_workload())
    with pytest.raises(RuntimeError, match="Database"):
        o.read_kv(0, 0, 1)


@pytest.mark.gpu
@pytest.mark.parametrize("proto,npz", [(abi.PAXOS, (5,)), (abi.WPAXOS, (3, 3, 3)), (abi.EPAXOS, (5,)),
                                       (abi.KPAXOS, (3,))])
def test_database_parity_gpu(proto, npz):
    from paxi_amd.sim import Simulation
    N = sum(npz)
    cfg = kv_cfg(proto, npz, clusters=100, keys=8, mbox_cap=32, window=32 if proto == abi.EPAXOS else 16)
    wl = abi.make_workload(outstanding=N, target=list(range(N)), write_ppm=600_000)
    fp = abi.make_fault_process(drop_ppm=1000, drop_len=10, slow_ppm=2000, slow_len=10, slow_min=1, slow_max=3)
    g, o = Simulation(cfg, wl, fp), ol.OracleSim(cfg, wl, fp)
    g.step(150)
    o.step(150)
    assert [r.as_tuple() for r in g.read_state()] == [r.as_tuple() for r in o.read_state()]
    for c in range(0, 100, 9):
        for r in range(N):
            assert g.read_kv(c, r, 8) == o.read_kv(c, r, 8)
