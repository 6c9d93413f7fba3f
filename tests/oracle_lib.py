"""Test-side loader for the CPU oracle (oracle/liboracle_paxisim.so).

The oracle is test infrastructure: only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg load it, and only as the checker.
"""
import ctypes as C
import os

from paxi_amd import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "liboracle_paxisim.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            raise RuntimeError(f"oracle not built: run `make -C oracle` ({ORACLE_SO})")
        L = C.CDLL(ORACLE_SO)
        abi.declare(L, "oracle")
        L.oracle_command.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32, C.POINTER(C.c_uint32),
                                     C.POINTER(C.c_uint32)]
        L.oracle_step.restype = C.c_int
        L.oracle_step.argtypes = [C.c_void_p, C.c_uint32, C.c_int]
        L.oracle_exec_log.restype = C.c_int
        L.oracle_exec_log.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32, C.POINTER(C.c_uint32),
                                      C.c_uint32, C.POINTER(C.c_uint32)]
        L.oracle_lin_check.restype = C.c_int
        L.oracle_lin_check.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        L.oracle_history.restype = C.c_int
        L.oracle_history.argtypes = [C.c_void_p, C.c_uint64, C.POINTER(C.c_uint32), C.c_uint32,
                                     C.POINTER(C.c_uint32)]
        L.oracle_new_ballot.restype = C.c_uint64
        L.oracle_new_ballot.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32]
        L.oracle_ballot_next.restype = C.c_uint64
        L.oracle_ballot_next.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32]
        L.oracle_quorum.restype = C.c_int
        L.oracle_quorum.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32), C.c_uint32]
        L.oracle_linearizable.restype = C.c_int
        L.oracle_linearizable.argtypes = [C.POINTER(C.c_int64), C.c_int]
        _lib = L
    return _lib


def _check(rc):
    if rc != 0:
        raise RuntimeError(f"oracle error {rc}: {lib().oracle_last_error().decode()}")


class OracleSim:
    """Same surface as paxi_amd.sim.Simulation, backed by the CPU restatement."""

    def __init__(self, cfg, wl, fp=None, faults=()):
        self.cfg, self.wl = cfg, wl
        self.N = abi.n_replicas(cfg)
        self.h = C.c_void_p()
        _check(lib().oracle_create(C.byref(cfg), C.byref(wl), C.byref(fp) if fp else None, C.byref(self.h)))
        for f in faults:
            _check(lib().oracle_fault_add(self.h, C.byref(f)))

    def step(self, n, threads=1):
        _check(lib().oracle_step(self.h, n, threads))

    def set_replica_order(self, mode):
        """Test hook: 0 = index order, 1 = reversed, 2 = shuffled per (cluster, step)."""
        _check(lib().oracle_set_replica_order(self.h, mode))

    def stats(self):
        s = abi.Stats()
        _check(lib().oracle_stats_get(self.h, C.byref(s)))
        return s

    def read_state(self, lo=0, n=None):
        n = self.cfg.clusters - lo if n is None else n
        arr = (abi.ReplicaState * (n * self.N))()
        _check(lib().oracle_read_state(self.h, lo, n, arr))
        return arr

    def read_instances(self, lo=0, n=None):
        n = self.cfg.clusters - lo if n is None else n
        arr = (abi.InstanceState * (n * self.N * abi.n_instances(self.cfg)))()
        _check(lib().oracle_read_instances(self.h, lo, n, arr))
        return arr

    def check(self):
        v = C.c_uint64()
        _check(lib().oracle_check(self.h, C.byref(v)))
        return v.value

    def inject(self, cluster, replica, cid):
        _check(lib().oracle_inject(self.h, cluster, replica, cid))

    def commands(self, cluster, cids):
        return [self.command(cluster, c) for c in cids]

    def read_inbox(self, cluster, replica):
        from paxi_amd.sim import _read_inbox
        lib().oracle_read_inbox.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32, C.POINTER(abi.InboxRecord),
                                            C.c_uint32, C.POINTER(C.c_uint32)]
        return _read_inbox(lib().oracle_read_inbox, self.h, cluster, replica, _check)

    def deliver(self, cluster, replica, src, recs):
        arr = (abi.InboxRecord * max(1, len(recs)))(*[abi.InboxRecord(src, *r[-4:]) for r in recs])
        _check(lib().oracle_deliver(self.h, cluster, replica, src, arr, len(recs)))

    def read_log(self, cluster, replica, slot_lo, n, key=0):
        arr = (abi.LogEntry * max(1, n))()
        _check(lib().oracle_read_log(self.h, cluster, replica, key, slot_lo, n, arr))
        return list(arr[:n])

    def exec_log(self, cluster, replica, key=0):
        rk = replica | (key << 16)
        n = C.c_uint32()
        _check(lib().oracle_exec_log(self.h, cluster, rk, None, 0, C.byref(n)))
        buf = (C.c_uint32 * max(1, n.value))()
        _check(lib().oracle_exec_log(self.h, cluster, rk, buf, n.value, C.byref(n)))
        return list(buf[: n.value])

    def linearizable(self):
        a, n = C.c_uint64(), C.c_uint64()
        _check(lib().oracle_lin_check(self.h, C.byref(a), C.byref(n)))
        return a.value, n.value

    def history(self, cluster):
        n = C.c_uint32()
        _check(lib().oracle_history(self.h, cluster, None, 0, C.byref(n)))
        buf = (C.c_uint32 * max(1, 5 * n.value))()
        _check(lib().oracle_history(self.h, cluster, buf, n.value, C.byref(n)))
        return [tuple(buf[5 * i: 5 * i + 5]) for i in range(n.value)]

    def read_client(self, cluster):
        from paxi_amd.sim import _read_client
        lib().oracle_read_client.argtypes = [C.c_void_p, C.c_uint64, C.POINTER(abi.WorkerState), C.c_uint32,
                                             C.POINTER(C.c_uint32)]
        return _read_client(lib().oracle_read_client, self.h, cluster, self.wl.outstanding, _check)

    def read_kv(self, cluster, replica, n):
        buf = (C.c_uint32 * max(1, n))()
        _check(lib().oracle_read_kv(self.h, cluster, replica, buf, n))
        return list(buf[:n])

    def command(self, cluster, cid):
        """(key, is_write) of command `cid` of a cluster, as the workers draw it."""
        k, w = C.c_uint32(), C.c_uint32()
        _check(lib().oracle_command(self.h, cluster, cid, C.byref(k), C.byref(w)))
        return k.value, bool(w.value)

    def history_load(self, cluster, replica, ops):
        flat = [int(v) for o in ops for v in o]
        buf = (C.c_uint32 * max(1, len(flat)))(*flat)
        _check(lib().oracle_history_load(self.h, cluster, replica, buf, len(ops)))

    def close(self):
        if self.h:
            lib().oracle_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def new_ballot(n, zone, node):
    return lib().oracle_new_ballot(n, zone, node)


def ballot_next(b, zone, node):
    return lib().oracle_ballot_next(b, zone, node)


def quorum(kind, npz, mask, fz=0):
    arr = (C.c_uint32 * len(npz))(*npz)
    return bool(lib().oracle_quorum(kind, fz, len(npz), arr, mask))


def linearizable(ops):
    """ops: list of (input, output, start, end) with None for nil (operation.go)."""
    flat = []
    for i, o, s, e in ops:
        flat += [0 if i is None else 1, 0 if i is None else i, 0 if o is None else 1, 0 if o is None else o, s, e]
    arr = (C.c_int64 * len(flat))(*flat)
    n = lib().oracle_linearizable(arr, len(ops))
    if n < 0:
        raise RuntimeError("linearizable failed")
    return n
