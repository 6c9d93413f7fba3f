"""Host-side mirror of the reference's simulation entry point over the HIP C-ABI.

`Simulation` plays the role of `server -sim` (server/server.go:87-101) for a
whole batch of clusters: it takes a paxi.Config-like description (zones and
nodes per zone, quorum options, config.go:14-35), a benchmark workload
(benchmark.go:21-48) and fault injection (socket.go:163-199), and advances all
clusters on one GPU through libpaxisim.so.  There is no CPU fallback: if the
HIP library or the device is missing, construction raises.
"""
import ctypes as C
import os

from . import abi

_HERE = os.path.dirname(os.path.abspath(__file__))
# PAXISIM_LIB selects another build of the same HIP library (tuning variants)
LIB_PATH = os.environ.get("PAXISIM_LIB") or os.path.join(_HERE, "libpaxisim.so")
_lib = None


class PaxisimError(RuntimeError):
    pass


def quorum(cfg, kind, ack_mask):
    """paxisim_quorum: the kernels' quorum predicate (quorum.go:55-119) for cfg's zones; host only."""
    ok = C.c_int()
    _check(load_library().paxisim_quorum(C.byref(cfg), kind, ack_mask, C.byref(ok)))
    return bool(ok.value)


def load_library():
    """Load the in-tree HIP library; raise if it is absent (no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise PaxisimError(f"HIP library not built: {LIB_PATH} (run `python -c 'import __graft_entry__ as g; g.build()'`)")
    L = C.CDLL(LIB_PATH)
    abi.declare(L, "paxisim")
    L.paxisim_abi_version.restype = C.c_int
    L.paxisim_build_id.restype = C.c_char_p
    L.paxisim_build_id.argtypes = []
    L.paxisim_step.restype = C.c_int
    L.paxisim_step.argtypes = [C.c_void_p, C.c_uint32]
    L.paxisim_sync.restype = C.c_int
    L.paxisim_sync.argtypes = [C.c_void_p]
    L.paxisim_kernel_time.restype = C.c_int
    L.paxisim_kernel_time.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_uint64), C.c_int]
    L.paxisim_linearizable.restype = C.c_int
    L.paxisim_linearizable.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                       C.POINTER(C.c_uint64)]
    L.paxisim_history.restype = C.c_int
    L.paxisim_history.argtypes = [C.c_void_p, C.c_uint64, C.POINTER(C.c_uint32), C.c_uint32,
                                  C.POINTER(C.c_uint32)]
    L.paxisim_occupancy.restype = C.c_int
    L.paxisim_occupancy.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
    L.paxisim_active_clusters.restype = C.c_int
    L.paxisim_active_clusters.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
    L.paxisim_quorum.restype = C.c_int
    L.paxisim_quorum.argtypes = [C.POINTER(abi.Config), C.c_uint32, C.c_uint32, C.POINTER(C.c_int)]
    L.paxisim_read_client.restype = C.c_int
    L.paxisim_read_client.argtypes = [C.c_void_p, C.c_uint64, C.POINTER(abi.WorkerState), C.c_uint32,
                                      C.POINTER(C.c_uint32)]
    L.paxisim_read_activity.restype = C.c_int
    L.paxisim_read_activity.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.POINTER(C.c_uint32)]
    L.paxisim_device_bytes.restype = C.c_int
    L.paxisim_device_bytes.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
    P = C.POINTER
    L.paxisim_dist_init.restype = C.c_int
    L.paxisim_dist_init.argtypes = [P(C.c_void_p), C.c_int, P(C.c_void_p)]
    L.paxisim_dist_unique_id.restype = C.c_int
    L.paxisim_dist_unique_id.argtypes = [C.c_char_p]
    L.paxisim_dist_init_rank.restype = C.c_int
    L.paxisim_dist_init_rank.argtypes = [C.c_void_p, C.c_char_p, C.c_int, C.c_int, P(C.c_void_p)]
    L.paxisim_dist_allreduce.restype = C.c_int
    L.paxisim_dist_allreduce.argtypes = [C.c_void_p, P(C.c_uint64), C.c_uint32, P(C.c_double), C.c_uint32,
                                         P(C.c_uint64), P(C.c_double)]
    L.paxisim_dist_stats.restype = C.c_int
    L.paxisim_dist_stats.argtypes = [C.c_void_p, P(abi.Stats), P(C.c_double)]
    L.paxisim_dist_destroy.restype = C.c_int
    L.paxisim_dist_destroy.argtypes = [C.c_void_p]
    L.paxisim_commands.restype = C.c_int
    L.paxisim_commands.argtypes = [C.c_void_p, C.c_uint64, P(C.c_uint32), C.c_uint32, P(C.c_uint32), P(C.c_uint32)]
    if L.paxisim_abi_version() != abi.ABI_VERSION:
        raise PaxisimError("ABI version mismatch between paxi_amd/abi.py and libpaxisim.so")
    _lib = L
    return L


def build_id():
    """The source fingerprint compiled into the loaded library (paxisim_build_id)."""
    return load_library().paxisim_build_id().decode()


EXPORTED = ["paxisim_abi_version", "paxisim_build_id", "paxisim_last_error", "paxisim_create", "paxisim_destroy",
            "paxisim_fault_add", "paxisim_step", "paxisim_sync", "paxisim_stats_get",
            "paxisim_read_state", "paxisim_read_instances", "paxisim_check", "paxisim_kernel_time", "paxisim_device_bytes",
            "paxisim_linearizable", "paxisim_history", "paxisim_occupancy", "paxisim_inject", "paxisim_read_log",
            "paxisim_history_load", "paxisim_active_clusters", "paxisim_read_activity", "paxisim_read_client", "paxisim_quorum", "paxisim_dist_init", "paxisim_dist_unique_id",
            "paxisim_dist_init_rank", "paxisim_dist_allreduce", "paxisim_dist_stats", "paxisim_dist_destroy",
            "paxisim_read_kv", "paxisim_read_inbox", "paxisim_deliver", "paxisim_commands"]


def _check(rc):
    if rc != 0:
        raise PaxisimError(f"paxisim error {rc}: {load_library().paxisim_last_error().decode()}")


def _read_inbox(fn, h, cluster, replica, check):
    n = C.c_uint32()
    cap = 256
    while True:
        arr = (abi.InboxRecord * cap)()
        check(fn(h, cluster, replica, arr, cap, C.byref(n)))
        if n.value <= cap:
            return [arr[i].as_tuple() for i in range(n.value)]
        cap = n.value


def _read_client(fn, h, cluster, n, check):
    arr = (abi.WorkerState * max(1, n))()
    got = C.c_uint32()
    check(fn(h, cluster, arr, n, C.byref(got)))
    return [arr[i].as_tuple() for i in range(min(n, got.value))]


class Simulation:
    """A batch of independent N-replica clusters on one GPU (one handle)."""

    def __init__(self, cfg, wl, fp=None, faults=()):
        L = load_library()
        self.cfg, self.wl, self.fp = cfg, wl, fp
        self.N = abi.n_replicas(cfg)
        self.h = C.c_void_p()
        _check(L.paxisim_create(C.byref(cfg), C.byref(wl), C.byref(fp) if fp else None, C.byref(self.h)))
        for f in faults:
            self.fault(f)

    # socket.go Drop/Slow/Flaky/Crash, scripted
    def fault(self, f):
        _check(load_library().paxisim_fault_add(self.h, C.byref(f)))

    def step(self, n):
        _check(load_library().paxisim_step(self.h, n))

    def sync(self):
        _check(load_library().paxisim_sync(self.h))

    def stats(self):
        s = abi.Stats()
        _check(load_library().paxisim_stats_get(self.h, C.byref(s)))
        return s

    def read_state(self, lo=0, n=None):
        n = self.cfg.clusters - lo if n is None else n
        arr = (abi.ReplicaState * (n * self.N))()
        _check(load_library().paxisim_read_state(self.h, lo, n, arr))
        return arr

    def read_instances(self, lo=0, n=None):
        """Per (cluster, replica, key) Paxos instance state (paxisim_read_instances)."""
        n = self.cfg.clusters - lo if n is None else n
        arr = (abi.InstanceState * (n * self.N * abi.n_instances(self.cfg)))()
        _check(load_library().paxisim_read_instances(self.h, lo, n, arr))
        return arr

    def check(self):
        v = C.c_uint64()
        _check(load_library().paxisim_check(self.h, C.byref(v)))
        return v.value

    def inject(self, cluster, replica, cid):
        """A client request for command `cid` at `replica` in the next step (http.go:99)."""
        _check(load_library().paxisim_inject(self.h, cluster, replica, cid))

    def read_inbox(self, cluster, replica):
        """Records replica `replica` receives at the next step, by source (paxisim_read_inbox)."""
        return _read_inbox(load_library().paxisim_read_inbox, self.h, cluster, replica, _check)

    def commands(self, cluster, cids):
        """[(key index, is_write)] of command ids of a cluster (paxisim_commands)."""
        n = len(cids)
        a = (C.c_uint32 * max(1, n))(*cids)
        k, w = (C.c_uint32 * max(1, n))(), (C.c_uint32 * max(1, n))()
        _check(load_library().paxisim_commands(self.h, cluster, a, n, k, w))
        return [(k[i], bool(w[i])) for i in range(n)]

    def deliver(self, cluster, replica, src, recs):
        """Append records (src, hdr, ballot, slot, cid) to the replica's next-step
        inbox from source `src` (paxisim_deliver; a record's own src is ignored)."""
        arr = (abi.InboxRecord * max(1, len(recs)))(*[abi.InboxRecord(src, *r[-4:]) for r in recs])
        _check(load_library().paxisim_deliver(self.h, cluster, replica, src, arr, len(recs)))

    def read_log(self, cluster, replica, slot_lo, n, key=0):
        """paxos.go entries of slots [slot_lo, slot_lo+n) of one instance (paxisim_read_log)."""
        arr = (abi.LogEntry * max(1, n))()
        _check(load_library().paxisim_read_log(self.h, cluster, replica, key, slot_lo, n, arr))
        return list(arr[:n])

    def linearizable(self):
        """History.Linearizable (history.go:55-71): (anomalies, ops checked, partitions skipped)."""
        a, n, sk = C.c_uint64(), C.c_uint64(), C.c_uint64()
        _check(load_library().paxisim_linearizable(self.h, C.byref(a), C.byref(n), C.byref(sk)))
        return a.value, n.value, sk.value

    def history(self, cluster):
        n = C.c_uint32()
        _check(load_library().paxisim_history(self.h, cluster, None, 0, C.byref(n)))
        buf = (C.c_uint32 * max(1, 5 * n.value))()
        _check(load_library().paxisim_history(self.h, cluster, buf, n.value, C.byref(n)))
        return [tuple(buf[5 * i: 5 * i + 5]) for i in range(n.value)]

    def read_client(self, cluster):
        """[(cid, issued, reply_value)] of the cluster's closed-loop workers (paxisim_read_client)."""
        return _read_client(load_library().paxisim_read_client, self.h, cluster, self.wl.outstanding, _check)

    def read_kv(self, cluster, replica, n):
        """Database.Get (db.go:116-121) of keys [0, n) of one replica (paxisim_read_kv)."""
        buf = (C.c_uint32 * max(1, n))()
        _check(load_library().paxisim_read_kv(self.h, cluster, replica, buf, n))
        return list(buf[:n])

    def history_load(self, cluster, replica, ops):
        """History.ReadFile into the device (paxisim_history_load): ops are
        (key, is_write, value, start, end) tuples."""
        flat = [int(v) for o in ops for v in o]
        buf = (C.c_uint32 * max(1, len(flat)))(*flat)
        _check(load_library().paxisim_history_load(self.h, cluster, replica, buf, len(ops)))

    def kernel_time(self, reset=False):
        ms, n = C.c_double(), C.c_uint64()
        _check(load_library().paxisim_kernel_time(self.h, C.byref(ms), C.byref(n), int(reset)))
        return ms.value, n.value

    def occupancy(self):
        """(workgroups resident per CU, dynamic LDS bytes per workgroup, messages staged per replica-step)"""
        b, lds, j = C.c_int(), C.c_uint32(), C.c_uint32()
        _check(load_library().paxisim_occupancy(self.h, C.byref(b), C.byref(lds), C.byref(j)))
        return b.value, lds.value, j.value

    def active_clusters(self):
        """Clusters the step kernels still visit (the rest are frozen at a fixed point)."""
        b = C.c_uint64()
        _check(load_library().paxisim_active_clusters(self.h, C.byref(b)))
        return b.value

    def activity(self, lo=0, n=None):
        """Per cluster: None while the step kernels visit it, else the step at
        which it froze at its fixed point (paxisim_read_activity)."""
        n = self.cfg.clusters - lo if n is None else n
        buf = (C.c_uint32 * max(1, n))()
        _check(load_library().paxisim_read_activity(self.h, lo, n, buf))
        return [None if buf[i] == 0xFFFFFFFF else buf[i] for i in range(n)]

    def device_bytes(self):
        b = C.c_uint64()
        _check(load_library().paxisim_device_bytes(self.h, C.byref(b)))
        return b.value

    def close(self):
        if self.h:
            load_library().paxisim_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Dist:
    """RCCL reduction of statistics over handles (paxisim_dist_*): either one
    process driving several handles (`Dist(sims)`) or one handle per process
    (`Dist.join(sim, uid, nranks, rank)` with `uid` from `Dist.unique_id()` on
    one rank, shipped by the caller's launcher)."""

    def __init__(self, sims=None, _h=None, _members=1):
        L = load_library()
        self.h = C.c_void_p()
        if _h is not None:
            self.h, self.members = _h, _members
            return
        arr = (C.c_void_p * len(sims))(*[s.h.value for s in sims])
        _check(L.paxisim_dist_init(arr, len(sims), C.byref(self.h)))
        self.members = len(sims)

    @staticmethod
    def unique_id():
        buf = C.create_string_buffer(128)
        _check(load_library().paxisim_dist_unique_id(buf))
        return buf.raw

    @classmethod
    def join(cls, sim, uid, nranks, rank):
        h = C.c_void_p()
        _check(load_library().paxisim_dist_init_rank(sim.h, uid, nranks, rank, C.byref(h)))
        return cls(_h=h, _members=1)

    def allreduce(self, sums, maxes):
        """Sum `sums` (per member: a list of ints) and max `maxes` (per member: floats)."""
        n, m = len(sums[0]) if sums else 0, len(maxes[0]) if maxes else 0
        si = (C.c_uint64 * max(1, n * self.members))(*[int(v) for row in sums for v in row])
        mi = (C.c_double * max(1, m * self.members))(*[float(v) for row in maxes for v in row])
        so, mo = (C.c_uint64 * max(1, n))(), (C.c_double * max(1, m))()
        _check(load_library().paxisim_dist_allreduce(self.h, si, n, mi, m, so, mo))
        return list(so[:n]), list(mo[:m])

    def stats(self):
        """(paxisim_stats summed over the job, max step-kernel ms of any handle)"""
        s, ms = abi.Stats(), C.c_double()
        _check(load_library().paxisim_dist_stats(self.h, C.byref(s), C.byref(ms)))
        return s, ms.value

    def close(self):
        if self.h:
            load_library().paxisim_dist_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
