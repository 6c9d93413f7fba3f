"""ctypes mirror of include/paxisim.h (the C-ABI boundary).

Only type and constant definitions live here; no library is loaded.  The HIP
product binding (paxi_amd.sim) and the test-side oracle loader both use these
structs, so the two speak exactly the same ABI.
"""
import ctypes as C

ABI_VERSION = 13
MAX_N = 16
MAX_ZONES = 16
MAX_WORKERS = 32
MAX_KEYS = 64
MAX_FAULTS = 64
MAX_WINDOW = 64
MAX_MBOX = 64
MAX_DELAY = 14
CLIENT_SRC = 31
ALL_DST = 0xFF

# error codes
OK, EINVAL, ENOMEM, EDEVICE, EUNSUPP, ERANGE = 0, -1, -2, -3, -4, -5

# protocols (server/server.go:38-84)
PAXOS, ABD, WPAXOS, M2PAXOS, KPAXOS, EPAXOS = 0, 1, 2, 3, 4, 5
PER_KEY = (WPAXOS, M2PAXOS, KPAXOS)   # protocols with one Paxos instance per key

# quorum predicates (quorum.go)
Q_MAJORITY, Q_ALL, Q_FAST, Q_GRID_ROW, Q_ZONE_MAJORITY, Q_GRID_COLUMN, Q_FGRID_Q1, Q_FGRID_Q2 = range(8)

# message types
(MSG_NONE, MSG_REQUEST, MSG_REPLY, MSG_P1A, MSG_P1B, MSG_P1B_ENTRY, MSG_P2A, MSG_P2B,
 MSG_P3, MSG_GET, MSG_GETREPLY, MSG_SET, MSG_SETREPLY, MSG_LEADERCHG, MSG_PREACCEPT, MSG_PREACCEPTREPLY,
 MSG_ACCEPT, MSG_ACCEPTREPLY, MSG_COMMIT) = range(19)
NMSG = 20
MSG_NAMES = {MSG_REQUEST: "Request", MSG_REPLY: "Reply", MSG_P1A: "P1a", MSG_P1B: "P1b",
             MSG_P2A: "P2a", MSG_P2B: "P2b", MSG_P3: "P3", MSG_GET: "Get",
             MSG_GETREPLY: "GetReply", MSG_SET: "Set", MSG_SETREPLY: "SetReply",
             MSG_LEADERCHG: "LeaderChange", MSG_PREACCEPT: "PreAccept", MSG_PREACCEPTREPLY: "PreAcceptReply",
             MSG_ACCEPT: "Accept", MSG_ACCEPTREPLY: "AcceptReply", MSG_COMMIT: "Commit"}

# flags
F_WOVF, F_GHOST, F_MBOX_OVF, F_PEND_OVF, F_UNFAITHFUL, F_POISON, F_BALLOT_OVF, F_HIST_OVF = (
    0x01, 0x02, 0x04, 0x08, 0x10, 0x20, 0x40, 0x80)

# WPaxos leader-migration policies (policy.go)
POLICY_CONSECUTIVE, POLICY_MAJORITY, POLICY_EMA = 0, 1, 2

# workload key distributions (benchmark.go:202-233)
DIST_UNIFORM, DIST_ORDER, DIST_CONFLICT, DIST_TABLE = 0, 1, 2, 3

# scripted faults (socket.go:163-199)
FAULT_DROP, FAULT_SLOW, FAULT_FLAKY, FAULT_CRASH = 0, 1, 2, 3


class Config(C.Structure):
    _fields_ = [
        ("protocol", C.c_uint32),
        ("n_zones", C.c_uint32),
        ("npz", C.c_uint32 * MAX_ZONES),
        ("q1", C.c_uint32), ("q2", C.c_uint32),
        ("fz", C.c_uint32),
        ("thrifty", C.c_uint32),
        ("ephemeral_leader", C.c_uint32),
        ("reply_when_commit", C.c_uint32),
        ("adaptive", C.c_uint32),
        ("policy_threshold", C.c_uint32),
        ("window", C.c_uint32),
        ("mbox_cap", C.c_uint32),
        ("max_delay", C.c_uint32),
        ("keys", C.c_uint32),
        ("steps_per_launch", C.c_uint32),
        ("history", C.c_uint32),
        ("device", C.c_int32),
        ("clusters", C.c_uint64),
        ("cluster_base", C.c_uint64),
        ("seed", C.c_uint64),
        ("policy", C.c_uint32),
        ("policy_interval", C.c_uint32),
        ("policy_alpha", C.c_double),
        ("agree_ring", C.c_uint32), ("kv", C.c_uint32),
    ]


class Workload(C.Structure):
    _fields_ = [
        ("outstanding", C.c_uint32),
        ("max_requests", C.c_uint32),
        ("write_ppm", C.c_uint32),
        ("locality_ppm", C.c_uint32),
        ("target", C.c_uint32 * MAX_WORKERS),
        ("distribution", C.c_uint32),
        ("conflicts", C.c_uint32),
        ("key_cdf", C.c_uint32 * MAX_KEYS),
        ("start_step", C.c_uint32 * MAX_WORKERS),
        ("key_min", C.c_uint32),
        ("key_space", C.c_uint32),
        ("key_tail", C.c_uint32),
        ("move_every", C.c_uint32),
        ("move_tables", C.c_uint32),
        ("move_loop", C.c_uint32),
        ("move_cdf", C.POINTER(C.c_uint32)),
    ]


class FaultProcess(C.Structure):
    _fields_ = [
        ("drop_ppm", C.c_uint32), ("drop_len", C.c_uint32),
        ("slow_ppm", C.c_uint32), ("slow_len", C.c_uint32),
        ("slow_min", C.c_uint32), ("slow_max", C.c_uint32),
    ]


class Fault(C.Structure):
    _fields_ = [
        ("kind", C.c_uint32), ("src", C.c_uint32), ("dst", C.c_uint32), ("param", C.c_uint32),
        ("cluster_lo", C.c_uint64), ("cluster_hi", C.c_uint64),
        ("step_from", C.c_uint32), ("step_to", C.c_uint32),
    ]


class ReplicaState(C.Structure):
    _fields_ = [
        ("ballot", C.c_uint64),
        ("slot", C.c_int32), ("execute", C.c_int32),
        ("active", C.c_uint32), ("flags", C.c_uint32),
        ("digest", C.c_uint64),
        ("p1_acks", C.c_uint32), ("npending", C.c_uint32),
        ("delivered", C.c_uint32 * NMSG),
        ("client_requests", C.c_uint32), ("sent", C.c_uint32),
        ("dropped", C.c_uint32), ("discarded", C.c_uint32),
        ("commits", C.c_uint32), ("replies", C.c_uint32),
        ("executed_writes", C.c_uint32), ("executions", C.c_uint32),
    ]

    def as_tuple(self):
        return (self.ballot, self.slot, self.execute, self.active, self.flags, self.digest,
                self.p1_acks, self.npending, tuple(self.delivered), self.client_requests,
                self.sent, self.dropped, self.discarded, self.commits, self.replies,
                self.executed_writes, self.executions)


class InstanceState(C.Structure):
    """One Paxos instance: a Multi-Paxos replica's paxos.Paxos, or a WPaxos kpaxos per key."""
    _fields_ = [
        ("ballot", C.c_uint64),
        ("slot", C.c_int32), ("execute", C.c_int32),
        ("active", C.c_uint32), ("exists", C.c_uint32),
        ("p1_acks", C.c_uint32), ("npending", C.c_uint32),
        ("digest", C.c_uint64),
        ("policy_last", C.c_uint32), ("policy_hits", C.c_uint32),
        ("policy_state", C.c_uint32 * 4),
    ]

    def as_tuple(self):
        return (self.ballot, self.slot, self.execute, self.active, self.exists, self.p1_acks,
                self.npending, self.digest, self.policy_last, self.policy_hits, tuple(self.policy_state))


LOG_EXISTS, LOG_COMMIT, LOG_QUORUM, LOG_REQUEST, LOG_HELD = 0x1, 0x2, 0x4, 0x8, 0x10


class LogEntry(C.Structure):
    """One paxos/paxos.go:11-18 entry of a replica's window (read_log)."""
    _fields_ = [
        ("ballot", C.c_uint64), ("slot", C.c_int32), ("cmd", C.c_uint32), ("flags", C.c_uint32),
        ("acks", C.c_uint32), ("request", C.c_uint32), ("pad", C.c_uint32),
    ]

    def as_tuple(self):
        return (self.ballot, self.slot, self.cmd, self.flags, self.acks, self.request)


class InboxRecord(C.Structure):
    """One record of a replica's next-step inbox (paxisim_read_inbox / paxisim_deliver)."""
    _fields_ = [("src", C.c_uint32), ("hdr", C.c_uint32), ("ballot", C.c_uint32), ("slot", C.c_uint32),
                ("cid", C.c_uint32)]

    def as_tuple(self):
        return (self.src, self.hdr, self.ballot, self.slot, self.cid)


class WorkerState(C.Structure):
    """paxisim_worker_state: a closed-loop worker (benchmark.go:246-275) and its last Reply.Value."""
    _fields_ = [("cid", C.c_uint32), ("issued", C.c_uint32), ("reply_value", C.c_uint32), ("pad", C.c_uint32)]

    def as_tuple(self):
        return (self.cid, self.issued, self.reply_value)


class Stats(C.Structure):
    _fields_ = [
        ("steps", C.c_uint64), ("clusters", C.c_uint64),
        ("delivered", C.c_uint64 * NMSG),
        ("delivered_total", C.c_uint64),
        ("client_requests", C.c_uint64),
        ("sent", C.c_uint64), ("dropped", C.c_uint64), ("discarded", C.c_uint64),
        ("commits", C.c_uint64), ("replies", C.c_uint64),
        ("flagged", C.c_uint64 * 8),
        ("agree_compared", C.c_uint64), ("agree_missed", C.c_uint64), ("agree_mismatch", C.c_uint64),
    ]

    def as_dict(self):
        d = {k: getattr(self, k) for k in ("steps", "clusters", "delivered_total", "client_requests",
                                            "sent", "dropped", "discarded", "commits", "replies",
                                            "agree_compared", "agree_missed", "agree_mismatch")}
        d["delivered"] = {MSG_NAMES.get(i, str(i)): self.delivered[i] for i in range(NMSG) if self.delivered[i]}
        d["flagged"] = list(self.flagged)
        return d


# C prototypes shared by the product library (prefix "paxisim") and the oracle ("oracle").
def declare(lib, prefix):
    P = C.POINTER
    h = C.c_void_p
    spec = {
        "create": (C.c_int, [P(Config), P(Workload), P(FaultProcess), P(h)]),
        "destroy": (C.c_int, [h]),
        "fault_add": (C.c_int, [h, P(Fault)]),
        "stats_get": (C.c_int, [h, P(Stats)]),
        "read_state": (C.c_int, [h, C.c_uint64, C.c_uint64, P(ReplicaState)]),
        "read_instances": (C.c_int, [h, C.c_uint64, C.c_uint64, P(InstanceState)]),
        "check": (C.c_int, [h, P(C.c_uint64)]),
        "inject": (C.c_int, [h, C.c_uint64, C.c_uint32, C.c_uint32]),
        "read_log": (C.c_int, [h, C.c_uint64, C.c_uint32, C.c_uint32, C.c_int32, C.c_uint32, P(LogEntry)]),
        "history_load": (C.c_int, [h, C.c_uint64, C.c_uint32, P(C.c_uint32), C.c_uint32]),
        "read_kv": (C.c_int, [h, C.c_uint64, C.c_uint32, P(C.c_uint32), C.c_uint32]),
        "read_inbox": (C.c_int, [h, C.c_uint64, C.c_uint32, P(InboxRecord), C.c_uint32, P(C.c_uint32)]),
        "deliver": (C.c_int, [h, C.c_uint64, C.c_uint32, C.c_uint32, P(InboxRecord), C.c_uint32]),
        "last_error": (C.c_char_p, []),
    }
    for name, (res, args) in spec.items():
        fn = getattr(lib, f"{prefix}_{name}")
        fn.restype = res
        fn.argtypes = args
    return lib


def make_config(npz=(5,), protocol=PAXOS, q1=Q_MAJORITY, q2=Q_MAJORITY, fz=0, thrifty=0,
                ephemeral_leader=0, reply_when_commit=0, adaptive=1, policy_threshold=3,
                window=16, mbox_cap=16, max_delay=4, keys=16, steps_per_launch=0, device=0,
                clusters=1, cluster_base=0, seed=1, history=0, policy=POLICY_CONSECUTIVE, policy_interval=1,
                policy_alpha=0.5, agree_ring=0, kv=0):
    c = Config()
    c.protocol = protocol
    c.n_zones = len(npz)
    for i, v in enumerate(npz):
        c.npz[i] = v
    c.q1, c.q2, c.fz = q1, q2, fz
    c.thrifty, c.ephemeral_leader, c.reply_when_commit = thrifty, ephemeral_leader, reply_when_commit
    c.adaptive, c.policy_threshold = adaptive, policy_threshold
    c.window, c.mbox_cap, c.max_delay, c.keys = window, mbox_cap, max_delay, keys
    c.steps_per_launch, c.device, c.history = steps_per_launch, device, history
    c.clusters, c.cluster_base, c.seed = clusters, cluster_base, seed
    c.policy, c.policy_interval, c.policy_alpha = policy, policy_interval, policy_alpha
    c.agree_ring = agree_ring
    c.kv = kv
    return c


def make_workload(outstanding=1, max_requests=0, write_ppm=1_000_000, locality_ppm=0, target=0,
                  distribution="uniform", keys=None, start_step=0, key_min=0, **dist_params):
    """Closed-loop workload.  `distribution` is a Bconfig.Distribution name
    (benchmark.go:202-233, see paxi_amd.workload); the table distributions
    ("normal", "zipfan", "exponential") need the cluster's `keys`.  Other
    options: key_space (Bconfig.K of order/uniform/conflict), move_every
    (Bconfig.Move for normal), and the distribution's parameters."""
    from . import workload as _wl
    w = Workload()
    w.outstanding, w.max_requests, w.write_ppm, w.locality_ppm = outstanding, max_requests, write_ppm, locality_ppm
    w.key_min = key_min
    for i in range(MAX_WORKERS):
        w.target[i] = target[i % len(target)] if isinstance(target, (list, tuple)) else target
        w.start_step[i] = start_step[i % len(start_step)] if isinstance(start_step, (list, tuple)) else start_step
    _wl.set_distribution(w, distribution, keys, **dist_params)
    return w


def make_fault_process(drop_ppm=0, drop_len=0, slow_ppm=0, slow_len=0, slow_min=0, slow_max=0):
    f = FaultProcess()
    f.drop_ppm, f.drop_len, f.slow_ppm, f.slow_len, f.slow_min, f.slow_max = (
        drop_ppm, drop_len, slow_ppm, slow_len, slow_min, slow_max)
    return f


def make_fault(kind, src, dst=ALL_DST, param=0, cluster_lo=0, cluster_hi=2**63, step_from=0,
               step_to=0xFFFFFFFF):
    f = Fault()
    f.kind, f.src, f.dst, f.param = kind, src, dst, param
    f.cluster_lo, f.cluster_hi, f.step_from, f.step_to = cluster_lo, cluster_hi, step_from, step_to
    return f


def n_replicas(cfg):
    return sum(cfg.npz[i] for i in range(cfg.n_zones))


def n_instances(cfg):
    """read_instances records per replica: one kpaxos per key (WPaxos, M2Paxos,
    KPaxos), one per owner log (EPaxos), else one."""
    if cfg.protocol == EPAXOS:
        return n_replicas(cfg)
    return cfg.keys if cfg.protocol in PER_KEY else 1
