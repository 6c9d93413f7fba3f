/*
 * paxisim.h — C-ABI of the MI355X batched Paxi simulator (drop-in boundary).
 *
 * What this boundary replaces in the reference (acharapko/paxi, Go):
 *   - `server -sim` (server/server.go:87-101): one goroutine per replica over
 *     the `chan` transport (transport.go:238-278) and the reflection
 *     dispatcher (node.go:79-115).  Here: millions of independent clusters,
 *     one lane per (cluster, replica), device mailboxes instead of channels.
 *   - paxi.Config (config.go:14-35, Load 97-114: n, z, npz)   -> paxisim_config
 *   - Socket fault injection Drop/Slow/Flaky/Crash (socket.go:163-199) and the
 *     filter order crash->drop->flaky->slow in Send (socket.go:66-109)
 *                                                             -> paxisim_fault
 *   - Benchmark closed-loop workers (benchmark.go:246-275)   -> paxisim_workload
 *   - paxos.NewPaxos options Q1/Q2/ReplyWhenCommit (paxos/paxos.go:35-58),
 *     Quorum predicates (quorum.go:55-119)                   -> q1/q2/fz fields
 *   - HTTPClient.Consensus agreement check (client.go:279-320) -> paxisim_check
 *
 * Conventions: every call returns 0 or a negative PAXISIM_E* code and never
 * aborts; the message of the last failure on the calling thread is returned
 * by paxisim_last_error().  The library owns all device memory; the caller
 * owns the host buffers it passes in.  Calls on one handle must be
 * serialized (mirrors the reference's one-handler-goroutine-per-replica);
 * distinct handles (one per GPU) may be driven from parallel host threads.
 *
 * The simulation semantics (delivery schedule, bounded-window rules, PRNG)
 * are specified in DESIGN.md §3; the CPU oracle under oracle/ restates them
 * from the reference's Go handlers and is the parity checker.
 */
#ifndef PAXISIM_H
#define PAXISIM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PAXISIM_ABI_VERSION 13

#define PAXISIM_MAX_N        16  /* replicas per cluster (ack masks are u16) */
#define PAXISIM_MAX_ZONES    16
#define PAXISIM_MAX_WORKERS  32  /* closed-loop client workers per cluster */
#define PAXISIM_MAX_KEYS     64  /* keys per cluster (workload key space) */
#define PAXISIM_MAX_FAULTS   64  /* scripted fault windows per handle */
#define PAXISIM_MAX_WINDOW   64  /* log window slots per replica */
#define PAXISIM_MAX_MBOX     64  /* records per (link, arrival-step) bucket */
#define PAXISIM_MAX_DELAY    14  /* Slow delay, in steps */
#define PAXISIM_CLIENT_SRC   31  /* request origin: the client (HTTP path, http.go:99) */

/* ---- error codes ---- */
#define PAXISIM_OK          0
#define PAXISIM_EINVAL     -1   /* bad argument / config */
#define PAXISIM_ENOMEM     -2   /* device or host allocation failed */
#define PAXISIM_EDEVICE    -3   /* HIP runtime error */
#define PAXISIM_EUNSUPP    -4   /* feature not built */
#define PAXISIM_ERANGE     -5   /* cluster range outside the handle */

/* ---- protocols (server/server.go:38-84 algorithm switch) ---- */
enum paxisim_protocol {
  PAXISIM_PAXOS  = 0,   /* paxos/paxos.go + paxos/replica.go */
  PAXISIM_ABD    = 1,   /* abd/replica.go */
  PAXISIM_WPAXOS = 2,   /* wpaxos/replica.go + wpaxos/kpaxos.go */
  PAXISIM_M2PAXOS = 3,  /* m2paxos/replica.go + m2paxos/kpaxos.go: WPaxos' per-key instances and
                           leader stealing with Majority Q1/Q2, always adaptive */
  PAXISIM_KPAXOS = 4,   /* kpaxos/replica.go: per-key paxos.Paxos (Majority), static leader of a key
                           by key range (index(), kpaxos/replica.go:32-44), no stealing */
  PAXISIM_EPAXOS = 5    /* epaxos/replica.go, instance.go: leaderless; every replica leads its own
                           instances (PreAccept fast path on FastQuorum, quorum.go:65-67, else
                           Accept on Majority); execution walks each owner's log in slot order */
};

/* ---- quorum predicates (quorum.go) ---- */
enum paxisim_quorum {
  PAXISIM_Q_MAJORITY     = 0,  /* size > n/2              quorum.go:60-62  */
  PAXISIM_Q_ALL          = 1,  /* size == n               quorum.go:55-57  */
  PAXISIM_Q_FAST         = 2,  /* size >= n*3/4           quorum.go:65-67  */
  PAXISIM_Q_GRID_ROW     = 3,  /* AllZones                quorum.go:70-72,85-87 */
  PAXISIM_Q_ZONE_MAJORITY= 4,  /*                         quorum.go:75-82  */
  PAXISIM_Q_GRID_COLUMN  = 5,  /*                         quorum.go:90-97  */
  PAXISIM_Q_FGRID_Q1     = 6,  /* zones w/ majority >= z-fz  quorum.go:100-108 */
  PAXISIM_Q_FGRID_Q2     = 7   /* zones w/ majority >= fz+1  quorum.go:111-119 */
};

/* ---- message types (one 16-byte record each) ---- */
enum paxisim_msg {
  PAXISIM_MSG_NONE      = 0,
  PAXISIM_MSG_REQUEST   = 1,  /* paxi.Request (message.go:24-30), forwarded via socket */
  PAXISIM_MSG_REPLY     = 2,  /* paxi.Reply (message.go:42-48) back to the forwarder */
  PAXISIM_MSG_P1A       = 3,  /* paxos/msg.go:19-21 */
  PAXISIM_MSG_P1B       = 4,  /* paxos/msg.go:33-37 (header; payload follows) */
  PAXISIM_MSG_P1B_ENTRY = 5,  /* one CommandBallot of P1b.Log */
  PAXISIM_MSG_P2A       = 6,  /* paxos/msg.go:44-48 */
  PAXISIM_MSG_P2B       = 7,  /* paxos/msg.go:55-59 */
  PAXISIM_MSG_P3        = 8,  /* paxos/msg.go:66-70 */
  PAXISIM_MSG_GET       = 9,  /* abd/msg.go:17-21 */
  PAXISIM_MSG_GETREPLY  = 10, /* abd/msg.go:24-30 */
  PAXISIM_MSG_SET       = 11, /* abd/msg.go:33-39 */
  PAXISIM_MSG_SETREPLY  = 12, /* abd/msg.go:42-46 */
  PAXISIM_MSG_LEADERCHG = 13, /* wpaxos/msg.go:78-84 */
  PAXISIM_MSG_PREACCEPT = 14, /* epaxos/msg.go:18-25 (payload: seq, Dep) */
  PAXISIM_MSG_PREACCEPTREPLY = 15, /* epaxos/msg.go:31-38 (payload: Dep, Committed) */
  PAXISIM_MSG_ACCEPT    = 16, /* epaxos/msg.go:44-50 (payload: Dep) */
  PAXISIM_MSG_ACCEPTREPLY = 17, /* epaxos/msg.go:52-56 */
  PAXISIM_MSG_COMMIT    = 18, /* epaxos/msg.go:58-65 (payload: seq, Dep) */
  PAXISIM_NMSG          = 20
};

/* ---- per-replica / per-cluster flags ---- */
#define PAXISIM_F_WOVF      0x01u  /* an entry beyond execute+W was not stored */
#define PAXISIM_F_GHOST     0x02u  /* an entry below execute was not (re)created */
#define PAXISIM_F_MBOX_OVF  0x04u  /* a send found its mailbox bucket full: message lost */
#define PAXISIM_F_PEND_OVF  0x08u  /* pending-request / forwards table full */
#define PAXISIM_F_UNFAITHFUL 0x10u /* bounded model may differ from unbounded Go from here */
#define PAXISIM_F_POISON    0x20u  /* the Go reference would panic here; cluster frozen */
#define PAXISIM_F_BALLOT_OVF 0x40u /* ballot counter beyond 2^27 */
#define PAXISIM_F_HIST_OVF  0x80u  /* ABD op history full: later ops not recorded */

/* ---- scripted faults (socket.go:163-199; http.go:137-162 admin hooks) ---- */
enum paxisim_fault_kind {
  PAXISIM_FAULT_DROP  = 0,  /* Drop(to, t): src->dst sends dropped            */
  PAXISIM_FAULT_SLOW  = 1,  /* Slow(to, d, t): src->dst delayed param steps   */
  PAXISIM_FAULT_FLAKY = 2,  /* Flaky(to, p, t): dropped w.p. param ppm        */
  PAXISIM_FAULT_CRASH = 3   /* Crash(t): replica src; step_to=UINT32_MAX = forever (G11) */
};
#define PAXISIM_ALL_DST 0xFFu

/* WPaxos leader-migration policies (policy.go:15-47 NewPolicy, one per kpaxos,
 * wpaxos/kpaxos.go:33).  Wall-clock time is the virtual step. */
enum paxisim_policy {
  PAXISIM_POLICY_CONSECUTIVE = 0, /* "consecutive" n = policy_threshold; 0 = "null" (policy.go:49-69) */
  PAXISIM_POLICY_MAJORITY    = 1, /* "majority": an id with >= sum/2 of the hits in an interval of
                                     policy_interval steps (policy.go:71-101) */
  PAXISIM_POLICY_EMA         = 2  /* "ema": exponential moving average of the zone, alpha =
                                     policy_alpha, epsilon 0.1 (policy.go:103-130) */
};

typedef struct paxisim_config {
  uint32_t protocol;          /* enum paxisim_protocol */
  uint32_t n_zones;           /* Z (config.go:113) */
  uint32_t npz[PAXISIM_MAX_ZONES]; /* nodes per zone; replica ids are "z.n", z,n >= 1,
                                      indexed in IDs.Less order (id.go:61-69) */
  uint32_t q1, q2;            /* enum paxisim_quorum for phase 1 / phase 2; WPaxos derives
                                 them from fz: GridRow/GridColumn or FGridQ1/Q2 (kpaxos.go:15-27) */
  uint32_t fz;                /* FGrid f_z (wpaxos/replica.go:11) */
  uint32_t thrifty;           /* config.Thrifty (paxos.go:126) */
  uint32_t ephemeral_leader;  /* -ephemeral_leader (paxos/replica.go:12) */
  uint32_t reply_when_commit; /* Paxos.ReplyWhenCommit (paxos.go:37) */
  uint32_t adaptive;          /* WPaxos -adaptive (wpaxos/replica.go:10) */
  uint32_t policy_threshold;  /* WPaxos consecutive policy n (policy.go:55-69); 0 = null policy */
  uint32_t window;            /* W: log window per replica (power of 2, 8..64) */
  uint32_t mbox_cap;          /* M: records per (link, arrival-step) bucket */
  uint32_t max_delay;         /* largest Slow delay in steps (<= PAXISIM_MAX_DELAY) */
  uint32_t keys;              /* keys per cluster (ABD <= 64; WPaxos/M2Paxos/KPaxos instances <= 32) */
  uint32_t steps_per_launch;  /* HIP backend: steps fused per kernel launch (0 = auto) */
  uint32_t history;           /* ABD: completed ops recorded per replica (0 = none) */
  int32_t  device;            /* HIP device ordinal */
  uint64_t clusters;          /* clusters held by this handle */
  uint64_t cluster_base;      /* global id of local cluster 0 (multi-GPU sharding) */
  uint64_t seed;
  uint32_t policy;            /* enum paxisim_policy: config.Policy */
  uint32_t policy_interval;   /* MAJORITY: config.Threshold seconds, in steps (>= 1) */
  double   policy_alpha;      /* EMA: config.Threshold, in (0, 1] */
  uint32_t agree_ring;        /* agreement scan: digest checkpoints (every 16 executed slots) kept per
                                 cluster and instance, i.e. the lag in slots / 16 it can bridge;
                                 0 = default (Paxos 1024, WPaxos 128, ABD none) */
  uint32_t kv;                /* 1: every Paxos / WPaxos / M2Paxos / KPaxos / EPaxos replica keeps the
                                 Database (db.go:53-134): Execute writes a write's value (its command
                                 id) to its key and counts database.version; ABD always keeps its KV */
} paxisim_config;

/* Key distributions of the benchmark's key generator (benchmark.go:202-244,
 * Bconfig.Distribution).  Key indices live in [0, keys); the key of a command
 * is a pure function of (cluster, cid), so both backends agree (DESIGN.md
 * §3.8).  The key *value* the reference's Database sees is key_min + index for
 * "order", "uniform" and "conflict" (Go adds Bconfig.Min), the index itself for
 * the table distributions (Go adds no Min there), and 0 for "conflict"'s
 * literal key 0 (benchmark.go:213-214), which has its own index key_space when
 * key_min != 0.  A table draw beyond [0, keys) ("exponential" is unbounded in
 * Go) is not folded: the replica that needs the key raises PAXISIM_F_UNFAITHFUL
 * and uses index keys-1. */
enum paxisim_distribution {
  PAXISIM_DIST_UNIFORM  = 0,  /* "uniform": rand.Intn(K) (benchmark.go:210-211)         */
  PAXISIM_DIST_ORDER    = 1,  /* "order": counter+1 mod K, counter = cid (205-207)      */
  PAXISIM_DIST_CONFLICT = 2,  /* "conflict": key 0 w.p. conflicts %, else order (213-219) */
  PAXISIM_DIST_TABLE    = 3   /* "normal"/"zipfan"/"exponential" (221-233): inverse CDF
                                 over key_cdf, built by the caller (paxi_amd.workload) */
};

typedef struct paxisim_workload {
  uint32_t outstanding;       /* closed-loop workers per cluster (Bconfig.Concurrency) */
  uint32_t max_requests;      /* per worker; 0 = unlimited (Bconfig.N) */
  uint32_t write_ppm;         /* P(write) in parts per million (Bconfig.W) */
  uint32_t locality_ppm;      /* WPaxos: P(key from the worker's own zone) */
  uint32_t target[PAXISIM_MAX_WORKERS]; /* replica each worker sends to */
  uint32_t distribution;      /* enum paxisim_distribution: Bconfig.Distribution */
  uint32_t conflicts;         /* CONFLICT: percent of commands on key 0 (Bconfig.Conflicts) */
  uint32_t key_cdf[PAXISIM_MAX_KEYS]; /* TABLE: key = #{k < keys-1 : u32 draw >= key_cdf[k]};
                                 non-decreasing over [0, keys-1) */
  uint32_t start_step[PAXISIM_MAX_WORKERS]; /* step at which worker w's first request reaches
                                 target[w] (0 = at creation): e.g. clients that turn to
                                 another replica after a crash (BASELINE config 4) */
  uint32_t key_min;           /* Bconfig.Min (benchmark.go:34): the key value of index 0 for ORDER,
                                 UNIFORM and CONFLICT; only KPaxos' static leader assignment (and
                                 trace export) reads key values */
  uint32_t key_space;         /* Bconfig.K of ORDER / UNIFORM / CONFLICT: their counter and draw
                                 range over indices [0, key_space) (0 = keys); CONFLICT with
                                 key_min != 0 puts the literal key 0 at index key_space (needs
                                 key_space < keys) */
  uint32_t key_tail;          /* TABLE: a u32 draw >= key_tail (when nonzero) is a key beyond the
                                 key space (the "exponential" tail): not folded, see above */
  uint32_t move_every;        /* TABLE with Bconfig.Move (benchmark.go:137-140): Mu moves once per
                                 move_every issued commands, i.e. command cid draws from table
                                 e = (cid-1) / move_every of the Mu sequence (0 = Mu fixed) */
  uint32_t move_tables;       /* tables in move_cdf: table e holds the key CDF for the e-th Mu */
  uint32_t move_loop;         /* after the last table the Mu sequence repeats from this one:
                                 e >= move_tables uses move_loop + (e - move_loop) % (move_tables - move_loop) */
  const uint32_t* move_cdf;   /* move_tables x PAXISIM_MAX_KEYS thresholds (copied at create); each
                                 table as key_cdf: non-decreasing over [0, keys-1) */
} paxisim_workload;

/* Random fault process, applied per (cluster, src, dst) link every step. */
typedef struct paxisim_fault_process {
  uint32_t drop_ppm;          /* P(a drop window starts) per step per idle link */
  uint32_t drop_len;          /* window length in steps */
  uint32_t slow_ppm;          /* P(a slow window starts) per step per idle link */
  uint32_t slow_len;
  uint32_t slow_min, slow_max;/* delay drawn uniformly from [min,max] steps */
} paxisim_fault_process;

typedef struct paxisim_fault {
  uint32_t kind;              /* enum paxisim_fault_kind */
  uint32_t src, dst;          /* replica indices; dst may be PAXISIM_ALL_DST */
  uint32_t param;             /* SLOW: delay steps; FLAKY: ppm */
  uint64_t cluster_lo, cluster_hi; /* GLOBAL cluster ids, [lo, hi) */
  uint32_t step_from, step_to;     /* active for step_from <= t < step_to */
} paxisim_fault;

/* Per-replica snapshot (read_state).  WPaxos replicas aggregate their key
 * instances: ballot = highest, slot = keys led (Replica.keys, replica.go:110-118),
 * execute = total executed, active = active instances, p1_acks = mask of
 * existing instances, npending = total pending, digest = chain of key digests. */
typedef struct paxisim_replica_state {
  uint64_t ballot;            /* 64-bit Ballot (ballot.go:15-17) */
  int32_t  slot;              /* highest slot (paxos.go:30) */
  int32_t  execute;           /* next slot to execute (paxos.go:27) */
  uint32_t active;
  uint32_t flags;             /* PAXISIM_F_* raised by this replica */
  uint64_t digest;            /* hash chain of executed (slot, command) */
  uint32_t p1_acks;           /* phase-1 ack mask */
  uint32_t npending;          /* len(p.requests) */
  uint32_t delivered[PAXISIM_NMSG]; /* socket messages consumed by handlers, by type */
  uint32_t client_requests;   /* client requests handled (HTTP path) */
  uint32_t sent;              /* Send() calls (incl. dropped) */
  uint32_t dropped;           /* sends removed by crash/drop/flaky, or lost to unknown id */
  uint32_t discarded;         /* inbound messages discarded while crashed (socket.go:111-118) */
  uint32_t commits;           /* leader commit events (paxos.go:291-292) / ABD Done */
  uint32_t replies;           /* replies delivered to the client */
  uint32_t executed_writes;   /* kv: database.version, the writes Execute applied (db.go:123-134) */
  uint32_t executions;        /* Execute calls (EPaxos counts re-executions, epaxos/replica.go:362-383) */
} paxisim_replica_state;

/* One Paxos instance (read_instances): the single paxos.Paxos of a Multi-Paxos
 * replica, or one kpaxos per key of a WPaxos replica (wpaxos/kpaxos.go:9-14). */
typedef struct paxisim_instance_state {
  uint64_t ballot;            /* 64-bit Ballot */
  int32_t  slot, execute;
  uint32_t active;
  uint32_t exists;            /* WPaxos: r.paxi[key] != nil (Replica.init, replica.go:36-40) */
  uint32_t p1_acks, npending;
  uint64_t digest;            /* hash chain of executed (slot, command) */
  uint32_t policy_last;       /* consecutive policy (policy.go:49-69): last id, 0xFF = "" */
  uint32_t policy_hits;
  uint32_t policy_state[4];   /* MAJORITY: {sum, interval start step, hash of the per-id hits, 0};
                                 EMA: {s (float64 bits) lo, hi, zone, 0}; else 0 */
} paxisim_instance_state;

/* Whole-handle totals (sum over clusters and replicas). */
typedef struct paxisim_stats {
  uint64_t steps;             /* steps simulated so far */
  uint64_t clusters;
  uint64_t delivered[PAXISIM_NMSG];
  uint64_t delivered_total;   /* socket messages delivered (the metric) */
  uint64_t client_requests;
  uint64_t sent, dropped, discarded;
  uint64_t commits;           /* committed slots (the second metric) */
  uint64_t replies;
  uint64_t flagged[8];        /* clusters with flag bit i set */
  /* agreement scan coverage (paxisim_check): a replica reaching a digest
   * checkpoint (every 16 executed slots) compares it with the first replica's
   * digest there; `missed` = the first digest had already left the ring */
  uint64_t agree_compared, agree_missed, agree_mismatch;
} paxisim_stats;

/* One log entry (read_log): paxos/paxos.go:11-18 entry of a slot in the
 * replica's window [execute, execute + W). */
#define PAXISIM_LOG_EXISTS  0x1u  /* p.log[slot] != nil */
#define PAXISIM_LOG_COMMIT  0x2u  /* entry.commit */
#define PAXISIM_LOG_QUORUM  0x4u  /* entry.quorum != nil (created by P2a / re-proposed) */
#define PAXISIM_LOG_REQUEST 0x8u  /* entry.request != nil */
#define PAXISIM_LOG_HELD    0x10u /* slot inside the window (else the fields are 0) */
typedef struct paxisim_log_entry {
  uint64_t ballot;            /* entry.ballot (64-bit Ballot) */
  int32_t  slot;
  uint32_t cmd;               /* command id */
  uint32_t flags;             /* PAXISIM_LOG_* */
  uint32_t acks;              /* entry.quorum ack mask (replica indices) */
  uint32_t request;           /* command id | origin << 27 (origin PAXISIM_CLIENT_SRC = HTTP), or 0 */
  uint32_t pad;
} paxisim_log_entry;

/* One socket record of a replica's inbox (paxisim_read_inbox / paxisim_deliver):
 * the 16-byte record of DESIGN.md §3.2 {hdr = type | n << 8 | key << 16,
 * ballot (compressed: n << 4 | replica index), slot, cid} and its source
 * (replica index, or N = the client queue).  A P1b (and an EPaxos message) is
 * its header record followed by hdr.n payload records from the same source. */
typedef struct paxisim_inbox_record {
  uint32_t src;
  uint32_t hdr;
  uint32_t ballot;
  uint32_t slot;
  uint32_t cid;
} paxisim_inbox_record;

/* One closed-loop worker of a cluster (benchmark.go:246-275 worker): the
 * command it waits on, how many it issued, and the Reply.Value of its last
 * reply - Execute's return value, the key's value before the command
 * (db.go:103-114, paxos.go:352-362; ABD: the value a read returned,
 * abd/replica.go:145-150), as a command id (0 = nil; needs config.kv for the
 * log-based protocols). */
typedef struct paxisim_worker_state {
  uint32_t cid;               /* current command id (0 = the worker is done) */
  uint32_t issued;            /* requests issued */
  uint32_t reply_value;       /* Reply.Value of the last reply */
  uint32_t pad;
} paxisim_worker_state;

typedef struct paxisim paxisim;   /* opaque handle */

int  paxisim_abi_version(void);
const char* paxisim_last_error(void);
/* Fingerprint of the HIP sources and compile flags this library was built
 * from (__graft_entry__.source_id), so a measurement names its binary. */
const char* paxisim_build_id(void);

/* Create a handle.  All clusters start at step 0 with empty state; worker w's
 * first request is waiting at its target replica at step 0. */
int  paxisim_create(const paxisim_config* cfg, const paxisim_workload* wl,
                    const paxisim_fault_process* fp, paxisim** out);
int  paxisim_destroy(paxisim* h);

/* Add a scripted fault window (Drop/Slow/Flaky/Crash). */
int  paxisim_fault_add(paxisim* h, const paxisim_fault* f);

/* Advance every cluster of the handle by nsteps virtual steps. */
int  paxisim_step(paxisim* h, uint32_t nsteps);
int  paxisim_sync(paxisim* h);

/* The HTTP request path (http.go:99, handleRoot puts the request straight on
 * MessageChan): a client request for command `cid` reaches `replica` of local
 * cluster `cluster` in the next step run (paxisim_step).  The closed-loop
 * workers own cids 1 + w + outstanding*j; an injected cid outside that set is
 * an external client whose reply reaches no worker.  EINVAL if the replica's
 * client mailbox for that step is full. */
int  paxisim_inject(paxisim* h, uint64_t cluster, uint32_t replica, uint32_t cid);

/* The records replica `replica` of local cluster `cluster` receives at the
 * next step, source by source (0..N-1, then the client), each source's in
 * FIFO order: what transport.go's per-connection gob decoder hands to
 * node.recv (transport.go:146-165, node.go:79-101) before socket.Recv
 * (socket.go:111-118).  Sent-and-dropped messages never reach a mailbox
 * (socket.go:66-109 drops them at the sender).  *n_out is the count (also
 * when it exceeds cap: then only cap records are written). */
int  paxisim_read_inbox(paxisim* h, uint64_t cluster, uint32_t replica, paxisim_inbox_record* out,
                        uint32_t cap, uint32_t* n_out);

/* Key index (0-based: Key = Bconfig.Min + key) and read/write kind of each of
 * n command ids of local cluster `cluster` (the workload functions of
 * a command's key and kind are functions of its id). */
int  paxisim_commands(paxisim* h, uint64_t cluster, const uint32_t* cids, uint32_t n, uint32_t* keys,
                      uint32_t* writes);

/* Append n records from source `src` (a replica index; N = the client queue)
 * to replica `replica`'s inbox for the next step, after the ones already
 * there: a message arriving off a transport, the replay of a trace decoded
 * from a gob stream (paxi_amd/trace.py).  EINVAL when the bucket is full
 * (mbox_cap records per link and step). */
int  paxisim_deliver(paxisim* h, uint64_t cluster, uint32_t replica, uint32_t src,
                     const paxisim_inbox_record* recs, uint32_t n);

/* The closed-loop workers of local cluster `cluster`: *n_out = outstanding
 * records (cap of them written). */
int  paxisim_read_client(paxisim* h, uint64_t cluster, paxisim_worker_state* out, uint32_t cap, uint32_t* n_out);

/* Totals over the handle. */
int  paxisim_stats_get(paxisim* h, paxisim_stats* out);

/* Per-replica snapshot of local clusters [cluster_lo, cluster_lo+n): out has
 * n*N records, cluster-major. */
int  paxisim_read_state(paxisim* h, uint64_t cluster_lo, uint64_t n,
                        paxisim_replica_state* out);

/* Per-instance snapshot of local clusters [cluster_lo, cluster_lo+n): out has
 * n*N*I records (I = keys for WPaxos, else 1), cluster-major, then replica,
 * then key. */
int  paxisim_read_instances(paxisim* h, uint64_t cluster_lo, uint64_t n,
                            paxisim_instance_state* out);

/* Log entries of slots [slot_lo, slot_lo + n) of one Paxos instance (replica;
 * WPaxos: the kpaxos of `key`) of local cluster `cluster`. */
int  paxisim_read_log(paxisim* h, uint64_t cluster, uint32_t replica, uint32_t key, int32_t slot_lo,
                      uint32_t n, paxisim_log_entry* out);

/* Agreement scan (client.go:279-320 / tla Safety): number of clusters in
 * which two replicas executed different commands in the same slot (of the
 * same key, for WPaxos).  Every replica's executed prefix is compared with
 * the first executor's at each 16-slot checkpoint as it is reached, however
 * far behind it runs (up to agree_ring checkpoints); replicas at the same
 * execute count, and the last 8 checkpoints of every pair, are compared here.
 * Coverage is in paxisim_stats.agree_*. */
int  paxisim_check(paxisim* h, uint64_t* violations);

/* Device time of the step kernels since the last reset (HIP events on the
 * launch stream), and the number of launches. */
int  paxisim_kernel_time(paxisim* h, double* ms, uint64_t* launches, int reset);

/* History.Linearizable (history.go:55-71, checker.go:69-104) over every
 * (cluster, key) of the recorded ABD operations: anomalous reads, operations
 * checked, and partitions skipped because they exceed the checker's bit sets
 * (more than 16384 ops in one (cluster, key); their ops are not in `ops`).
 * Any pointer may be NULL. */
int  paxisim_linearizable(paxisim* h, uint64_t* anomalies, uint64_t* ops, uint64_t* skipped);

/* Completed ABD operations of one local cluster: 5 words per op {key,
 * is_write, value, start step, end step}; replicas in index order, each in
 * completion order (the canonical history order). */
int  paxisim_history(paxisim* h, uint64_t cluster, uint32_t* buf, uint32_t cap_ops, uint32_t* n_out);

/* History.ReadFile (history.go:115-178) into the device: replace the recorded
 * operations of one replica of a local cluster with n ops in the format of
 * paxisim_history (5 words each; n <= config.history), so that
 * paxisim_linearizable checks an imported history (e.g. one written by the
 * reference's client) on the GPU.  ABD handles only. */
int  paxisim_history_load(paxisim* h, uint64_t cluster, uint32_t replica, const uint32_t* ops, uint32_t n);

/* 64-cluster tiles of the step kernel resident per CU (hipOccupancy x tiles
 * per workgroup), LDS per tile, and messages staged into LDS per
 * replica-step (any pointer but the first may be NULL). */
int  paxisim_occupancy(paxisim* h, int* blocks_per_cu, uint32_t* lds_bytes, uint32_t* staged);

/* Database.Get (db.go:116-121) for keys [0, n) of one replica of a local
 * cluster (kv on; ABD: its KV): the value is the command id of the write that
 * set it, 0 = nil.  A read's reply value (Execute's previous value, db.go:
 * 103-114) is the value its key held when the command executed. */
int  paxisim_read_kv(paxisim* h, uint64_t cluster, uint32_t replica, uint32_t* values, uint32_t n);

/* Clusters still stepped: a Paxos cluster whose mailboxes are all empty is at
 * a fixed point (no timers, no retries: paxos/paxos.go) and is frozen and
 * packed behind the active ones; an injected request wakes it.  Results are
 * identical either way; this reports how many clusters the
 * step kernels still visit. */
int  paxisim_active_clusters(paxisim* h, uint64_t* active);

/* Per local cluster of [cluster_lo, cluster_lo+n): PAXISIM_STEPPED if the step
 * kernels still visit it, else the step at which it was frozen at its fixed
 * point.  Diagnostics for sampling parity checks; the state
 * of a cluster does not depend on it. */
#define PAXISIM_STEPPED 0xFFFFFFFFu
int  paxisim_read_activity(paxisim* h, uint64_t cluster_lo, uint64_t n, uint32_t* frozen_at);

/* The quorum predicate the kernels evaluate (quorum.go:55-119 on an ack mask
 * of replica indices in IDs.Less order), for the zones of cfg (n_zones, npz,
 * fz): a host function, no device needed.  Lets a caller hold the kernels'
 * predicates against its own quorum.go (sim.Quorum). */
int  paxisim_quorum(const paxisim_config* cfg, uint32_t kind, uint32_t ack_mask, int* satisfied);

/* Bytes of device memory held by the handle. */
int  paxisim_device_bytes(paxisim* h, uint64_t* bytes);

/* ---- Multi-GPU: clusters shard by range over handles
 * (paxisim_config.cluster_base = rank * clusters), the simulation itself has
 * no collective, and totals are reduced with RCCL (opened at run time:
 * EUNSUPP without librccl.so.1).  Replaces nothing in the reference, which
 * simulates one cluster per process. */
typedef struct paxisim_dist paxisim_dist;
/* One process driving one handle per device: a communicator clique. */
int  paxisim_dist_init(paxisim* const* handles, int n, paxisim_dist** out);
/* One handle per process: one rank gets an id, the caller ships its 128 bytes
 * to every rank, and each rank joins with it. */
int  paxisim_dist_unique_id(unsigned char id[128]);
int  paxisim_dist_init_rank(paxisim* h, const unsigned char id[128], int nranks, int rank, paxisim_dist** out);
/* Sum n u64 values and max m doubles over every handle of every rank; member
 * k of this process supplies sums_in[k*n..] and maxes_in[k*m..] (n, m <= 64). */
int  paxisim_dist_allreduce(paxisim_dist* d, const uint64_t* sums_in, uint32_t n, const double* maxes_in,
                            uint32_t m, uint64_t* sums_out, double* maxes_out);
/* paxisim_stats summed over every handle of the job (flagged[] are cluster
 * counts, so they sum too), and the largest step-kernel time (may be NULL). */
int  paxisim_dist_stats(paxisim_dist* d, paxisim_stats* out, double* kernel_ms_max);
int  paxisim_dist_destroy(paxisim_dist* d);

#ifdef __cplusplus
}
#endif
#endif /* PAXISIM_H */
