/*
 * oracle.c — single-threaded CPU restatement of Paxi's simulation-mode hot
 * path under the delivery schedule of DESIGN.md §3.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h): the parity checker for the HIP
 * product path and the source of the CPU baseline timing.  It is written to
 * read like the Go it restates — one function per reference handler, each
 * citing the file:line it follows — not to be fast.
 *
 * Parity pinning: see oracle.h and DESIGN.md §4 (Go toolchain absent; pinned
 * by ballot_test.go / checker_test.go KATs and hand-derived KATs).
 */
#include "oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static __thread char g_err[256];
static int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
  return code;
}
const char* oracle_last_error(void) { return g_err; }

/* ------------------------------------------------------------------------ */
/* PRNG: counter-based, keyed by (seed, cluster, step, tag). */
/* ------------------------------------------------------------------------ */
static inline uint64_t mix64(uint64_t z) {
  z ^= z >> 30; z *= 0xbf58476d1ce4e5b9ULL;
  z ^= z >> 27; z *= 0x94d049bb133111ebULL;
  z ^= z >> 31;
  return z;
}
static inline uint32_t fmix32(uint32_t h) {
  h ^= h >> 16; h *= 0x85ebca6bu;
  h ^= h >> 13; h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}
/* per-cluster 32-bit key, derived once from the 64-bit seed and global id */
static inline uint32_t cluster_key(uint64_t seed, uint64_t gid) {
  return (uint32_t)mix64(seed ^ mix64(gid + 0x9E3779B97F4A7C15ULL));
}
/* per-(cluster, step) stream key; every draw of that step hashes a tag into it */
static inline uint32_t step_key(uint32_t kc, uint32_t t) { return fmix32(kc ^ (t * 0x9E3779B1u)); }
static inline uint32_t draw(uint32_t hs, uint32_t tag) { return fmix32(hs ^ tag); }
#define TAG(p, a, b) (((uint32_t)(p) << 28) | ((uint32_t)(a) << 20) | (uint32_t)(b))
enum { PUR_ORDER = 1, PUR_LINK = 2, PUR_SLOWD = 3, PUR_FLAKY = 4, PUR_WL = 5 };
/* P(x32 hits) = ppm / 1e6 */
static inline int ppm_hit(uint32_t x, uint32_t ppm) {
  return (uint32_t)(((uint64_t)x * 1000000ULL) >> 32) < ppm;
}
/* 16-bit variant: (x16 * 1e6) >> 16 == (x16 * 15625) >> 10 exactly */
static inline int ppm_hit16(uint32_t x16, uint32_t ppm) { return ((x16 * 15625u) >> 10) < ppm; }

/* ------------------------------------------------------------------------ */
/* Ballot / ID (ballot.go:15-52, id.go:14-69).  In-simulation a ballot is      */
/* kept compressed as (n << 4) | r, r = replica index in IDs.Less order, which */
/* preserves the uint64 order of (n<<32 | zone<<16 | node).                    */
/* ------------------------------------------------------------------------ */
#define NO_ID 0xFFu
static inline uint32_t bal_id(uint32_t b) { return b ? (b & 15u) : NO_ID; } /* Ballot.ID() ballot.go:43-47; 0 -> "0.0" */
static inline uint32_t bal_next(uint32_t b, uint32_t self) {                /* Ballot.Next ballot.go:50-52 */
  return (((b >> 4) + 1u) << 4) | self;
}

uint64_t oracle_new_ballot(uint32_t n, uint32_t zone, uint32_t node) { /* NewBallot ballot.go:15-17 */
  return ((uint64_t)n << 32) | ((uint64_t)zone << 16) | (uint64_t)node;
}
uint64_t oracle_ballot_next(uint64_t b, uint32_t zone, uint32_t node) {
  return oracle_new_ballot((uint32_t)(b >> 32) + 1u, zone, node);
}

/* ------------------------------------------------------------------------ */
/* Quorum predicates (quorum.go:55-119) over an ack mask.                      */
/* ------------------------------------------------------------------------ */
static int popc(uint32_t x) { return __builtin_popcount(x); }

static int quorum_eval(uint32_t kind, uint32_t fz, uint32_t nz, const uint32_t* npz,
                       const uint32_t* zmask, uint32_t n, uint32_t mask) {
  int size = popc(mask);
  uint32_t z, zones_any = 0, zones_maj = 0, col = 0, zmaj = 0;
  for (z = 0; z < nz; z++) {
    uint32_t c = (uint32_t)popc(mask & zmask[z]);
    if (c > 0) zones_any++;
    if (c > npz[z] / 2) { zones_maj++; zmaj = 1; }
    if (c == npz[z]) col = 1;
  }
  switch (kind) {
    case PAXISIM_Q_MAJORITY:      return size > (int)(n / 2);           /* quorum.go:60-62 */
    case PAXISIM_Q_ALL:           return size == (int)n;                /* quorum.go:55-57 */
    case PAXISIM_Q_FAST:          return size >= (int)(n * 3 / 4);      /* quorum.go:65-67 */
    case PAXISIM_Q_GRID_ROW:      return zones_any == nz;               /* quorum.go:70-72,85-87 */
    case PAXISIM_Q_ZONE_MAJORITY: return (int)zmaj;                     /* quorum.go:75-82 */
    case PAXISIM_Q_GRID_COLUMN:   return (int)col;                      /* quorum.go:90-97 */
    case PAXISIM_Q_FGRID_Q1:      return (int)zones_maj >= (int)nz - (int)fz; /* quorum.go:100-108 */
    case PAXISIM_Q_FGRID_Q2:      return (int)zones_maj >= (int)fz + 1; /* quorum.go:111-119 */
  }
  return 0;
}

int oracle_quorum(uint32_t kind, uint32_t fz, uint32_t n_zones, const uint32_t* npz,
                  uint32_t ack_mask) {
  uint32_t zmask[PAXISIM_MAX_ZONES], z, r = 0, n = 0;
  for (z = 0; z < n_zones; z++) {
    zmask[z] = ((1u << npz[z]) - 1u) << r;
    r += npz[z];
  }
  n = r;
  return quorum_eval(kind, fz, n_zones, npz, zmask, n, ack_mask);
}

/* ------------------------------------------------------------------------ */
/* Simulation state                                                          */
/* ------------------------------------------------------------------------ */
typedef struct { uint32_t hdr, ballot, slot, cid; } rec_t;   /* 16-B message record */
/* an entry re-created below execute: slot, ballot, commit, live while t < until */
typedef struct { uint32_t slot, ballot, commit, until; } ghost_t;
#define GMAX 8
#define HDR(type, n) ((uint32_t)(type) | ((uint32_t)(n) << 8))
#define HDR_TYPE(h) ((h) & 0xFFu)
#define HDR_N(h) (((h) >> 8) & 0xFFu)
#define HDR_KEY(h) ((h) >> 16)       /* WPaxos key (wpaxos/msg.go Key fields) */
/* records of a message: a P1b and the EPaxos messages carry payload records */
static inline uint32_t rec_len(uint32_t h) {
  const uint32_t t = HDR_TYPE(h);
  return 1u + ((t == PAXISIM_MSG_P1B || (t >= PAXISIM_MSG_PREACCEPT && t <= PAXISIM_MSG_COMMIT)) ? HDR_N(h) : 0u);
}

/* log entry (paxos/paxos.go:11-18): ballot, command, request, quorum, commit */
typedef struct { uint32_t ballot, cmd, req, meta; } entry_t;
#define E_EXISTS 1u
#define E_COMMIT 2u
#define E_QUORUM 4u   /* quorum != nil */
#define E_ACK(m) ((m) >> 16)

/* a request = command id + who to reply to (message.go:24-30 NodeID/c) */
#define REQ(cid, origin) ((uint32_t)(cid) | ((uint32_t)(origin) << 27))
#define REQ_CID(q) ((q) & 0x07FFFFFFu)
#define REQ_ORIGIN(q) ((q) >> 27)
#define CID_MAX 0x07FFFFFFu

#define PMAX 32
#define FMAX 32
#define KMAX 64  /* ABD keys per cluster */
#define WP_KMAX 32  /* WPaxos keys (kpaxos instances) per cluster */
#define CKI 16   /* checkpoint every CKI executed slots */
#define CKR 8    /* checkpoints kept per replica */

/* ABD op table entry (abd/replica.go:17-24), ring indexed by coordinator cid */
typedef struct { uint32_t tag, req, state, getmask, setmask, value, version, start; } abd_op_t;
enum { ABD_FREE = 0, ABD_GET = 1, ABD_SET = 2, ABD_DONE = 3 };
/* one completed client operation (operation.go:5-11), for History.Linearizable */
typedef struct { uint32_t key, is_write, value, start, end; } hist_t;

/* One paxos.Paxos instance (paxos/paxos.go:21-38).  Paxos: one per replica;
 * WPaxos: one kpaxos per (replica, key) (wpaxos/kpaxos.go:9-14), created on
 * first use by Replica.init (wpaxos/replica.go:37-41). */
typedef struct inst {
  uint32_t ballot;
  int32_t slot, execute;
  uint32_t active;
  uint32_t p1mask;                 /* p.quorum (phase 1) */
  uint32_t npend, pend[PMAX];      /* p.requests */
  entry_t* log;                    /* p.log, window [execute, execute+W) */
  /* executed-history digest + checkpoints */
  uint64_t digest;
  uint32_t ck_e[CKR];
  uint64_t ck_d[CKR];
  /* exec log (KATs) */
  uint32_t* xlog;
  uint32_t nx, capx;
  /* WPaxos: r.paxi[key] != nil, and the consecutive policy (policy.go:49-69) */
  uint32_t exists, pol_last, pol_hits;
  /* majority (policy.go:71-101): hits per id, their sum, interval start step;
   * ema (policy.go:103-130): s and zone */
  uint32_t pol_n[PAXISIM_MAX_N], pol_sum, pol_time, pol_zone;
  double pol_s;
  uint32_t iflags;                 /* WOVF / GHOST raised on this instance's log */
  /* Entries Go holds below execute ("ghosts"), while they can still be observed */
  ghost_t ghost[GMAX];
} inst_t;

/* EPaxos instance (epaxos/instance.go:16-28); dep[id] = 0 reads as absent, as a Go map does */
typedef struct {
  uint32_t cmd, req, acks;
  int32_t seq, slot;               /* slot: which of the ring's slots this entry holds */
  uint8_t exists, ballot, status, changed;
  uint32_t nrep;                   /* replies sent for this instance's request */
  int32_t dep[PAXISIM_MAX_N];
} ep_inst_t;

typedef struct replica {
  inst_t* inst;                    /* NK instances (key-major) */
  /* EPaxos (epaxos/replica.go:14-27): per owner log ring, slot/committed/executed, conflicts */
  ep_inst_t* ep_log;               /* [N][W] */
  int32_t ep_slot[PAXISIM_MAX_N], ep_committed[PAXISIM_MAX_N], ep_executed[PAXISIM_MAX_N];
  int32_t* ep_cf;                  /* [N][keys][2] {slot or -1, seq} */
  int32_t* ep_maxseq;              /* [keys], -1 = absent */
  uint32_t ep_execs;               /* Execute calls (re-executions included) */
  uint32_t* db;                    /* kv: Database (db.go) values per key, command id of the last write */
  uint32_t db_version;             /* database.version */
  /* node.forwards (node.go:35, 165-172) */
  uint32_t nfwd, fwd[FMAX];
  /* socket fault state (socket.go:26-34), random process */
  uint32_t drop_until[PAXISIM_MAX_N], slow_until[PAXISIM_MAX_N], slow_delay[PAXISIM_MAX_N];
  uint32_t flags;
  uint32_t send_seq;
  /* counters */
  uint32_t delivered[PAXISIM_NMSG];
  uint32_t client_requests, sent, dropped, discarded, commits, replies;
  uint32_t agc, agm, agb;          /* agreement checkpoints compared / missed / mismatched */
  uint32_t nag;                    /* agreement arrivals in the current step (AGMAX rule) */
  /* ABD (abd/replica.go:28-34): cid counter, versioned KV, op table */
  uint32_t abd_cid;
  uint32_t *kv_val, *kv_ver;
  abd_op_t* ops;
  hist_t* hist;                    /* completed ops coordinated here (cfg.history of them) */
  uint32_t nh;
} replica_t;

typedef struct cluster {
  uint64_t gid;
  uint32_t kc;
  uint32_t poison_step;            /* first step at which a replica panicked */
  uint32_t wk_cur[PAXISIM_MAX_WORKERS], wk_issued[PAXISIM_MAX_WORKERS];
  uint32_t wk_rep[PAXISIM_MAX_WORKERS];   /* Reply.Value of the worker's last reply (0 = nil) */
  replica_t rep[PAXISIM_MAX_N];
  rec_t* mbox;                     /* [D][N][N+1][M] */
  uint64_t* agr;                   /* [NK][AR] first executor's digest per checkpoint: k << 40 | fold */
  uint8_t* cnt;                    /* [D][N][N+1] */
} cluster_t;

struct oracle_sim {
  paxisim_config cfg;
  paxisim_workload wl;
  paxisim_fault_process fp;
  uint32_t N, Z, W, M, D, NS;      /* NS = N+1 sources (N = client) */
  uint32_t zone_of[PAXISIM_MAX_N], node_of[PAXISIM_MAX_N], zmask[PAXISIM_MAX_ZONES];
  paxisim_fault faults[PAXISIM_MAX_FAULTS];
  uint32_t nfaults;
  uint64_t C;
  cluster_t* cl;
  uint32_t t;                      /* next step to simulate */
  int keep_xlog;
  uint32_t OW;                     /* ABD op table size */
  uint32_t NK;                     /* Paxos instances per replica: WPaxos keys, else 1 */
  uint32_t q1, q2;                 /* quorum kinds in use (WPaxos: from fz, wpaxos/kpaxos.go:16-28) */
  uint32_t late_workers;           /* some worker has start_step > 0 */
  uint32_t variant;                /* per-key protocol (cfg.protocol reads WPAXOS): WPAXOS, M2PAXOS, KPAXOS */
  uint32_t zfirst[PAXISIM_MAX_ZONES]; /* replica index of "z.1" */
  uint32_t AR;                     /* agreement ring: checkpoints kept per (cluster, instance) */
  uint32_t order;                  /* test hook: replica order within a step (oracle_set_replica_order) */
  int kv;                          /* replicas keep the Database (paxisim_config.kv) */
  uint32_t* move_cdf;              /* moving-Mu key CDF tables (a copy of paxisim_workload.move_cdf) */
};

/* handler context: one replica of one cluster at one step */
typedef struct ctx {
  const struct oracle_sim* s;
  cluster_t* c;
  replica_t* n;                    /* the node (paxi.Node: socket, forwards, counters) */
  inst_t* p;                       /* the bound Paxos instance */
  uint32_t ktag;                   /* WPaxos: key << 16, tagged onto P1a..P3 records */
  uint32_t r, t, hs;
  int stop;                        /* replica panicked in this step */
} ctx_t;

static inline rec_t* mb_rec(const struct oracle_sim* s, cluster_t* c, uint32_t b, uint32_t dst,
                            uint32_t src, uint32_t k) {
  return &c->mbox[(((size_t)b * s->N + dst) * s->NS + src) * s->M + k];
}
static inline uint8_t* mb_cnt(const struct oracle_sim* s, cluster_t* c, uint32_t b, uint32_t dst,
                              uint32_t src) {
  return &c->cnt[((size_t)b * s->N + dst) * s->NS + src];
}

static inline void raise_flag(ctx_t* x, uint32_t f) {
  x->n->flags |= f;
  x->p->iflags |= f & (PAXISIM_F_WOVF | PAXISIM_F_GHOST);   /* window flags are per instance */
}

/* ------------------------------------------------------------------------ */
/* Fault filter (socket.go:66-109): crash -> drop -> flaky -> slow           */
/* ------------------------------------------------------------------------ */
static int scripted(const struct oracle_sim* s, uint32_t kind, uint64_t gid, uint32_t src,
                    uint32_t dst, uint32_t t, uint32_t* param) {
  int hit = 0;
  uint32_t i;
  for (i = 0; i < s->nfaults; i++) {
    const paxisim_fault* f = &s->faults[i];
    if (f->kind != kind || f->src != src) continue;
    if (kind != PAXISIM_FAULT_CRASH && f->dst != PAXISIM_ALL_DST && f->dst != dst) continue;
    if (gid < f->cluster_lo || gid >= f->cluster_hi) continue;
    if (t < f->step_from || t >= f->step_to) continue;
    hit = 1;
    if (param && f->param > *param) *param = f->param;
  }
  return hit;
}
static int crashed(const struct oracle_sim* s, const cluster_t* c, uint32_t r, uint32_t t) {
  return scripted(s, PAXISIM_FAULT_CRASH, c->gid, r, 0, t, NULL);
}

/* socket.Send (socket.go:66-109) with the bucketed mailbox of DESIGN.md §3.2. */
static void sock_send(ctx_t* x, uint32_t to, const rec_t* recs, uint32_t nrec) {
  const struct oracle_sim* s = x->s;
  replica_t* p = x->n;
  uint32_t seq = p->send_seq++, delay = 0, flaky = 0, b;
  uint8_t* cnt;
  p->sent++;
  if (to >= s->N) { p->dropped++; return; }                      /* unknown id: socket.go:86-88 */
  if (crashed(s, x->c, x->r, x->t)) { p->dropped++; return; }    /* socket.go:69 */
  if (x->t < p->drop_until[to] ||
      scripted(s, PAXISIM_FAULT_DROP, x->c->gid, x->r, to, x->t, NULL)) { p->dropped++; return; } /* 73 */
  if (scripted(s, PAXISIM_FAULT_FLAKY, x->c->gid, x->r, to, x->t, &flaky) && flaky > 0) {         /* 77-81 */
    uint32_t u = draw(x->hs, TAG(PUR_FLAKY, x->r, seq));
    if (ppm_hit(u, flaky)) { p->dropped++; return; }
  }
  if (x->t < p->slow_until[to]) delay = p->slow_delay[to];        /* 99-106 */
  scripted(s, PAXISIM_FAULT_SLOW, x->c->gid, x->r, to, x->t, &delay);
  if (delay > s->cfg.max_delay) delay = s->cfg.max_delay;
  b = (x->t + 1u + delay) % s->D;
  cnt = mb_cnt(s, x->c, b, to, x->r);
  if ((uint32_t)*cnt + nrec > s->M) {                             /* bounded mailbox: lost */
    raise_flag(x, PAXISIM_F_MBOX_OVF | PAXISIM_F_UNFAITHFUL);
    p->dropped++;
    return;
  }
  memcpy(mb_rec(s, x->c, b, to, x->r, *cnt), recs, nrec * sizeof(rec_t));
  *cnt = (uint8_t)(*cnt + nrec);
}

static void send1(ctx_t* x, uint32_t to, uint32_t type, uint32_t ballot, uint32_t slot, uint32_t cid) {
  rec_t m;
  m.hdr = HDR(type, 0); m.ballot = ballot; m.slot = slot; m.cid = cid;
  sock_send(x, to, &m, 1);
}

/* Broadcast: every peer except self, in IDs.Less order (socket.go:147-155; G1, G2) */
static void broadcast1(ctx_t* x, uint32_t type, uint32_t ballot, uint32_t slot, uint32_t cid) {
  uint32_t d;
  for (d = 0; d < x->s->N; d++)
    if (d != x->r) send1(x, d, type, ballot, slot, cid);
}
/* MulticastQuorum(q): the first q peers in ring order after self (socket.go:132-145; G8) */
static void multicast_quorum1(ctx_t* x, uint32_t q, uint32_t type, uint32_t ballot, uint32_t slot,
                              uint32_t cid) {
  uint32_t i, sent = 0, N = x->s->N;
  for (i = 1; i < N && sent < q; i++, sent++) send1(x, (x->r + i) % N, type, ballot, slot, cid);
}

/* ------------------------------------------------------------------------ */
/* Client (benchmark.go:246-275 worker; http.go:99 request path)            */
/* ------------------------------------------------------------------------ */
static void client_enqueue(ctx_t* x, uint32_t target, uint32_t cid) {
  const struct oracle_sim* s = x->s;
  uint32_t b = (x->t + 1u) % s->D;
  uint8_t* cnt = mb_cnt(s, x->c, b, target, s->N);
  rec_t* m;
  if (*cnt >= s->M) { raise_flag(x, PAXISIM_F_MBOX_OVF | PAXISIM_F_UNFAITHFUL); return; }
  m = mb_rec(s, x->c, b, target, s->N, *cnt);
  m->hdr = HDR(PAXISIM_MSG_REQUEST, 0); m->ballot = 0; m->slot = 0; m->cid = cid;
  (*cnt)++;
}

/* The HTTP response reaches worker w (its Reply.Value kept: the value a
 * read returned, benchmark.go:259-262); it issues its next request. */
static void client_reply(ctx_t* x, uint32_t cid, uint32_t value) {
  const struct oracle_sim* s = x->s;
  uint32_t WK = s->wl.outstanding, w = (cid - 1u) % WK;
  if (x->c->wk_cur[w] != cid) return;                /* duplicate reply: worker moved on */
  x->n->replies++;
  x->c->wk_rep[w] = value;
  if (s->wl.max_requests == 0 || x->c->wk_issued[w] < s->wl.max_requests) {
    uint64_t nc = 1ull + w + (uint64_t)WK * x->c->wk_issued[w];
    if (nc > CID_MAX) { raise_flag(x, PAXISIM_F_PEND_OVF | PAXISIM_F_UNFAITHFUL); x->c->wk_cur[w] = 0; return; }
    x->c->wk_issued[w]++;
    x->c->wk_cur[w] = (uint32_t)nc;
    client_enqueue(x, s->wl.target[w], (uint32_t)nc);
  } else {
    x->c->wk_cur[w] = 0;
  }
}

/* Request.Reply (message.go:32-34): to the client, or back over the socket to
 * the node the request came from (node.go:83-90 reply goroutine). */
static void request_reply(ctx_t* x, uint32_t req, uint32_t reply_cmd, uint32_t value) {
  uint32_t o = REQ_ORIGIN(req);
  if (o == PAXISIM_CLIENT_SRC) client_reply(x, REQ_CID(req), value);
  else send1(x, o, PAXISIM_MSG_REPLY, value, 0, reply_cmd);   /* Reply{Command, Value}: value in the ballot word */
}

/* node.Forward (node.go:165-172): remember the request, send it to id. */
static void node_forward(ctx_t* x, uint32_t to, uint32_t req) {
  replica_t* p = x->n;
  uint32_t i, cid = REQ_CID(req);
  for (i = 0; i < p->nfwd; i++)
    if (REQ_CID(p->fwd[i]) == cid) break;
  if (i == p->nfwd) {
    if (p->nfwd == FMAX) raise_flag(x, PAXISIM_F_PEND_OVF | PAXISIM_F_UNFAITHFUL);
    else p->fwd[p->nfwd++] = req;
  } else {
    p->fwd[i] = req;
  }
  send1(x, to, PAXISIM_MSG_REQUEST, 0, 0, cid);
}

/* node.recv Reply case (node.go:83-90): forwards[cmd].Reply(m). */
static void handle_reply(ctx_t* x, uint32_t cid, uint32_t value) {
  replica_t* p = x->n;
  uint32_t i;
  for (i = 0; i < p->nfwd; i++)
    if (REQ_CID(p->fwd[i]) == cid) break;
  if (i == p->nfwd) {               /* Go: nil *Request (panic) or a retired entry */
    raise_flag(x, PAXISIM_F_UNFAITHFUL);
    return;
  }
  {
    uint32_t req = p->fwd[i];
    p->fwd[i] = p->fwd[--p->nfwd];  /* retire (bounded memory) */
    request_reply(x, req, cid, value);
  }
}

/* ------------------------------------------------------------------------ */
/* Multi-Paxos (paxos/paxos.go, paxos/replica.go)                            */
/* ------------------------------------------------------------------------ */
static inline int in_window(const ctx_t* x, int32_t s) {
  return s >= x->p->execute && s < x->p->execute + (int32_t)x->s->W;
}
static inline entry_t* log_at(const ctx_t* x, int32_t s) { return &x->p->log[(uint32_t)s & (x->s->W - 1u)]; }
static inline int q1_ok(const ctx_t* x, uint32_t m) {
  const struct oracle_sim* s = x->s;
  return quorum_eval(s->q1, s->cfg.fz, s->Z, s->cfg.npz, s->zmask, s->N, m);
}
static inline int q2_ok(const ctx_t* x, uint32_t m) {
  const struct oracle_sim* s = x->s;
  return quorum_eval(s->q2, s->cfg.fz, s->Z, s->cfg.npz, s->zmask, s->N, m);
}
static inline int is_leader(const ctx_t* x) {             /* Paxos.IsLeader paxos.go:61-63 */
  return x->p->active || bal_id(x->p->ballot) == x->r;
}

/* Entries below execute ("ghosts").  exec() deletes an executed entry
 * (paxos.go:366), but update() (173-177), HandleP2a (254-258) and HandleP3
 * (326) re-create one when a message for an executed slot arrives, and Go
 * keeps it forever.  Such an entry is read only by HandleP2b (270-310): a P2b
 * for the slot adopts a higher ballot, or panics on the nil quorum when the
 * ballot is this replica's own and equals the entry's.  A P2b for slot s
 * reaches replica r only as the answer to a P2a(s) r sent while s >= execute,
 * so it arrives at most 2 + 2*max_delay steps after r executed s: a ghost is
 * kept for that long after it is (re)created and then forgotten.  Within that
 * life the table is exact; a full table raises UNFAITHFUL. */
static inline uint32_t ghost_life(const ctx_t* x) { return 3u + 2u * x->s->cfg.max_delay; }
static ghost_t* ghost_find(ctx_t* x, int32_t s) {
  uint32_t i;
  for (i = 0; i < GMAX; i++) {
    ghost_t* g = &x->p->ghost[i];
    if (g->until > x->t && g->slot == (uint32_t)s) return g;
  }
  return NULL;
}
static ghost_t* ghost_alloc(ctx_t* x, int32_t s) {
  uint32_t i;
  raise_flag(x, PAXISIM_F_GHOST);
  for (i = 0; i < GMAX; i++) {
    ghost_t* g = &x->p->ghost[i];
    if (g->until <= x->t) {
      g->slot = (uint32_t)s; g->ballot = 0; g->commit = 0; g->until = x->t + ghost_life(x);
      return g;
    }
  }
  raise_flag(x, PAXISIM_F_UNFAITHFUL);                     /* cannot keep this ghost */
  return NULL;
}
/* update() / HandleP2a on a slot below execute: create, or raise an uncommitted ballot */
static void ghost(ctx_t* x, int32_t s, uint32_t b) {
  ghost_t* g = ghost_find(x, s);
  if (g) {
    if (!g->commit && b > g->ballot) g->ballot = b;
    return;
  }
  if ((g = ghost_alloc(x, s))) g->ballot = b;
}
/* HandleP3 on a slot below execute: the entry exists and is committed (326-331) */
static void ghost_commit(ctx_t* x, int32_t s) {
  ghost_t* g = ghost_find(x, s);
  if (!g) g = ghost_alloc(x, s);
  if (g) g->commit = 1;
}
/* HandleP2b (270-310) for a slot below execute */
static void ghost_p2b(ctx_t* x, int32_t ms, uint32_t mb) {
  inst_t* p = x->p;
  ghost_t* g = ghost_find(x, ms);
  if (!g || mb < g->ballot || g->commit) return;           /* !exist || m.Ballot < e.ballot || e.commit */
  if (mb > p->ballot) {
    p->ballot = mb;
    p->active = 0;
  }
  if (bal_id(mb) == x->r && mb == g->ballot) {             /* nil quorum: Go panics */
    raise_flag(x, PAXISIM_F_POISON);
    x->stop = 1;
  }
}

static void paxos_forward(ctx_t* x) {                     /* paxos.go:371-376 */
  inst_t* p = x->p;
  uint32_t i;
  for (i = 0; i < p->npend; i++) node_forward(x, bal_id(p->ballot), p->pend[i]);
  p->npend = 0;
}

static void paxos_p1a(ctx_t* x) {                         /* paxos.go:100-108 */
  inst_t* p = x->p;
  if (p->active) return;
  if ((p->ballot >> 4) + 1u >= (1u << 27)) raise_flag(x, PAXISIM_F_BALLOT_OVF | PAXISIM_F_UNFAITHFUL);
  p->ballot = bal_next(p->ballot, x->r);
  p->p1mask = 1u << x->r;
  broadcast1(x, PAXISIM_MSG_P1A | x->ktag, p->ballot, 0, 0);
}

static void paxos_p2a(ctx_t* x, uint32_t req) {           /* paxos.go:111-131 */
  const struct oracle_sim* s = x->s;
  inst_t* p = x->p;
  p->slot++;
  if (in_window(x, p->slot)) {
    entry_t* e = log_at(x, p->slot);
    e->ballot = p->ballot;
    e->cmd = REQ_CID(req);
    e->req = req;
    e->meta = E_EXISTS | E_QUORUM | ((1u << x->r) << 16);
  } else {
    raise_flag(x, PAXISIM_F_WOVF | PAXISIM_F_UNFAITHFUL);  /* request lost */
  }
  if (s->cfg.thrifty) multicast_quorum1(x, s->N / 2 + 1, PAXISIM_MSG_P2A | x->ktag, p->ballot, (uint32_t)p->slot, REQ_CID(req));
  else broadcast1(x, PAXISIM_MSG_P2A | x->ktag, p->ballot, (uint32_t)p->slot, REQ_CID(req));
}

static void paxos_handle_request(ctx_t* x, uint32_t req) { /* paxos.go:86-97 */
  inst_t* p = x->p;
  if (!p->active) {
    if (p->npend == PMAX) raise_flag(x, PAXISIM_F_PEND_OVF | PAXISIM_F_UNFAITHFUL);
    else p->pend[p->npend++] = req;
    if (bal_id(p->ballot) != x->r) paxos_p1a(x);
  } else {
    paxos_p2a(x, req);
  }
}

/* Replica.handleRequest (paxos/replica.go:42-66; read modes out of scope). */
static void replica_handle_request(ctx_t* x, uint32_t req) {
  if (x->s->cfg.ephemeral_leader || is_leader(x) || x->p->ballot == 0)
    paxos_handle_request(x, req);
  else
    node_forward(x, bal_id(x->p->ballot), req);            /* `go r.Forward(...)` */
}

static void paxos_exec(ctx_t* x);
static void agree_arrive(ctx_t* x, uint32_t k);
static inline uint32_t wl_key(const struct oracle_sim* s, uint32_t kc, uint32_t cid);
static inline uint32_t key_fit(ctx_t* x, uint32_t k);
static inline int wl_write(const struct oracle_sim* s, uint32_t kc, uint32_t cid);

static void paxos_handle_p1a(ctx_t* x, uint32_t mb) {      /* paxos.go:134-162 */
  inst_t* p = x->p;
  rec_t out[1 + PAXISIM_MAX_WINDOW];
  uint32_t n = 0;
  int32_t s, hi;
  if (mb > p->ballot) {
    p->ballot = mb;
    p->active = 0;
    paxos_forward(x);
  }
  if (x->p->iflags & PAXISIM_F_WOVF) raise_flag(x, PAXISIM_F_UNFAITHFUL);  /* Go may hold skipped entries */
  hi = p->slot;
  if (hi > p->execute + (int32_t)x->s->W - 1) hi = p->execute + (int32_t)x->s->W - 1;
  for (s = p->execute; s <= hi; s++) {
    entry_t* e = log_at(x, s);
    if (!(e->meta & E_EXISTS) || (e->meta & E_COMMIT)) continue;
    n++;
    out[n].hdr = HDR(PAXISIM_MSG_P1B_ENTRY, 0);
    out[n].ballot = e->ballot;
    out[n].slot = (uint32_t)s;
    out[n].cid = e->cmd;
  }
  out[0].hdr = HDR(PAXISIM_MSG_P1B, n) | x->ktag;
  out[0].ballot = p->ballot;
  out[0].slot = 0;
  out[0].cid = 0;
  sock_send(x, bal_id(mb), out, 1 + n);
}

static void paxos_update(ctx_t* x, const rec_t* log, uint32_t n) { /* paxos.go:164-180 */
  inst_t* p = x->p;
  uint32_t i;
  for (i = 0; i < n; i++) {
    int32_t s = (int32_t)log[i].slot;
    if (s > p->slot) p->slot = s;
    if (in_window(x, s)) {
      entry_t* e = log_at(x, s);
      if (e->meta & E_EXISTS) {
        if (!(e->meta & E_COMMIT) && log[i].ballot > e->ballot) {
          e->ballot = log[i].ballot;
          e->cmd = log[i].cid;
        }
      } else {
        e->ballot = log[i].ballot;
        e->cmd = log[i].cid;
        e->req = 0;
        e->meta = E_EXISTS;                                /* quorum nil */
      }
    } else if (s < p->execute) {
      ghost(x, s, log[i].ballot);
    } else {
      raise_flag(x, PAXISIM_F_WOVF);
    }
  }
}

static void paxos_handle_p1b(ctx_t* x, uint32_t src, uint32_t mb, const rec_t* log, uint32_t n) { /* paxos.go:183-230 */
  inst_t* p = x->p;
  if (mb < p->ballot || p->active) return;
  paxos_update(x, log, n);
  if (mb > p->ballot) {
    p->ballot = mb;
    p->active = 0;
    paxos_forward(x);
  }
  if (bal_id(mb) == x->r && mb == p->ballot) {
    p->p1mask |= 1u << src;
    if (q1_ok(x, p->p1mask)) {
      int32_t i, hi;
      uint32_t k, npend;
      uint32_t pend[PMAX];
      p->active = 1;
      if (x->p->iflags & PAXISIM_F_WOVF) raise_flag(x, PAXISIM_F_UNFAITHFUL);
      hi = p->slot;
      if (hi > p->execute + (int32_t)x->s->W - 1) hi = p->execute + (int32_t)x->s->W - 1;
      for (i = p->execute; i <= hi; i++) {
        entry_t* e = log_at(x, i);
        if (!(e->meta & E_EXISTS) || (e->meta & E_COMMIT)) continue;   /* nil gap skipped (G5) */
        e->ballot = p->ballot;
        e->meta = (e->meta & (E_EXISTS | E_COMMIT)) | E_QUORUM | ((1u << x->r) << 16);
        broadcast1(x, PAXISIM_MSG_P2A | x->ktag, p->ballot, (uint32_t)i, e->cmd);
      }
      npend = p->npend;
      memcpy(pend, p->pend, npend * sizeof(uint32_t));
      p->npend = 0;
      for (k = 0; k < npend; k++) paxos_p2a(x, pend[k]);
    }
  }
}

static void paxos_handle_p2a(ctx_t* x, uint32_t mb, int32_t ms, uint32_t mcid) { /* paxos.go:233-267 */
  inst_t* p = x->p;
  if (mb >= p->ballot) {
    p->ballot = mb;
    p->active = 0;
    if (ms > p->slot) p->slot = ms;
    if (in_window(x, ms)) {
      entry_t* e = log_at(x, ms);
      if (e->meta & E_EXISTS) {
        if (!(e->meta & E_COMMIT) && mb > e->ballot) {
          if (e->cmd != mcid && e->req) {
            node_forward(x, bal_id(mb), e->req);
            e->req = 0;
          }
          e->cmd = mcid;
          e->ballot = mb;
        }
      } else {
        e->ballot = mb;
        e->cmd = mcid;
        e->req = 0;
        e->meta = E_EXISTS;
      }
    } else if (ms < p->execute) {
      ghost(x, ms, mb);
    } else {
      raise_flag(x, PAXISIM_F_WOVF);
    }
  }
  send1(x, bal_id(mb), PAXISIM_MSG_P2B | x->ktag, p->ballot, (uint32_t)ms, 0);
}

static void paxos_handle_p2b(ctx_t* x, uint32_t src, uint32_t mb, int32_t ms) { /* paxos.go:270-310 */
  inst_t* p = x->p;
  entry_t* e;
  if (!in_window(x, ms)) {
    if (ms < p->execute) ghost_p2b(x, ms, mb);
    else if (x->p->iflags & PAXISIM_F_WOVF) raise_flag(x, PAXISIM_F_UNFAITHFUL);
    return;
  }
  e = log_at(x, ms);
  if (!(e->meta & E_EXISTS) || mb < e->ballot || (e->meta & E_COMMIT)) return;
  if (mb > p->ballot) {
    p->ballot = mb;
    p->active = 0;
  }
  if (bal_id(mb) == x->r && mb == e->ballot) {
    if (!(e->meta & E_QUORUM)) {                           /* nil quorum: Go panics */
      raise_flag(x, PAXISIM_F_POISON);
      x->stop = 1;
      return;
    }
    e->meta |= (1u << src) << 16;
    if (q2_ok(x, E_ACK(e->meta))) {
      e->meta |= E_COMMIT;
      x->n->commits++;
      broadcast1(x, PAXISIM_MSG_P3 | x->ktag, mb, (uint32_t)ms, e->cmd);
      if (x->s->cfg.reply_when_commit) {
        if (!e->req) { raise_flag(x, PAXISIM_F_POISON); x->stop = 1; return; } /* nil r.Reply */
        request_reply(x, e->req, REQ_CID(e->req), 0);      /* Reply{Command: r.Command}: no Value */
      } else {
        paxos_exec(x);
      }
    }
  }
}

static void paxos_handle_p3(ctx_t* x, uint32_t mb, int32_t ms, uint32_t mcid) { /* paxos.go:313-343 */
  inst_t* p = x->p;
  if (ms > p->slot) p->slot = ms;
  if (in_window(x, ms)) {
    entry_t* e = log_at(x, ms);
    if (e->meta & E_EXISTS) {
      if (e->cmd != mcid && e->req) {
        node_forward(x, bal_id(mb), e->req);
        e->req = 0;
      }
    } else {
      e->ballot = 0;                                       /* &entry{} (G6) */
      e->req = 0;
      e->meta = E_EXISTS;
    }
    e->cmd = mcid;
    e->meta |= E_COMMIT;
    if (x->s->cfg.reply_when_commit) {
      if (e->req) request_reply(x, e->req, REQ_CID(e->req), 0);
      return;
    }
  } else if (ms < p->execute) {
    ghost_commit(x, ms);
  } else {
    raise_flag(x, PAXISIM_F_WOVF);
  }
  if (!x->s->cfg.reply_when_commit) paxos_exec(x);
}

/* Agreement as a running check (client.go:279-320 Consensus: per index the
 * executed values form a set of size <= 1): the first replica to reach digest
 * checkpoint k (every CKI executed slots) records it in the cluster's ring,
 * every later one compares.  Replicas run one after another within a step, so
 * arrivals apply in replica index order, then arrival order - the order the
 * device drains its per-step arrival lists in (sim_core.h agree_drain).  A
 * replica's arrivals beyond AGMAX in one step count as missed (up to the
 * device's 8-bit count of 255). */
#define AGMAX 8
static void agree_arrive(ctx_t* x, uint32_t k) {
  const uint32_t key = (uint32_t)(x->p - x->n->inst);
  uint64_t* a = &x->c->agr[(size_t)key * x->s->AR + k % x->s->AR];
  const uint64_t d = x->p->digest;
  const uint64_t want = ((uint64_t)k << 40) | ((d ^ (d >> 24)) & 0xFFFFFFFFFFull);
  const uint32_t tv = (uint32_t)(*a >> 40);
  const uint32_t i = x->n->nag++;
  if (i >= AGMAX) {
    if (i < 255) x->n->agm++;
    return;
  }
  if (*a == 0 || tv < k) { *a = want; return; }
  if (tv > k) { x->n->agm++; return; }                      /* the first digest has left the ring */
  x->n->agc++;
  if (*a != want) x->n->agb++;
}

/* The key of an executed command when replicas keep the Database: a per-key
 * instance (WPaxos, M2Paxos, KPaxos) executes only commands of its own key;
 * otherwise the workload's key, fitted to the key space. */
static uint32_t exec_key(ctx_t* x, uint32_t cmd) {
  if (!x->s->kv) return 0u;
  if (x->s->cfg.protocol == PAXISIM_WPAXOS) return x->ktag >> 16;
  return key_fit(x, wl_key(x->s, x->c->kc, cmd));
}

/* Database.Execute's return value (db.go:103-114): the key's value before the
 * command (0 = nil), the Reply.Value of an executed request. */
static uint32_t kv_get(ctx_t* x, uint32_t key) {
  return x->s->kv ? x->n->db[key] : 0u;
}

/* Database.Execute (db.go:103-114) when replicas keep the KV: a write's value
 * (its command id) goes to its key, database.version counts it (put,
 * db.go:123-134); a read changes nothing. */
static void kv_exec(ctx_t* x, uint32_t key, uint32_t cmd) {
  if (!x->s->kv || !wl_write(x->s, x->c->kc, cmd)) return;
  x->n->db[key] = cmd;
  x->n->db_version++;
}

static void paxos_exec(ctx_t* x) {                         /* paxos.go:345-369 */
  inst_t* p = x->p;
  for (;;) {
    entry_t* e = log_at(x, p->execute);
    if (!(e->meta & E_EXISTS) || !(e->meta & E_COMMIT)) break;
    if (x->p->iflags & PAXISIM_F_WOVF) raise_flag(x, PAXISIM_F_UNFAITHFUL);
    const uint32_t key = exec_key(x, e->cmd);
    if (e->req) {                                          /* Reply{Value: p.Execute(...)}: the previous value */
      request_reply(x, e->req, e->cmd, kv_get(x, key));
      e->req = 0;
    }
    p->digest = mix64(p->digest ^ (((uint64_t)(uint32_t)p->execute << 32) | e->cmd));
    kv_exec(x, key, e->cmd);                               /* p.Execute(e.command), paxos.go:352 */
    if (x->s->keep_xlog) {
      if (p->nx == p->capx) {
        p->capx = p->capx ? 2 * p->capx : 1024;
        p->xlog = (uint32_t*)realloc(p->xlog, p->capx * sizeof(uint32_t));
      }
      p->xlog[p->nx++] = e->cmd;
    }
    e->meta = 0;                                           /* delete(p.log, p.execute) */
    p->execute++;
    if ((uint32_t)p->execute % CKI == 0) {
      uint32_t k = ((uint32_t)p->execute / CKI) % CKR;
      p->ck_e[k] = (uint32_t)p->execute;
      p->ck_d[k] = p->digest;
      if (x->s->AR) agree_arrive(x, (uint32_t)p->execute / CKI);
    }
  }
}

/* node.handle dispatch (node.go:104-115) for one inbound message. */
static void paxos_dispatch(ctx_t* x, uint32_t src, const rec_t* m) {
  switch (HDR_TYPE(m->hdr)) {
    case PAXISIM_MSG_REQUEST:
      replica_handle_request(x, REQ(m->cid, src == x->s->N ? PAXISIM_CLIENT_SRC : src));
      break;
    case PAXISIM_MSG_REPLY: handle_reply(x, m->cid, m->ballot); break;
    case PAXISIM_MSG_P1A: paxos_handle_p1a(x, m->ballot); break;
    case PAXISIM_MSG_P1B: paxos_handle_p1b(x, src, m->ballot, m + 1, HDR_N(m->hdr)); break;
    case PAXISIM_MSG_P2A: paxos_handle_p2a(x, m->ballot, (int32_t)m->slot, m->cid); break;
    case PAXISIM_MSG_P2B: paxos_handle_p2b(x, src, m->ballot, (int32_t)m->slot); break;
    case PAXISIM_MSG_P3: paxos_handle_p3(x, m->ballot, (int32_t)m->slot, m->cid); break;
    default: break;
  }
}

/* ------------------------------------------------------------------------ */
/* Workload: key and read/write of command cid (benchmark.go:202-275)        */
/* ------------------------------------------------------------------------ */
static inline uint32_t wl_hash(uint32_t kc, uint32_t cid) { return fmix32(fmix32(kc ^ 0x5BD1E995u) ^ cid); }
/* Key of command cid.  With locality (the WPaxos per-zone clients, each
 * drawing from its zone's keys: benchmark.go:202-213 "conflict"/Min), worker
 * w's command is, with P = locality, one of the keys k = z (mod Z) of the zone
 * z of the replica it sends to, otherwise uniform over all keys. */
static inline uint32_t wl_key(const struct oracle_sim* s, uint32_t kc, uint32_t cid) {
  const uint32_t h = wl_hash(kc, cid), K = s->cfg.keys;
  const uint32_t KS = s->wl.key_space ? s->wl.key_space : K;   /* Bconfig.K of order/uniform/conflict */
  if (s->wl.locality_ppm) {
    const uint32_t w = (cid - 1u) % s->wl.outstanding;
    const uint32_t z = s->zone_of[s->wl.target[w]] - 1u, Z = s->Z;
    const uint32_t nk = z < K ? (K - z + Z - 1u) / Z : 0u;
    if (nk && ppm_hit(fmix32(h ^ 0x165667B1u), s->wl.locality_ppm)) return z + Z * (h % nk);
  }
  /* Bconfig.Distribution (benchmark.go:202-233) as a function of cid:
   * "order" counter+1 mod K with the counter = cid (205-207); "conflict" the
   * literal key 0 with rand.Intn(100) < Conflicts (213-214: no Min added, so
   * with Min != 0 it is a key of its own, index KS), else order (216-217);
   * "normal", "zipfan", "exponential" (221-233) by inverse CDF over the
   * caller's table.  A draw at or above key_tail lies beyond the key space
   * (Go's "exponential" is unbounded): index K, flagged by key_fit.  With
   * Bconfig.Move (137-140) Mu steps once per move_every issued commands: cid
   * draws from table (cid-1)/move_every of the Mu sequence. */
  switch (s->wl.distribution) {
    case PAXISIM_DIST_ORDER: return cid % KS;
    case PAXISIM_DIST_CONFLICT:
      return fmix32(h ^ 0x3C6EF372u) % 100u < s->wl.conflicts ? (s->wl.key_min ? KS : 0u) : cid % KS;
    case PAXISIM_DIST_TABLE: {
      const uint32_t u = fmix32(h ^ 0x2545F491u);
      const uint32_t* cdf = s->wl.key_cdf;
      uint32_t k = 0, i;
      if (s->wl.move_every) {
        uint32_t e = (cid - 1u) / s->wl.move_every;
        if (e >= s->wl.move_tables) e = s->wl.move_loop + (e - s->wl.move_loop) % (s->wl.move_tables - s->wl.move_loop);
        cdf = s->move_cdf + (size_t)e * PAXISIM_MAX_KEYS;
      } else if (s->wl.key_tail && u >= s->wl.key_tail) {
        return K;
      }
      for (i = 0; i + 1u < K; i++) k += u >= cdf[i] ? 1u : 0u;
      return k;
    }
    default: return h % KS;
  }
}
/* The key value the reference's Database sees for index k (paxisim.h): Min +
 * k for order/uniform/conflict, k itself for the table distributions (Go adds
 * no Min), 0 for conflict's literal key. */
static inline uint32_t key_value(const struct oracle_sim* s, uint32_t k) {
  if (s->wl.distribution == PAXISIM_DIST_TABLE) return k;
  if (s->wl.distribution == PAXISIM_DIST_CONFLICT && s->wl.key_min &&
      k == (s->wl.key_space ? s->wl.key_space : s->cfg.keys))
    return 0u;
  return s->wl.key_min + k;
}
/* A key the replica uses: a draw beyond the key space has no state here (in Go
 * it would be a new map entry), so the replica raises UNFAITHFUL and uses the
 * last index. */
static inline uint32_t key_fit(ctx_t* x, uint32_t k) {
  if (k >= x->s->cfg.keys) {
    raise_flag(x, PAXISIM_F_UNFAITHFUL);
    k = x->s->cfg.keys - 1u;
  }
  return k;
}
static inline int wl_write(const struct oracle_sim* s, uint32_t kc, uint32_t cid) {
  return ppm_hit(fmix32(wl_hash(kc, cid) ^ 0x27D4EB2Fu), s->wl.write_ppm);
}

/* ------------------------------------------------------------------------ */
/* WPaxos (wpaxos/replica.go, wpaxos/kpaxos.go): one Paxos instance per key, */
/* Q1/Q2 = GridRow/GridColumn (fz = 0) or FGridQ1/Q2(fz) (kpaxos.go:15-27),  */
/* consecutive leader-migration policy.  The kpaxos Broadcast/Send wrappers  */
/* (kpaxos.go:51-74) tag P1a..P3 with the key: x->ktag.                      */
/* ------------------------------------------------------------------------ */
#define POL_NONE 0xFFu                                     /* ID "" */
static inline void wp_bind(ctx_t* x, uint32_t key) {
  x->p = &x->n->inst[key];
  x->ktag = key << 16;
}
static inline void wp_init(ctx_t* x, uint32_t key) {       /* Replica.init replica.go:36-40 */
  wp_bind(x, key);
  if (!x->p->exists) x->p->pol_time = x->t;                /* newKPaxos -> NewPolicy: time.Now() */
  x->p->exists = 1;
}
/* r.paxi[m.Key] without init: a nil *kpaxos, whose use panics in Go */
static inline int wp_get(ctx_t* x, uint32_t key) {
  wp_bind(x, key);
  if (x->p->exists) return 1;
  raise_flag(x, PAXISIM_F_POISON);
  x->stop = 1;
  return 0;
}

/* majority.Hit (policy.go:79-93) with the step as the clock: an id holding
 * at least sum/2 of the hits once `policy_interval` steps have passed since the
 * last reset.  Go ranges over a map (random order) and keeps the last id that
 * qualifies; here ids are visited in index order, so the highest index wins. */
static uint32_t majority_hit(ctx_t* x, uint32_t id) {
  inst_t* p = x->p;
  const struct oracle_sim* s = x->s;
  uint32_t res = POL_NONE, i;
  if (p->pol_n[id] < 0xFFFFu) p->pol_n[id]++;              /* counters saturate at 16 bits */
  p->pol_sum++;
  if (p->pol_sum > 1 && x->t - p->pol_time >= s->cfg.policy_interval) {
    for (i = 0; i < s->N; i++)
      if (p->pol_n[i] >= p->pol_sum / 2) res = i;
    for (i = 0; i < s->N; i++) p->pol_n[i] = 0;            /* reset (policy.go:95-101) */
    p->pol_sum = 0;
    p->pol_time = x->t;
  }
  return res;
}

/* ema.Hit (policy.go:111-130): s = alpha*zone + (1-alpha)*s, each operation
 * rounded separately (no fused multiply-add); a settled s (within epsilon
 * 0.1 of an integer) naming a new zone z returns NewID(z, 1). */
static uint32_t ema_hit(ctx_t* x, uint32_t id) {
  inst_t* p = x->p;
  const struct oracle_sim* s = x->s;
  const double a = s->cfg.policy_alpha, zid = (double)s->zone_of[id];
  volatile double t1, t2, t3;                              /* keep every product rounded */
  int32_t z;
  uint32_t r = 0, k;
  if (p->pol_s == 0.0) {
    p->pol_s = zid;
    return POL_NONE;
  }
  t1 = a * zid;
  t2 = 1.0 - a;
  t3 = t2 * p->pol_s;
  p->pol_s = t1 + t3;
  if (fabs(p->pol_s - round(p->pol_s)) > 0.1) return POL_NONE;
  z = (int32_t)round(p->pol_s);
  if ((uint32_t)z == p->pol_zone) return POL_NONE;
  p->pol_zone = (uint32_t)z;
  for (k = 0; k + 1u < (uint32_t)z; k++) r += s->cfg.npz[k]; /* index of ID z.1 */
  return r;
}

/* consecutive.Hit (policy.go:55-69); threshold 0 is the null policy (policy.go:18-21) */
static uint32_t policy_hit(ctx_t* x, uint32_t id) {
  inst_t* p = x->p;
  uint32_t res = POL_NONE;
  if (x->s->cfg.policy == PAXISIM_POLICY_MAJORITY) return majority_hit(x, id);
  if (x->s->cfg.policy == PAXISIM_POLICY_EMA) return ema_hit(x, id);
  if (x->s->cfg.policy_threshold == 0) return POL_NONE;
  if (id == p->pol_last) {
    p->pol_hits++;
  } else {
    p->pol_last = id;
    p->pol_hits = 1;
  }
  if (p->pol_hits >= x->s->cfg.policy_threshold) {
    res = p->pol_last;
    p->pol_last = POL_NONE;
    p->pol_hits = 0;
  }
  return res;
}

/* KPaxos index() (kpaxos/replica.go:32-44): leader "z.1", z = 1 + key/200 (at
 * most 5); an ID outside the configuration is an unknown address. */
static uint32_t kp_leader(const struct oracle_sim* s, uint32_t key) {
  const uint32_t z = key < 800u ? key / 200u : 4u;
  return z < s->Z ? s->zfirst[z] : NO_ID;
}

static void wp_handle_request(ctx_t* x, uint32_t req) {   /* replica.go:42-66 */
  const struct oracle_sim* s = x->s;
  const uint32_t key = key_fit(x, wl_key(s, x->c->kc, REQ_CID(req)));
  wp_init(x, key);
  if (s->variant == PAXISIM_KPAXOS) {                      /* kpaxos/replica.go:52-62 */
    const uint32_t leader = kp_leader(s, key_value(s, key));
    if (leader == x->r) paxos_handle_request(x, req);
    else node_forward(x, leader, req);                     /* `go r.Forward(leader, m)` */
    return;
  }
  if (!s->cfg.adaptive) {
    paxos_handle_request(x, req);
    return;
  }
  if (is_leader(x) || x->p->ballot == 0) {
    const uint32_t o = REQ_ORIGIN(req);
    uint32_t to;
    paxos_handle_request(x, req);
    /* m.NodeID: the receiving node for an HTTP request (http.go:96), the forwarder otherwise (node.go:167) */
    to = policy_hit(x, o == PAXISIM_CLIENT_SRC ? x->r : o);
    if (to != POL_NONE && s->zone_of[to] != s->zone_of[x->r])
      send1(x, to, PAXISIM_MSG_LEADERCHG | x->ktag, x->p->ballot, to, x->r);   /* LeaderChange{Key,To,From,Ballot} */
  } else {
    node_forward(x, bal_id(x->p->ballot), req);            /* `go r.Forward(p.Leader(), m)` */
  }
}

static void wp_handle_leader_change(ctx_t* x, uint32_t key, uint32_t mb, uint32_t to) { /* replica.go:101-108 */
  if (!wp_get(x, key)) return;
  if (mb == x->p->ballot && to == x->r) paxos_p1a(x);
}

static void wpaxos_dispatch(ctx_t* x, uint32_t src, const rec_t* m) {   /* registrations replica.go:25-32 */
  const uint32_t key = HDR_KEY(m->hdr);
  switch (HDR_TYPE(m->hdr)) {
    case PAXISIM_MSG_REQUEST:
      wp_handle_request(x, REQ(m->cid, src == x->s->N ? PAXISIM_CLIENT_SRC : src));
      break;
    case PAXISIM_MSG_REPLY: handle_reply(x, m->cid, m->ballot); break;
    case PAXISIM_MSG_P1A: wp_init(x, key); paxos_handle_p1a(x, m->ballot); break;          /* handlePrepare 72-76 */
    case PAXISIM_MSG_P1B:                                                                  /* handlePromise 78-82 */
      if (wp_get(x, key)) paxos_handle_p1b(x, src, m->ballot, m + 1, HDR_N(m->hdr));
      break;
    case PAXISIM_MSG_P2A: wp_init(x, key); paxos_handle_p2a(x, m->ballot, (int32_t)m->slot, m->cid); break; /* 84-88 */
    case PAXISIM_MSG_P2B: if (wp_get(x, key)) paxos_handle_p2b(x, src, m->ballot, (int32_t)m->slot); break; /* 90-93 */
    case PAXISIM_MSG_P3: wp_init(x, key); paxos_handle_p3(x, m->ballot, (int32_t)m->slot, m->cid); break;   /* 95-99 */
    case PAXISIM_MSG_LEADERCHG: wp_handle_leader_change(x, key, m->ballot, m->slot); break;
    default: break;
  }
}

/* ------------------------------------------------------------------------ */
/* EPaxos (epaxos/replica.go, epaxos/instance.go)                            */
/* Leaderless: a replica leads the instances of its own log.  Instance (o, s)*/
/* of owner o lives in a ring of W over slots (executed[o], executed[o] + W];*/
/* slots at or below executed[o] are COMMITTED for good (execute() only      */
/* advances over committed instances, and no handler changes one after it);  */
/* a message for a slot beyond the ring cannot be held: WOVF | UNFAITHFUL.   */
/* Records: PreAccept {hdr, ballot, slot, cmd} + (seq, Dep[N]);              */
/* PreAcceptReply {hdr, ballot, slot, seq} + (Dep[N], Committed[N]);        */
/* Accept {hdr, ballot, slot, seq} + Dep[N]; AcceptReply {hdr, ballot, slot};*/
/* Commit {hdr, ballot, slot, cmd} + (seq, Dep[N]).  The owner of an        */
/* instance is the sender of PreAccept/Accept/Commit (only it sends them).  */
/* Ballots are NewBallot(0, owner) only (replica.go:77): stored as 1 + owner.*/
/* ------------------------------------------------------------------------ */
enum { EP_NONE = 0, EP_PREACCEPTED = 1, EP_ACCEPTED = 2, EP_COMMITTED = 3 };

static inline uint32_t ep_words_rec(uint32_t words) { return (words + 3u) / 4u; }
static ep_inst_t* ep_ring(ctx_t* x, uint32_t o, int32_t s) {
  return &x->n->ep_log[(size_t)o * x->s->W + ((uint32_t)s & (x->s->W - 1u))];
}
/* the ring entry holds instance s (an entry keeps its data after execute()
 * passes it, as Go keeps the instance, until a later slot takes the entry) */
static inline int ep_live(const ep_inst_t* i, int32_t s) { return i->exists && i->slot == s; }
static inline void ep_new(ep_inst_t* i, int32_t s) { memset(i, 0, sizeof *i); i->exists = 1; i->slot = s; }
/* 1: in the ring (*out), 0: at or below executed (COMMITTED), 2: beyond the ring */
static int ep_where(ctx_t* x, uint32_t o, int32_t s, ep_inst_t** out) {
  const int32_t ex = x->n->ep_executed[o];
  if (s <= ex) return 0;
  if (s > ex + (int32_t)x->s->W) return 2;
  *out = ep_ring(x, o, s);
  return 1;
}
static inline int32_t* ep_cf(ctx_t* x, uint32_t o, uint32_t key) {       /* {slot (-1 none), seq} */
  return &x->n->ep_cf[((size_t)o * x->s->cfg.keys + key) * 2u];
}
static inline uint32_t ep_key(ctx_t* x, uint32_t cmd) { return key_fit(x, wl_key(x->s, x->c->kc, cmd)); }

/* the current seq of instance (o, d), the slot conflicts[o][key] names */
static int32_t ep_seq_of(ctx_t* x, uint32_t o, int32_t d, uint32_t key) {
  ep_inst_t* i;
  if (ep_where(x, o, d, &i) == 1 && ep_live(i, d)) return i->seq;
  return ep_cf(x, o, key)[1];                              /* left the ring with this seq */
}

/* attributes (replica.go:58-80) */
static void ep_attributes(ctx_t* x, uint32_t key, int32_t* seq_out, int32_t* dep) {
  const struct oracle_sim* s = x->s;
  int32_t seq = 0;
  uint32_t id;
  for (id = 0; id < s->N; id++) dep[id] = 0;
  for (id = 0; id < s->N; id++) {                          /* Go ranges over a map: max, order-free */
    const int32_t* cf = ep_cf(x, id, key);
    if (cf[0] >= 0 && cf[0] > dep[id]) {
      const int32_t sd = ep_seq_of(x, id, cf[0], key);
      dep[id] = cf[0];
      if (seq <= sd) seq = sd + 1;
    }
  }
  if (x->n->ep_maxseq[key] >= 0 && seq <= x->n->ep_maxseq[key]) seq = x->n->ep_maxseq[key] + 1;
  *seq_out = seq;
}

/* update (replica.go:83-101) */
static void ep_update(ctx_t* x, uint32_t cmd, uint32_t id, int32_t slot, int32_t seq) {
  const uint32_t k = ep_key(x, cmd);
  int32_t* cf = ep_cf(x, id, k);
  if (cf[0] < 0 || cf[0] < slot) { cf[0] = slot; cf[1] = seq; }
  if (x->n->ep_maxseq[k] < seq) x->n->ep_maxseq[k] = seq;    /* -1 = absent */
}

static void ep_send(ctx_t* x, uint32_t to, uint32_t type, uint32_t w1, uint32_t w2, uint32_t w3,
                    const uint32_t* pay, uint32_t npay) {
  rec_t m[1 + (2 * PAXISIM_MAX_N + 3) / 4];
  const uint32_t n = ep_words_rec(npay);
  uint32_t k;
  memset(m, 0, sizeof m);
  m[0].hdr = HDR(type, n); m[0].ballot = w1; m[0].slot = w2; m[0].cid = w3;
  for (k = 0; k < npay; k++) ((uint32_t*)&m[1])[k] = pay[k];
  sock_send(x, to, m, 1u + n);
}
static void ep_broadcast(ctx_t* x, uint32_t type, uint32_t w1, uint32_t w2, uint32_t w3, const uint32_t* pay,
                         uint32_t npay) {
  uint32_t d;
  for (d = 0; d < x->s->N; d++)
    if (d != x->r) ep_send(x, d, type, w1, w2, w3, pay, npay);
}

static void ep_reply(ctx_t* x, ep_inst_t* i, uint32_t value) { /* i.request.Reply (message.go:32-34) */
  /* req.c is buffered 1 (http.go:97): the HTTP handler takes the first reply,
   * the second waits in the buffer, a third would block this goroutine */
  if (++i->nrep >= 3) raise_flag(x, PAXISIM_F_UNFAITHFUL);
  request_reply(x, i->req, i->cmd, value);
}

/* execute (replica.go:355-384): owners in index order where Go ranges over a map */
static void ep_execute(ctx_t* x) {
  const struct oracle_sim* s = x->s;
  replica_t* p = x->n;
  uint32_t id;
  for (id = 0; id < s->N; id++) {
    int32_t sl;
    for (sl = p->ep_executed[id] + 1; sl <= p->ep_slot[id]; sl++) {
      ep_inst_t* i = NULL;
      const int w = ep_where(x, id, sl, &i);
      if (w == 2) { raise_flag(x, PAXISIM_F_WOVF | PAXISIM_F_UNFAITHFUL); continue; }
      if (!ep_live(i, sl)) continue;                       /* nil: skipped, not executed */
      if (i->status != EP_COMMITTED) break;
      p->inst[0].digest = mix64(p->inst[0].digest ^ (((uint64_t)((id << 24) | (uint32_t)sl) << 32) | i->cmd));
      p->ep_execs++;
      {
        const uint32_t key = exec_key(x, i->cmd);
        const uint32_t v = kv_get(x, key);                  /* v := r.Execute(i.cmd), replica.go:373 */
        kv_exec(x, key, i->cmd);
        if (i->req) ep_reply(x, i, v);
      }
      if (s->keep_xlog) {
        inst_t* q = &p->inst[0];
        if (q->nx == q->capx) {
          q->capx = q->capx ? 2 * q->capx : 1024;
          q->xlog = (uint32_t*)realloc(q->xlog, q->capx * sizeof(uint32_t));
        }
        q->xlog[q->nx++] = i->cmd;
      }
      if (sl == p->ep_executed[id] + 1) {
        const uint32_t k = ep_key(x, i->cmd);
        int32_t* cf = ep_cf(x, id, k);
        if (cf[0] == sl) cf[1] = i->seq;                   /* it leaves the ring with this seq */
        p->ep_executed[id] = sl;
      }
    }
  }
}

/* updateCommit (replica.go:103-111) */
static void ep_update_commit(ctx_t* x, uint32_t id) {
  replica_t* p = x->n;
  for (;;) {
    ep_inst_t* i = NULL;
    const int32_t nx = p->ep_committed[id] + 1;
    const int w = ep_where(x, id, nx, &i);
    if (w == 2) {
      if (nx <= p->ep_slot[id]) raise_flag(x, PAXISIM_F_WOVF | PAXISIM_F_UNFAITHFUL);
      break;
    }
    if (w == 1 && !(ep_live(i, nx) && i->status == EP_COMMITTED)) break;
    p->ep_committed[id] = nx;                              /* w == 0: committed for good */
  }
  ep_execute(x);
}

static void ep_handle_request(ctx_t* x, uint32_t req) {    /* replica.go:113-145 */
  replica_t* p = x->n;
  const uint32_t self = x->r, cmd = REQ_CID(req), key = ep_key(x, cmd);
  int32_t seq, dep[PAXISIM_MAX_N], s;
  ep_inst_t* i = NULL;
  uint32_t pay[1 + PAXISIM_MAX_N], k;
  p->ep_slot[self]++;
  s = p->ep_slot[self];
  ep_attributes(x, key, &seq, dep);
  if (ep_where(x, self, s, &i) != 1) { raise_flag(x, PAXISIM_F_WOVF | PAXISIM_F_UNFAITHFUL); return; }
  ep_new(i, s);
  i->cmd = cmd; i->ballot = (uint8_t)(1u + self); i->status = EP_PREACCEPTED;
  i->seq = seq; memcpy(i->dep, dep, sizeof dep); i->req = req;
  i->acks = 1u << self;                                    /* self ack */
  ep_update(x, cmd, self, s, seq);
  pay[0] = (uint32_t)seq;
  for (k = 0; k < x->s->N; k++) pay[1 + k] = (uint32_t)dep[k];
  ep_broadcast(x, PAXISIM_MSG_PREACCEPT, i->ballot, (uint32_t)s, cmd, pay, 1u + x->s->N);
}

static void ep_handle_preaccept(ctx_t* x, uint32_t o, const rec_t* m) {   /* replica.go:147-191 */
  replica_t* p = x->n;
  const uint32_t* pw = (const uint32_t*)(m + 1);
  const int32_t s = (int32_t)m->slot;
  const uint32_t mb = m->ballot, mcmd = m->cid;
  int32_t seq, dep[PAXISIM_MAX_N];
  ep_inst_t* i = NULL;
  uint32_t pay[2 * PAXISIM_MAX_N], k;
  const int w = ep_where(x, o, s, &i);
  if (w == 0) return;                                      /* COMMITTED, cmd set: no reply */
  if (w == 2) { raise_flag(x, PAXISIM_F_WOVF | PAXISIM_F_UNFAITHFUL); return; }
  if (!ep_live(i, s)) ep_new(i, s);                         /* &instance{} */
  if (i->status == EP_COMMITTED || i->status == EP_ACCEPTED) {
    if (!i->cmd) { i->cmd = mcmd; ep_update(x, mcmd, o, s, (int32_t)pw[0]); }
    return;
  }
  if (s > p->ep_slot[o]) p->ep_slot[o] = s;
  ep_attributes(x, ep_key(x, mcmd), &seq, dep);
  if (mb >= i->ballot) {
    i->ballot = (uint8_t)mb; i->cmd = mcmd; i->status = EP_PREACCEPTED; i->seq = seq;
    memcpy(i->dep, dep, sizeof dep);
  }
  ep_update(x, mcmd, o, s, seq);
  for (k = 0; k < x->s->N; k++) {
    pay[k] = (uint32_t)i->dep[k];
    pay[x->s->N + k] = (uint32_t)p->ep_committed[k];
  }
  ep_send(x, o, PAXISIM_MSG_PREACCEPTREPLY, i->ballot, (uint32_t)s, (uint32_t)seq, pay, 2u * x->s->N);
}

static void ep_commit_broadcast(ctx_t* x, ep_inst_t* i, int32_t s) {
  uint32_t pay[1 + PAXISIM_MAX_N], k;
  pay[0] = (uint32_t)i->seq;
  for (k = 0; k < x->s->N; k++) pay[1 + k] = (uint32_t)i->dep[k];
  ep_broadcast(x, PAXISIM_MSG_COMMIT, i->ballot, (uint32_t)s, i->cmd, pay, 1u + x->s->N);
}

static void ep_handle_preaccept_reply(ctx_t* x, uint32_t src, const rec_t* m) {   /* replica.go:193-260 */
  const struct oracle_sim* s = x->s;
  replica_t* p = x->n;
  const uint32_t* pw = (const uint32_t*)(m + 1);
  const int32_t sl = (int32_t)m->slot;
  ep_inst_t* i = NULL;
  int committed = 1;
  uint32_t id;
  if (ep_where(x, x->r, sl, &i) != 1 || !ep_live(i, sl)) return;   /* executed: COMMITTED */
  if (i->status != EP_PREACCEPTED) return;
  if (m->ballot > i->ballot) return;
  i->acks |= 1u << src;
  if ((int32_t)m->cid > i->seq) { i->seq = (int32_t)m->cid; i->changed = 1; }     /* merge (instance.go:30-41) */
  for (id = 0; id < s->N; id++)
    if ((int32_t)pw[id] > i->dep[id]) { i->dep[id] = (int32_t)pw[id]; i->changed = 1; }
  for (id = 0; id < s->N; id++) {
    const int32_t d = (int32_t)pw[s->N + id];
    if (d > p->ep_committed[id]) p->ep_committed[id] = d;
    if (p->ep_committed[id] >= 0 && p->ep_committed[id] < i->dep[id]) committed = 0;
  }
  if (popc(i->acks) >= (int)(s->N * 3 / 4)) {             /* FastQuorum (quorum.go:65-67) */
    if (!i->changed && committed) {                        /* fast path */
      i->status = EP_COMMITTED;
      p->commits++;
      ep_update_commit(x, x->r);
      ep_commit_broadcast(x, i, sl);
      if (s->cfg.reply_when_commit && i->req) ep_reply(x, i, 0);
    } else {                                               /* slow path */
      uint32_t pay[PAXISIM_MAX_N], k;
      i->status = EP_ACCEPTED;
      i->acks = 1u << x->r;
      for (k = 0; k < s->N; k++) pay[k] = (uint32_t)i->dep[k];
      ep_broadcast(x, PAXISIM_MSG_ACCEPT, i->ballot, (uint32_t)sl, (uint32_t)i->seq, pay, s->N);
    }
  }
}

static void ep_handle_accept(ctx_t* x, uint32_t o, const rec_t* m) {   /* replica.go:262-290 */
  replica_t* p = x->n;
  const uint32_t* pw = (const uint32_t*)(m + 1);
  const int32_t s = (int32_t)m->slot;
  ep_inst_t* i = NULL;
  uint32_t k;
  const int w = ep_where(x, o, s, &i);
  if (w == 0) return;
  if (w == 2) { raise_flag(x, PAXISIM_F_WOVF | PAXISIM_F_UNFAITHFUL); return; }
  if (!ep_live(i, s)) ep_new(i, s);
  if (i->status == EP_COMMITTED) return;
  if (s > p->ep_slot[o]) p->ep_slot[o] = s;
  if (m->ballot >= i->ballot) {
    i->status = EP_ACCEPTED; i->ballot = (uint8_t)m->ballot; i->seq = (int32_t)m->cid;
    for (k = 0; k < x->s->N; k++) i->dep[k] = (int32_t)pw[k];
  }
  send1(x, o, PAXISIM_MSG_ACCEPTREPLY, i->ballot, (uint32_t)s, 0);
}

static void ep_handle_accept_reply(ctx_t* x, uint32_t src, const rec_t* m) {   /* replica.go:292-321 */
  const int32_t sl = (int32_t)m->slot;
  ep_inst_t* i = NULL;
  if (ep_where(x, x->r, sl, &i) != 1 || !ep_live(i, sl)) return;
  if (i->status != EP_ACCEPTED) return;
  if (i->ballot < m->ballot) { i->ballot = (uint8_t)m->ballot; return; }
  i->acks |= 1u << src;
  if (popc(i->acks) > (int)(x->s->N / 2)) {              /* Majority */
    i->status = EP_COMMITTED;
    x->n->commits++;
    ep_update_commit(x, x->r);
    if (x->s->cfg.reply_when_commit && i->req) ep_reply(x, i, 0);
    ep_commit_broadcast(x, i, sl);
  }
}

static void ep_handle_commit(ctx_t* x, uint32_t o, const rec_t* m) {   /* replica.go:323-353 */
  replica_t* p = x->n;
  const uint32_t* pw = (const uint32_t*)(m + 1);
  const int32_t s = (int32_t)m->slot;
  ep_inst_t* i = NULL;
  uint32_t k;
  const int w = ep_where(x, o, s, &i);
  if (s > p->ep_slot[o]) p->ep_slot[o] = s;
  if (w == 2) { raise_flag(x, PAXISIM_F_WOVF | PAXISIM_F_UNFAITHFUL); return; }
  if (w == 0) {                                            /* committed for good: re-commit in place */
    int32_t* cf = ep_cf(x, o, ep_key(x, m->cid));
    ep_update(x, m->cid, o, s, (int32_t)pw[0]);
    if (cf[0] == s) cf[1] = (int32_t)pw[0];
    ep_update_commit(x, o);
    return;
  }
  if (!ep_live(i, s)) ep_new(i, s);
  if (m->ballot >= i->ballot) {
    i->ballot = (uint8_t)m->ballot; i->cmd = m->cid; i->status = EP_COMMITTED; i->seq = (int32_t)pw[0];
    for (k = 0; k < x->s->N; k++) i->dep[k] = (int32_t)pw[1 + k];
    ep_update(x, m->cid, o, s, (int32_t)pw[0]);
  }
  if (i->req) {                                            /* r.Retry: back into MessageChan */
    client_enqueue(x, x->r, REQ_CID(i->req));
    i->req = 0;
  }
  ep_update_commit(x, o);
}

static void epaxos_dispatch(ctx_t* x, uint32_t src, const rec_t* m) {   /* registrations replica.go:49-54 */
  switch (HDR_TYPE(m->hdr)) {
    case PAXISIM_MSG_REQUEST:
      ep_handle_request(x, REQ(m->cid, src == x->s->N ? PAXISIM_CLIENT_SRC : src));
      break;
    case PAXISIM_MSG_REPLY: handle_reply(x, m->cid, m->ballot); break;
    case PAXISIM_MSG_PREACCEPT: ep_handle_preaccept(x, src, m); break;
    case PAXISIM_MSG_PREACCEPTREPLY: ep_handle_preaccept_reply(x, src, m); break;
    case PAXISIM_MSG_ACCEPT: ep_handle_accept(x, src, m); break;
    case PAXISIM_MSG_ACCEPTREPLY: ep_handle_accept_reply(x, src, m); break;
    case PAXISIM_MSG_COMMIT: ep_handle_commit(x, src, m); break;
    default: break;
  }
}

/* ------------------------------------------------------------------------ */
/* ABD atomic storage (abd/replica.go)                                       */
/* Record fields: hdr = type | key << 8, ballot = coordinator op id (CID),   */
/* slot = version, cid = value (a write's value is its command id; 0 = nil). */
/* ------------------------------------------------------------------------ */
static void abd_send(ctx_t* x, uint32_t to, uint32_t type, uint32_t key, uint32_t opid, uint32_t ver, uint32_t val) {
  rec_t m;
  m.hdr = HDR(type, key); m.ballot = opid; m.slot = ver; m.cid = val;
  sock_send(x, to, &m, 1);
}
static void abd_broadcast(ctx_t* x, uint32_t type, uint32_t key, uint32_t opid, uint32_t ver, uint32_t val) {
  uint32_t d;
  for (d = 0; d < x->s->N; d++)
    if (d != x->r) abd_send(x, d, type, key, opid, ver, val);
}
static inline int majority(const ctx_t* x, uint32_t mask) { return popc(mask) > (int)(x->s->N / 2); } /* quorum.go:60-62 */

/* database.Put (db.go:123-134): only a non-nil value is written */
static inline void abd_put(replica_t* p, uint32_t key, uint32_t val) { if (val) p->kv_val[key] = val; }

static void abd_handle_request(ctx_t* x, uint32_t cid) {                    /* abd/replica.go:50-71 */
  replica_t* p = x->n;
  const uint32_t k = key_fit(x, wl_key(x->s, x->c->kc, cid));
  abd_op_t* e;
  p->abd_cid++;
  e = &p->ops[p->abd_cid & (x->s->OW - 1u)];
  if (e->state == ABD_GET || e->state == ABD_SET)
    raise_flag(x, PAXISIM_F_PEND_OVF | PAXISIM_F_UNFAITHFUL);               /* evicting a live op */
  e->tag = p->abd_cid;
  e->req = cid;
  e->state = ABD_GET;
  e->getmask = 1u << x->r;
  e->setmask = 0;
  e->value = p->kv_val[k];
  e->version = p->kv_ver[k];
  e->start = x->t;
  abd_broadcast(x, PAXISIM_MSG_GET, k, p->abd_cid, 0, 0);
}

static void abd_handle_get(ctx_t* x, uint32_t src, uint32_t key, uint32_t opid) { /* abd/replica.go:73-82 */
  abd_send(x, src, PAXISIM_MSG_GETREPLY, key, opid, x->n->kv_ver[key], x->n->kv_val[key]);
}

static void abd_handle_set(ctx_t* x, uint32_t src, uint32_t key, uint32_t opid, uint32_t ver, uint32_t val) { /* 84-95 */
  replica_t* p = x->n;
  if (ver > p->kv_ver[key]) {
    abd_put(p, key, val);
    p->kv_ver[key] = ver;
  }
  abd_send(x, src, PAXISIM_MSG_SETREPLY, key, opid, 0, 0);
}

static abd_op_t* abd_op(ctx_t* x, uint32_t opid) {
  abd_op_t* e = &x->n->ops[opid & (x->s->OW - 1u)];
  return e->tag == opid ? e : NULL;   /* a retired op: Go's entry is Done, or was flagged when evicted */
}

static void abd_handle_getreply(ctx_t* x, uint32_t src, uint32_t key, uint32_t opid, uint32_t ver, uint32_t val) { /* 97-136 */
  replica_t* p = x->n;
  abd_op_t* e = abd_op(x, opid);
  if (!e || e->state != ABD_GET) return;
  if (ver > e->version) {
    e->value = val;
    e->version = ver;
    abd_put(p, key, val);
    p->kv_ver[key] = ver;
  }
  e->getmask |= 1u << src;
  if (majority(x, e->getmask)) {
    e->state = ABD_SET;
    e->setmask |= 1u << x->r;
    if (!wl_write(x->s, x->c->kc, e->req)) {
      abd_broadcast(x, PAXISIM_MSG_SET, key, opid, e->version, e->value);
    } else {
      e->value = e->req;                                                    /* the write's value */
      e->version++;
      abd_put(p, key, e->value);
      p->kv_ver[key] = e->version;
      abd_broadcast(x, PAXISIM_MSG_SET, key, opid, e->version, e->value);
    }
  }
}

static void abd_handle_setreply(ctx_t* x, uint32_t src, uint32_t key, uint32_t opid) { /* 138-157 */
  cluster_t* c = x->c;
  abd_op_t* e = abd_op(x, opid);
  if (!e || e->state != ABD_SET) return;
  e->setmask |= 1u << src;
  if (majority(x, e->setmask)) {
    int w = wl_write(x->s, c->kc, e->req);
    replica_t* p = x->n;
    e->state = ABD_DONE;
    p->commits++;
    if (p->nh < x->s->cfg.history) {                 /* History.AddOperation (history.go:44-52) */
      hist_t* h = &p->hist[p->nh++];
      h->key = key;
      h->is_write = (uint32_t)w;
      h->value = e->value;
      h->start = e->start;
      h->end = x->t;
    } else if (x->s->cfg.history) {
      raise_flag(x, PAXISIM_F_HIST_OVF);
    }
    client_reply(x, e->req, w ? 0u : e->value);          /* Reply{Value: e.value} for a read only */
  }
}

static void abd_dispatch(ctx_t* x, uint32_t src, const rec_t* m) {
  const uint32_t key = HDR_N(m->hdr);
  switch (HDR_TYPE(m->hdr)) {
    case PAXISIM_MSG_REQUEST: abd_handle_request(x, m->cid); break;
    case PAXISIM_MSG_GET: abd_handle_get(x, src, key, m->ballot); break;
    case PAXISIM_MSG_GETREPLY: abd_handle_getreply(x, src, key, m->ballot, m->slot, m->cid); break;
    case PAXISIM_MSG_SET: abd_handle_set(x, src, key, m->ballot, m->slot, m->cid); break;
    case PAXISIM_MSG_SETREPLY: abd_handle_setreply(x, src, key, m->ballot); break;
    default: break;
  }
}

/* ------------------------------------------------------------------------ */
/* One replica, one step                                    */
/* ------------------------------------------------------------------------ */
static void fault_process(ctx_t* x) {
  const struct oracle_sim* s = x->s;
  const paxisim_fault_process* fp = &s->fp;
  replica_t* p = x->n;
  uint32_t d;
  if (fp->drop_ppm == 0 && fp->slow_ppm == 0) return;
  for (d = 0; d < s->N; d++) {
    uint32_t u;
    if (d == x->r) continue;
    u = draw(x->hs, TAG(PUR_LINK, x->r, d));
    if (fp->drop_ppm && x->t >= p->drop_until[d] && ppm_hit16(u & 0xFFFFu, fp->drop_ppm))
      p->drop_until[d] = x->t + fp->drop_len;
    if (fp->slow_ppm && x->t >= p->slow_until[d] && ppm_hit16(u >> 16, fp->slow_ppm)) {
      uint32_t span = fp->slow_max - fp->slow_min + 1u;
      uint32_t v = draw(x->hs, TAG(PUR_SLOWD, x->r, d));
      p->slow_until[d] = x->t + fp->slow_len;
      p->slow_delay[d] = fp->slow_min + (uint32_t)(((uint64_t)v * span) >> 32);
    }
  }
}

/* A worker whose first request is due at step t sends it to its target now
 * (paxisim_workload.start_step); it joins the target's client queue after the
 * requests already there. */
static void client_start(ctx_t* x) {
  const struct oracle_sim* s = x->s;
  uint32_t w;
  for (w = 0; w < s->wl.outstanding; w++) {
    uint8_t* cnt;
    rec_t* m;
    if (s->wl.start_step[w] != x->t || x->t == 0 || s->wl.target[w] != x->r) continue;
    x->c->wk_cur[w] = 1u + w;
    x->c->wk_issued[w] = 1;
    cnt = mb_cnt(s, x->c, x->t % s->D, x->r, s->N);
    if (*cnt >= s->M) { raise_flag(x, PAXISIM_F_MBOX_OVF | PAXISIM_F_UNFAITHFUL); continue; }
    m = mb_rec(s, x->c, x->t % s->D, x->r, s->N, *cnt);
    m->hdr = HDR(PAXISIM_MSG_REQUEST, 0); m->ballot = 0; m->slot = 0; m->cid = 1u + w;
    (*cnt)++;
  }
}

static void replica_step(const struct oracle_sim* s, cluster_t* c, uint32_t r, uint32_t t) {
  ctx_t x;
  uint32_t b = t % s->D, src, rem[PAXISIM_MAX_N + 1], pos[PAXISIM_MAX_N + 1], total = 0, i;
  int crash;
  x.s = s; x.c = c; x.n = &c->rep[r]; x.p = &x.n->inst[0]; x.ktag = 0;
  x.r = r; x.t = t; x.stop = 0;
  x.hs = step_key(c->kc, t);
  x.n->send_seq = 0;
  x.n->nag = 0;
  if (s->late_workers) client_start(&x);
  fault_process(&x);
  crash = crashed(s, c, r, t);
  for (src = 0; src < s->NS; src++) {
    rem[src] = *mb_cnt(s, c, b, r, src);
    pos[src] = 0;
    if (crash && src < s->N && rem[src]) {               /* socket.Recv discards (socket.go:111-118) */
      uint32_t k = 0;
      while (k < rem[src]) {
        rec_t* m = mb_rec(s, c, b, r, src, k);
        x.n->discarded++;
        k += rec_len(m->hdr);
      }
      rem[src] = 0;
    }
    total += rem[src];
  }
  for (i = 0; total > 0 && !x.stop; i++) {
    uint32_t u = draw(x.hs, TAG(PUR_ORDER, r, i >> 1));       /* two 16-bit picks per draw */
    uint32_t pick = (((i & 1u) ? (u >> 16) : (u & 0xFFFFu)) * total) >> 16, len;
    rec_t* m;
    for (src = 0; pick >= rem[src]; src++) pick -= rem[src];
    m = mb_rec(s, c, b, r, src, pos[src]);
    len = rec_len(m->hdr);
    pos[src] += len;
    rem[src] -= len;
    total -= len;
    if (src == s->N) x.n->client_requests++;
    else x.n->delivered[HDR_TYPE(m->hdr)]++;
    if (s->cfg.protocol == PAXISIM_ABD) abd_dispatch(&x, src, m);
    else if (s->cfg.protocol == PAXISIM_WPAXOS) wpaxos_dispatch(&x, src, m);
    else if (s->cfg.protocol == PAXISIM_EPAXOS) epaxos_dispatch(&x, src, m);
    else paxos_dispatch(&x, src, m);
  }
  for (src = 0; src < s->NS; src++) *mb_cnt(s, c, b, r, src) = 0;
  if (x.stop && c->poison_step > t) c->poison_step = t;
}

static void cluster_step(const struct oracle_sim* s, cluster_t* c, uint32_t t) {
  uint32_t r, k, perm[PAXISIM_MAX_N];
  if (c->poison_step < t) return;                          /* a panic froze the process */
  if (!s->order) {
    for (r = 0; r < s->N; r++) replica_step(s, c, r, t);
    return;
  }
  /* test hook: the replicas of the step in another order - reversed (1), or
   * shuffled per (cluster, step) by a hash (2) - to check that a step's
   * replica-steps are independent (DESIGN.md §3.3, §5.6 busiest first) */
  for (r = 0; r < s->N; r++) perm[r] = s->order == 1 ? s->N - 1u - r : r;
  if (s->order == 2) {
    uint32_t h = (uint32_t)(c - s->cl) * 0x9E3779B1u ^ t * 0x85EBCA77u;
    for (k = s->N - 1u; k > 0; k--) {
      uint32_t j, tmp;
      h ^= h >> 15; h *= 0x2C1B3C6Du; h ^= h >> 12;
      j = h % (k + 1u);
      tmp = perm[k]; perm[k] = perm[j]; perm[j] = tmp;
    }
  }
  for (k = 0; k < s->N; k++) replica_step(s, c, perm[k], t);
}

int oracle_set_replica_order(oracle_sim* s, uint32_t mode) {
  if (!s || mode > 2) return fail(PAXISIM_EINVAL, "replica order mode");
  s->order = mode;
  return 0;
}

/* ------------------------------------------------------------------------ */
/* API                                                                       */
/* ------------------------------------------------------------------------ */
static int check_config(const paxisim_config* cfg, const paxisim_workload* wl,
                        const paxisim_fault_process* fp, uint32_t* N_out) {
  uint32_t z, N = 0, w;
  if (cfg->protocol > PAXISIM_EPAXOS || cfg->protocol == PAXISIM_M2PAXOS || cfg->protocol == PAXISIM_KPAXOS)
    return fail(PAXISIM_EUNSUPP, "protocol %u not built", cfg->protocol);
  if (cfg->protocol == PAXISIM_EPAXOS && (cfg->keys < 1 || cfg->keys > WP_KMAX))
    return fail(PAXISIM_EINVAL, "EPaxos keys must be in [1,%u]", WP_KMAX);
  if (cfg->protocol == PAXISIM_ABD && (cfg->keys < 1 || cfg->keys > KMAX)) return fail(PAXISIM_EINVAL, "keys");
  if (cfg->protocol == PAXISIM_WPAXOS && (cfg->keys < 1 || cfg->keys > WP_KMAX))
    return fail(PAXISIM_EINVAL, "WPaxos keys must be in [1,%u]", WP_KMAX);
  if (cfg->policy_threshold > 255) return fail(PAXISIM_EINVAL, "policy_threshold");
  if (cfg->policy > PAXISIM_POLICY_EMA) return fail(PAXISIM_EINVAL, "policy %u", cfg->policy);
  if (cfg->policy == PAXISIM_POLICY_MAJORITY && cfg->policy_interval < 1) return fail(PAXISIM_EINVAL, "policy_interval");
  if (cfg->policy == PAXISIM_POLICY_EMA && !(cfg->policy_alpha > 0.0 && cfg->policy_alpha <= 1.0))
    return fail(PAXISIM_EINVAL, "policy_alpha must be in (0, 1]");
  if (wl->locality_ppm && cfg->keys < 1) return fail(PAXISIM_EINVAL, "locality needs keys");
  if (cfg->n_zones < 1 || cfg->n_zones > PAXISIM_MAX_ZONES) return fail(PAXISIM_EINVAL, "n_zones");
  for (z = 0; z < cfg->n_zones; z++) {
    if (cfg->npz[z] < 1) return fail(PAXISIM_EINVAL, "npz[%u] must be >= 1", z);
    N += cfg->npz[z];
  }
  if (N < 1 || N > PAXISIM_MAX_N) return fail(PAXISIM_EINVAL, "N=%u out of range", N);
  if (cfg->protocol == PAXISIM_EPAXOS && N > 12) return fail(PAXISIM_EINVAL, "EPaxos supports N <= 12");
  if (cfg->window < 8 || cfg->window > PAXISIM_MAX_WINDOW || (cfg->window & (cfg->window - 1)))
    return fail(PAXISIM_EINVAL, "window must be a power of 2 in [8,64]");
  if (cfg->mbox_cap < 2 || cfg->mbox_cap > PAXISIM_MAX_MBOX) return fail(PAXISIM_EINVAL, "mbox_cap");
  if (cfg->max_delay > PAXISIM_MAX_DELAY) return fail(PAXISIM_EINVAL, "max_delay");
  if (cfg->q1 > PAXISIM_Q_FGRID_Q2 || cfg->q2 > PAXISIM_Q_FGRID_Q2) return fail(PAXISIM_EINVAL, "quorum kind");
  if (cfg->clusters < 1) return fail(PAXISIM_EINVAL, "clusters");
  if (cfg->agree_ring > 65536) return fail(PAXISIM_EINVAL, "agree_ring > 65536");
  if (wl->outstanding < 1 || wl->outstanding > PAXISIM_MAX_WORKERS) return fail(PAXISIM_EINVAL, "outstanding");
  if (wl->outstanding > cfg->mbox_cap) return fail(PAXISIM_EINVAL, "outstanding exceeds mbox_cap");
  if (wl->distribution > PAXISIM_DIST_TABLE) return fail(PAXISIM_EINVAL, "distribution %u", wl->distribution);
  if (wl->distribution == PAXISIM_DIST_CONFLICT && wl->conflicts > 100) return fail(PAXISIM_EINVAL, "conflicts > 100");
  {   /* the workload's key space (paxisim.h paxisim_workload) */
    const uint32_t K = cfg->keys ? cfg->keys : 1u, KS = wl->key_space ? wl->key_space : K;
    uint32_t e;
    if (KS > K) return fail(PAXISIM_EINVAL, "key_space %u exceeds keys %u", KS, K);
    if (wl->distribution == PAXISIM_DIST_CONFLICT && wl->key_min && KS >= K)
      return fail(PAXISIM_EINVAL, "conflict with key_min != 0 needs key_space < keys (literal key 0 has its own index)");
    if (wl->distribution == PAXISIM_DIST_TABLE) {
      for (w = 1; w + 1u < K; w++)
        if (wl->key_cdf[w] < wl->key_cdf[w - 1]) return fail(PAXISIM_EINVAL, "key_cdf must be non-decreasing");
      if (wl->key_tail && K >= 2 && wl->key_tail < wl->key_cdf[K - 2])
        return fail(PAXISIM_EINVAL, "key_tail below the last key_cdf threshold");
    } else if (wl->key_tail) {
      return fail(PAXISIM_EINVAL, "key_tail needs a table distribution");
    }
    if (wl->move_every) {
      if (wl->distribution != PAXISIM_DIST_TABLE) return fail(PAXISIM_EINVAL, "move_every needs a table distribution");
      if (!wl->move_cdf || wl->move_tables < 1 || wl->move_loop >= wl->move_tables)
        return fail(PAXISIM_EINVAL, "move_cdf / move_tables / move_loop");
      for (e = 0; e < wl->move_tables; e++)
        for (w = 1; w + 1u < K; w++)
          if (wl->move_cdf[e * PAXISIM_MAX_KEYS + w] < wl->move_cdf[e * PAXISIM_MAX_KEYS + w - 1])
            return fail(PAXISIM_EINVAL, "move_cdf table %u must be non-decreasing", e);
    }
  }
  for (w = 0; w < wl->outstanding; w++)
    if (wl->target[w] >= N) return fail(PAXISIM_EINVAL, "target[%u]", w);
  if (fp->slow_ppm && (fp->slow_min > fp->slow_max || fp->slow_max > cfg->max_delay))
    return fail(PAXISIM_EINVAL, "slow delay range exceeds max_delay");
  *N_out = N;
  return 0;
}

static uint32_t abd_ow(uint32_t outstanding) {  /* ABD op table: pow2 >= 2*outstanding, >= 4 */
  uint32_t ow = 4;
  while (ow < 2u * outstanding) ow <<= 1;
  return ow;
}

static void cluster_init(struct oracle_sim* s, cluster_t* c, uint64_t gid, entry_t* logs, inst_t* insts) {
  uint32_t r, w;
  memset(c->rep, 0, sizeof c->rep);
  c->gid = gid;
  c->kc = cluster_key(s->cfg.seed, gid);
  c->poison_step = 0xFFFFFFFFu;
  for (r = 0; r < s->N; r++) {
    uint32_t k;
    c->rep[r].inst = insts + (size_t)r * s->NK;
    for (k = 0; k < s->NK; k++) {
      inst_t* p = &c->rep[r].inst[k];
      p->slot = -1;                                        /* paxos.go:45 */
      p->log = logs + ((size_t)r * s->NK + k) * s->W;
      p->exists = s->cfg.protocol != PAXISIM_WPAXOS;
      p->pol_last = POL_NONE;
    }
    if (s->cfg.protocol == PAXISIM_EPAXOS) {             /* replica.go:37-47: slot, committed, executed = -1 */
      replica_t* p = &c->rep[r];
      uint32_t o;
      p->ep_log = (ep_inst_t*)calloc((size_t)s->N * s->W, sizeof(ep_inst_t));
      p->ep_cf = (int32_t*)malloc((size_t)s->N * s->cfg.keys * 2 * sizeof(int32_t));
      p->ep_maxseq = (int32_t*)malloc((size_t)s->cfg.keys * sizeof(int32_t));
      for (o = 0; o < s->N * s->cfg.keys; o++) { p->ep_cf[2 * o] = -1; p->ep_cf[2 * o + 1] = 0; }
      for (o = 0; o < s->cfg.keys; o++) p->ep_maxseq[o] = -1;
      for (o = 0; o < s->N; o++) p->ep_slot[o] = p->ep_committed[o] = p->ep_executed[o] = -1;
    }
    if (s->kv) c->rep[r].db = (uint32_t*)calloc(s->cfg.keys ? s->cfg.keys : 1, sizeof(uint32_t));
    if (s->cfg.protocol == PAXISIM_ABD) {
      c->rep[r].kv_val = (uint32_t*)calloc(2u * s->cfg.keys, sizeof(uint32_t));
      c->rep[r].kv_ver = c->rep[r].kv_val + s->cfg.keys;
      c->rep[r].ops = (abd_op_t*)calloc(s->OW, sizeof(abd_op_t));
      c->rep[r].hist = (hist_t*)calloc(s->cfg.history ? s->cfg.history : 1, sizeof(hist_t));
    }
  }
  memset(c->wk_cur, 0, sizeof c->wk_cur);
  memset(c->wk_issued, 0, sizeof c->wk_issued);
  /* every worker's first request waits at its target at step 0 */
  for (w = 0; w < s->wl.outstanding; w++) {
    uint32_t tg = s->wl.target[w];
    uint8_t* cnt = mb_cnt(s, c, 0, tg, s->N);
    if (s->wl.start_step[w]) continue;                     /* joins later (client_start) */
    rec_t* m = mb_rec(s, c, 0, tg, s->N, *cnt);
    m->hdr = HDR(PAXISIM_MSG_REQUEST, 0); m->ballot = 0; m->slot = 0; m->cid = 1u + w;
    (*cnt)++;
    c->wk_cur[w] = 1u + w;
    c->wk_issued[w] = 1;
  }
}

int oracle_create(const paxisim_config* cfg, const paxisim_workload* wl,
                  const paxisim_fault_process* fp, oracle_sim** out) {
  struct oracle_sim* s;
  uint32_t N = 0, z, r = 0;
  uint64_t i;
  paxisim_fault_process nofp;
  int rc;
  paxisim_config ncfg;
  uint32_t variant;
  if (!cfg || !wl || !out) return fail(PAXISIM_EINVAL, "null argument");
  /* M2Paxos and KPaxos are per-key Paxos as WPaxos is: same state, another
   * request path and Majority quorums (m2paxos/kpaxos.go:15-21, kpaxos/replica.go) */
  ncfg = *cfg;
  variant = cfg->protocol;
  if (variant == PAXISIM_M2PAXOS || variant == PAXISIM_KPAXOS) ncfg.protocol = PAXISIM_WPAXOS;
  cfg = &ncfg;
  if (!fp) { memset(&nofp, 0, sizeof nofp); fp = &nofp; }
  if ((rc = check_config(cfg, wl, fp, &N))) return rc;
  s = (struct oracle_sim*)calloc(1, sizeof *s);
  if (!s) return fail(PAXISIM_ENOMEM, "oom");
  s->cfg = *cfg; s->wl = *wl; s->fp = *fp;
  s->wl.move_cdf = NULL;                                   /* the caller's buffer is not kept */
  if (wl->move_every) {
    const size_t mb = (size_t)wl->move_tables * PAXISIM_MAX_KEYS * sizeof(uint32_t);
    if (!(s->move_cdf = (uint32_t*)malloc(mb))) { free(s); return fail(PAXISIM_ENOMEM, "oom"); }
    memcpy(s->move_cdf, wl->move_cdf, mb);
  }
  s->N = N; s->Z = cfg->n_zones; s->W = cfg->window; s->M = cfg->mbox_cap;
  s->D = cfg->max_delay + 2u; s->NS = N + 1u;
  if (s->wl.outstanding > PAXISIM_MAX_WORKERS) s->wl.outstanding = PAXISIM_MAX_WORKERS;
  for (z = 0; z < s->Z; z++) {
    uint32_t k;
    s->zmask[z] = ((1u << cfg->npz[z]) - 1u) << r;
    for (k = 0; k < cfg->npz[z]; k++, r++) { s->zone_of[r] = z + 1; s->node_of[r] = k + 1; }
  }
  s->C = cfg->clusters;
  s->keep_xlog = cfg->clusters <= 16;
  for (z = 0; z < s->wl.outstanding; z++) s->late_workers |= s->wl.start_step[z] != 0;
  s->OW = abd_ow(wl->outstanding);
  s->NK = cfg->protocol == PAXISIM_WPAXOS ? cfg->keys : 1u;
  s->AR = (cfg->protocol == PAXISIM_ABD || cfg->protocol == PAXISIM_EPAXOS) ? 0u
          : cfg->agree_ring ? cfg->agree_ring : (cfg->protocol == PAXISIM_WPAXOS ? 128u : 1024u);
  s->q1 = cfg->q1;
  s->q2 = cfg->q2;
  if (cfg->protocol == PAXISIM_WPAXOS) {
    /* kpaxos: Q1/Q2 from fz (wpaxos/kpaxos.go:15-27); no ReplyWhenCommit option
     * (kpaxos.go:35-39) and the Paxos replica's -ephemeral_leader is not consulted */
    s->q1 = cfg->fz ? PAXISIM_Q_FGRID_Q1 : PAXISIM_Q_GRID_ROW;
    s->q2 = cfg->fz ? PAXISIM_Q_FGRID_Q2 : PAXISIM_Q_GRID_COLUMN;
    s->cfg.reply_when_commit = 0;
    s->cfg.ephemeral_leader = 0;
  }
  s->variant = variant;
  s->kv = cfg->kv && cfg->protocol != PAXISIM_ABD;
  if (variant == PAXISIM_M2PAXOS || variant == PAXISIM_KPAXOS) s->q1 = s->q2 = PAXISIM_Q_MAJORITY;
  if (variant == PAXISIM_M2PAXOS) s->cfg.adaptive = 1;      /* m2paxos/replica.go:34-52: no -adaptive switch */
  for (z = 0, r = 0; z < s->Z; r += cfg->npz[z], z++) s->zfirst[z] = r;
  s->cl = (cluster_t*)calloc(s->C, sizeof(cluster_t));
  if (!s->cl) { free(s->move_cdf); free(s); return fail(PAXISIM_ENOMEM, "oom clusters"); }
  for (i = 0; i < s->C; i++) {
    cluster_t* c = &s->cl[i];
    entry_t* logs = (entry_t*)calloc((size_t)N * s->NK * s->W, sizeof(entry_t));
    inst_t* insts = (inst_t*)calloc((size_t)N * s->NK, sizeof(inst_t));
    c->mbox = (rec_t*)malloc((size_t)s->D * N * s->NS * s->M * sizeof(rec_t));
    c->cnt = (uint8_t*)calloc((size_t)s->D * N * s->NS, 1);
    c->agr = s->AR ? (uint64_t*)calloc((size_t)s->NK * s->AR, sizeof(uint64_t)) : NULL;
    if (!logs || !insts || !c->mbox || !c->cnt || (s->AR && !c->agr)) {
      free(logs);
      free(insts);
      s->C = i;
      free(c->mbox);
      free(c->cnt);
      free(c->agr);
      oracle_destroy(s);
      return fail(PAXISIM_ENOMEM, "oom");
    }
    cluster_init(s, c, cfg->cluster_base + i, logs, insts);
  }
  *out = s;
  return 0;
}

int oracle_destroy(oracle_sim* s) {
  uint64_t i;
  uint32_t r;
  if (!s) return 0;
  free(s->move_cdf);
  for (i = 0; i < s->C; i++) {
    cluster_t* c = &s->cl[i];
    if (c->rep[0].inst) {
      free(c->rep[0].inst[0].log);
      for (r = 0; r < s->N; r++) {
        uint32_t k;
        for (k = 0; k < s->NK; k++) free(c->rep[r].inst[k].xlog);
      }
      free(c->rep[0].inst);
    }
    for (r = 0; r < s->N; r++) {
      free(c->rep[r].kv_val);
      free(c->rep[r].ops);
      free(c->rep[r].hist);
      free(c->rep[r].ep_log);
      free(c->rep[r].ep_cf);
      free(c->rep[r].ep_maxseq);
      free(c->rep[r].db);
    }
    free(c->mbox);
    free(c->cnt);
    free(c->agr);
  }
  free(s->cl);
  free(s);
  return 0;
}

static uint64_t expand_ballot(const struct oracle_sim* s, uint32_t b);

/* The HTTP request path (http.go:99): client request `cid` reaches replica r
 * of cluster cl in the next step (paxisim_inject). */
int oracle_inject(oracle_sim* s, uint64_t cl, uint32_t r, uint32_t cid) {
  cluster_t* c;
  uint8_t* cnt;
  rec_t* m;
  if (!s || cl >= s->C || r >= s->N || cid < 1 || cid > CID_MAX) return fail(PAXISIM_EINVAL, "bad inject");
  c = &s->cl[cl];
  cnt = mb_cnt(s, c, s->t % s->D, r, s->N);
  if (*cnt >= s->M) return fail(PAXISIM_EINVAL, "client mailbox full");
  m = mb_rec(s, c, s->t % s->D, r, s->N, *cnt);
  m->hdr = HDR(PAXISIM_MSG_REQUEST, 0); m->ballot = 0; m->slot = 0; m->cid = cid;
  (*cnt)++;
  return 0;
}

/* What replica r of cluster cl receives at the next step, source by source,
 * FIFO within a source: what a per-connection gob decoder hands node.recv
 * (transport.go:146-165, node.go:79-101); paxisim_read_inbox. */
int oracle_read_inbox(oracle_sim* s, uint64_t cl, uint32_t r, paxisim_inbox_record* out, uint32_t cap,
                      uint32_t* n_out) {
  cluster_t* c;
  uint32_t src, k, n = 0;
  if (!s || !n_out || (cap && !out) || cl >= s->C || r >= s->N) return fail(PAXISIM_EINVAL, "bad inbox");
  c = &s->cl[cl];
  for (src = 0; src < s->NS; src++) {
    const uint32_t kn = *mb_cnt(s, c, s->t % s->D, r, src);
    for (k = 0; k < kn; k++, n++) {
      const rec_t* m = mb_rec(s, c, s->t % s->D, r, src, k);
      if (n >= cap) continue;
      out[n].src = src; out[n].hdr = m->hdr; out[n].ballot = m->ballot; out[n].slot = m->slot; out[n].cid = m->cid;
    }
  }
  *n_out = n;
  return 0;
}

/* A message off a transport (paxisim_deliver): appended to (r, src) for the next step. */
int oracle_deliver(oracle_sim* s, uint64_t cl, uint32_t r, uint32_t src, const paxisim_inbox_record* in,
                   uint32_t n) {
  cluster_t* c;
  uint8_t* cnt;
  uint32_t i;
  if (!s || (n && !in) || cl >= s->C || r >= s->N || src > s->N) return fail(PAXISIM_EINVAL, "bad deliver");
  if (n == 0) return 0;
  c = &s->cl[cl];
  cnt = mb_cnt(s, c, s->t % s->D, r, src);
  if (*cnt + n > s->M) return fail(PAXISIM_EINVAL, "mailbox full");
  for (i = 0; i < n; i++) {
    rec_t* m = mb_rec(s, c, s->t % s->D, r, src, *cnt + i);
    m->hdr = in[i].hdr; m->ballot = in[i].ballot; m->slot = in[i].slot; m->cid = in[i].cid;
  }
  *cnt = (uint8_t)(*cnt + n);
  return 0;
}

int oracle_read_log(oracle_sim* s, uint64_t cl, uint32_t r, uint32_t key, int32_t lo, uint32_t n,
                    paxisim_log_entry* out) {
  const inst_t* p;
  uint32_t i;
  if (!s || !out || cl >= s->C || r >= s->N || key >= s->NK) return fail(PAXISIM_EINVAL, "bad argument");
  p = &s->cl[cl].rep[r].inst[key];
  for (i = 0; i < n; i++) {
    const int32_t sl = lo + (int32_t)i;
    paxisim_log_entry* o = &out[i];
    memset(o, 0, sizeof *o);
    o->slot = sl;
    if (sl < p->execute || sl >= p->execute + (int32_t)s->W) continue;
    {
      const entry_t* e = &p->log[(uint32_t)sl & (s->W - 1u)];
      o->flags = PAXISIM_LOG_HELD;
      if (!(e->meta & E_EXISTS)) continue;
      o->flags |= PAXISIM_LOG_EXISTS | (e->meta & E_COMMIT ? PAXISIM_LOG_COMMIT : 0u) |
                  (e->meta & E_QUORUM ? PAXISIM_LOG_QUORUM : 0u) | (e->req ? PAXISIM_LOG_REQUEST : 0u);
      o->ballot = expand_ballot(s, e->ballot);
      o->cmd = e->cmd;
      o->acks = E_ACK(e->meta);
      o->request = e->req;
    }
  }
  return 0;
}

int oracle_fault_add(oracle_sim* s, const paxisim_fault* f) {
  if (!s || !f) return fail(PAXISIM_EINVAL, "null argument");
  if (s->nfaults == PAXISIM_MAX_FAULTS) return fail(PAXISIM_EINVAL, "fault table full");
  if (f->kind > PAXISIM_FAULT_CRASH || f->src >= s->N ||
      (f->dst != PAXISIM_ALL_DST && f->dst >= s->N))
    return fail(PAXISIM_EINVAL, "bad fault");
  if (f->kind == PAXISIM_FAULT_SLOW && f->param > s->cfg.max_delay)
    return fail(PAXISIM_EINVAL, "slow delay exceeds max_delay");
  s->faults[s->nfaults++] = *f;
  return 0;
}

typedef struct { struct oracle_sim* s; uint64_t lo, hi; uint32_t t0, n; } shard_t;
static void* run_shard(void* a) {
  shard_t* sh = (shard_t*)a;
  uint64_t i;
  uint32_t k;
  for (i = sh->lo; i < sh->hi; i++)
    for (k = 0; k < sh->n; k++) cluster_step(sh->s, &sh->s->cl[i], sh->t0 + k);
  return NULL;
}

int oracle_step(oracle_sim* s, uint32_t nsteps, int nthreads) {
  if (!s) return fail(PAXISIM_EINVAL, "null handle");
  if (nthreads <= 1) {
    shard_t sh = {s, 0, s->C, s->t, nsteps};
    run_shard(&sh);
  } else {
    pthread_t th[256];
    shard_t sh[256];
    int k;
    if (nthreads > 256) nthreads = 256;
    for (k = 0; k < nthreads; k++) {
      sh[k].s = s; sh[k].t0 = s->t; sh[k].n = nsteps;
      sh[k].lo = s->C * (uint64_t)k / (uint64_t)nthreads;
      sh[k].hi = s->C * (uint64_t)(k + 1) / (uint64_t)nthreads;
      pthread_create(&th[k], NULL, run_shard, &sh[k]);
    }
    for (k = 0; k < nthreads; k++) pthread_join(th[k], NULL);
  }
  s->t += nsteps;
  return 0;
}

static uint64_t expand_ballot(const struct oracle_sim* s, uint32_t b) {   /* to ballot.go:15-17 */
  uint32_t rid = bal_id(b);
  return b ? oracle_new_ballot(b >> 4, s->zone_of[rid], s->node_of[rid]) : 0;
}

static void fill_state(const struct oracle_sim* s, const cluster_t* c, uint32_t r,
                       paxisim_replica_state* o) {
  const replica_t* p = &c->rep[r];
  const inst_t* q = &p->inst[0];
  memset(o, 0, sizeof *o);
  o->ballot = expand_ballot(s, q->ballot);
  o->slot = q->slot;
  o->execute = q->execute;
  o->active = q->active;
  o->flags = p->flags;
  o->digest = q->digest;
  o->p1_acks = q->p1mask;
  o->npending = q->npend;
  memcpy(o->delivered, p->delivered, sizeof o->delivered);
  if (s->cfg.protocol == PAXISIM_WPAXOS) {   /* per-replica aggregate over the key instances */
    uint32_t k, hi = 0;
    uint64_t d = 0;
    int32_t led = 0, ex = 0;
    o->active = o->p1_acks = o->npending = 0;
    for (k = 0; k < s->NK; k++) {
      q = &p->inst[k];
      if (q->ballot > hi) hi = q->ballot;
      led += q->exists && (q->active || bal_id(q->ballot) == r);   /* Replica.keys() replica.go:110-118 */
      ex += q->execute;
      o->active += q->active;
      o->p1_acks |= q->exists ? 1u << k : 0u;
      o->npending += q->npend;
      d = mix64(d ^ q->digest);
    }
    o->ballot = expand_ballot(s, hi);
    o->slot = led;
    o->execute = ex;
    o->digest = d;
  }
  if (s->cfg.protocol == PAXISIM_EPAXOS) {         /* own log head, executed prefix over all logs */
    uint32_t o2;
    o->ballot = 0;
    o->slot = p->ep_slot[r];
    o->execute = 0;
    for (o2 = 0; o2 < s->N; o2++) o->execute += p->ep_executed[o2] + 1;
    o->active = o->p1_acks = o->npending = 0;
  }
  if (s->cfg.protocol == PAXISIM_ABD) {            /* ABD: op counter, Done ops, KV digest, live ops */
    uint32_t k, live = 0;
    uint64_t d = 0;
    for (k = 0; k < s->cfg.keys; k++) d = mix64(d ^ (((uint64_t)p->kv_ver[k] << 32) | p->kv_val[k]));
    for (k = 0; k < s->OW; k++) live += p->ops[k].state == ABD_GET || p->ops[k].state == ABD_SET;
    o->ballot = 0;
    o->slot = (int32_t)p->abd_cid;
    o->execute = (int32_t)p->nh;
    o->digest = d;
    o->npending = live;
  }
  o->executions = s->cfg.protocol == PAXISIM_EPAXOS ? p->ep_execs : s->cfg.protocol == PAXISIM_ABD ? 0u
                                                                   : (uint32_t)o->execute;
  o->executed_writes = s->kv ? p->db_version : 0u;
  o->client_requests = p->client_requests;
  o->sent = p->sent;
  o->dropped = p->dropped;
  o->discarded = p->discarded;
  o->commits = p->commits;
  o->replies = p->replies;
}

int oracle_read_state(oracle_sim* s, uint64_t lo, uint64_t n, paxisim_replica_state* out) {
  uint64_t i;
  uint32_t r;
  if (!s || !out) return fail(PAXISIM_EINVAL, "null argument");
  if (lo + n > s->C) return fail(PAXISIM_ERANGE, "cluster range");
  for (i = 0; i < n; i++)
    for (r = 0; r < s->N; r++) fill_state(s, &s->cl[lo + i], r, &out[i * s->N + r]);
  return 0;
}

int oracle_read_instances(oracle_sim* s, uint64_t lo, uint64_t n, paxisim_instance_state* out) {
  uint64_t i;
  uint32_t r, k;
  if (!s || !out) return fail(PAXISIM_EINVAL, "null argument");
  if (lo + n > s->C) return fail(PAXISIM_ERANGE, "cluster range");
  if (s->cfg.protocol == PAXISIM_EPAXOS) {         /* one record per (replica, owner log) */
    for (i = 0; i < n; i++)
      for (r = 0; r < s->N; r++)
        for (k = 0; k < s->N; k++) {
          const replica_t* p = &s->cl[lo + i].rep[r];
          paxisim_instance_state* o = &out[(i * s->N + r) * s->N + k];
          memset(o, 0, sizeof *o);
          o->slot = p->ep_slot[k];
          o->execute = p->ep_executed[k] + 1;
          o->p1_acks = (uint32_t)(p->ep_committed[k] + 1);
          o->exists = 1;
          o->policy_last = POL_NONE;
        }
    return 0;
  }
  for (i = 0; i < n; i++)
    for (r = 0; r < s->N; r++)
      for (k = 0; k < s->NK; k++) {
        const inst_t* q = &s->cl[lo + i].rep[r].inst[k];
        paxisim_instance_state* o = &out[(i * s->N + r) * s->NK + k];
        memset(o, 0, sizeof *o);
        o->ballot = expand_ballot(s, q->ballot);
        o->slot = q->slot;
        o->execute = q->execute;
        o->active = q->active;
        o->exists = q->exists;
        o->p1_acks = q->p1mask;
        o->npending = q->npend;
        o->digest = q->digest;
        o->policy_last = q->pol_last;
        o->policy_hits = q->pol_hits;
        if (s->cfg.policy == PAXISIM_POLICY_MAJORITY) {
          uint32_t h = 0x811C9DC5u, j;
          for (j = 0; j < s->N; j++) h = fmix32(h ^ (q->pol_n[j] | j << 16));
          o->policy_state[0] = q->pol_sum;
          o->policy_state[1] = q->pol_time;
          o->policy_state[2] = h;
        } else if (s->cfg.policy == PAXISIM_POLICY_EMA) {
          uint64_t b;
          memcpy(&b, &q->pol_s, sizeof b);
          o->policy_state[0] = (uint32_t)b;
          o->policy_state[1] = (uint32_t)(b >> 32);
          o->policy_state[2] = q->pol_zone;
        }
      }
  return 0;
}

int oracle_stats_get(oracle_sim* s, paxisim_stats* o) {
  uint64_t i;
  uint32_t r, k;
  if (!s || !o) return fail(PAXISIM_EINVAL, "null argument");
  memset(o, 0, sizeof *o);
  o->steps = s->t;
  o->clusters = s->C;
  for (i = 0; i < s->C; i++) {
    uint32_t cf = 0;
    for (r = 0; r < s->N; r++) {
      const replica_t* p = &s->cl[i].rep[r];
      for (k = 0; k < PAXISIM_NMSG; k++) {
        o->delivered[k] += p->delivered[k];
        o->delivered_total += p->delivered[k];
      }
      o->client_requests += p->client_requests;
      o->sent += p->sent;
      o->dropped += p->dropped;
      o->discarded += p->discarded;
      o->commits += p->commits;
      o->replies += p->replies;
      o->agree_compared += p->agc;
      o->agree_missed += p->agm;
      o->agree_mismatch += p->agb;
      cf |= p->flags;
    }
    for (k = 0; k < 8; k++) if (cf & (1u << k)) o->flagged[k]++;
  }
  return 0;
}

/* Agreement scan (client.go:279-320 per-index set size <= 1; tla Safety):
 * checkpoints of the executed-history digest must agree across replicas. */
int oracle_check(oracle_sim* s, uint64_t* violations) {
  uint64_t i, v = 0;
  uint32_t a, b, k, j;
  if (!s || !violations) return fail(PAXISIM_EINVAL, "null argument");
  for (i = 0; i < s->C; i++) {
    const cluster_t* c = &s->cl[i];
    int bad = 0;
    uint32_t key;
    if (s->cfg.protocol == PAXISIM_EPAXOS) continue;           /* no single log: paxisim.h */
    for (a = 0; a < s->N; a++) bad |= c->rep[a].agb != 0;      /* running check (agree_arrive) */
    for (key = 0; key < s->NK && !bad; key++)      /* per Paxos instance: WPaxos per key (tla Safety) */
      for (a = 0; a < s->N && !bad; a++)
        for (b = a + 1; b < s->N && !bad; b++) {
          const inst_t *p = &c->rep[a].inst[key], *q = &c->rep[b].inst[key];
          if (p->execute == q->execute && p->digest != q->digest) bad = 1;
          for (k = 0; k < CKR && !bad; k++)
            for (j = 0; j < CKR && !bad; j++)
              if (p->ck_e[k] && p->ck_e[k] == q->ck_e[j] && p->ck_d[k] != q->ck_d[j]) bad = 1;
        }
    v += (uint64_t)bad;
  }
  *violations = v;
  return 0;
}

int oracle_exec_log(oracle_sim* s, uint64_t cl, uint32_t r, uint32_t* buf, uint32_t cap, uint32_t* n_out) {
  const inst_t* p;
  uint32_t n, key = r >> 16;                       /* WPaxos: replica | key << 16 */
  r &= 0xFFFFu;
  if (!s || !n_out || cl >= s->C || r >= s->N || key >= s->NK) return fail(PAXISIM_EINVAL, "bad argument");
  if (!s->keep_xlog) return fail(PAXISIM_EUNSUPP, "exec log kept only for <= 16 clusters");
  p = &s->cl[cl].rep[r].inst[key];
  n = p->nx < cap ? p->nx : cap;
  if (buf && n) memcpy(buf, p->xlog, n * sizeof(uint32_t));
  *n_out = p->nx;
  return 0;
}

/* ------------------------------------------------------------------------ */
/* Linearizability checker (checker.go:11-104, lib/graph.go:180-232)         */
/* Vertex iteration is in insertion order (Go's map order is random; the     */
/* reference's KATs do not depend on it).                                    */
/* ------------------------------------------------------------------------ */
typedef struct {
  int n;
  int64_t *hin, *in, *hout, *out, *start, *end;
  unsigned char* present;    /* vertex in graph */
  int* order;                /* insertion order of vertices */
  int norder;
  unsigned char* adj;        /* adj[u*n+v]: edge u -> v */
} lgraph_t;

static int lg_has(lgraph_t* g, int v) { return g->present[v]; }
static void lg_add(lgraph_t* g, int v) {
  if (g->present[v]) return;
  g->present[v] = 1;
  g->order[g->norder++] = v;
}
static void lg_remove(lgraph_t* g, int v) {
  int i, k = 0;
  if (!g->present[v]) return;
  g->present[v] = 0;
  for (i = 0; i < g->n; i++) { g->adj[v * g->n + i] = 0; g->adj[i * g->n + v] = 0; }
  for (i = 0; i < g->norder; i++) if (g->order[i] != v) g->order[k++] = g->order[i];
  g->norder = k;
}
static void lg_edge(lgraph_t* g, int u, int v) {
  lg_add(g, u);
  lg_add(g, v);
  g->adj[u * g->n + v] = 1;
}
static int happen_before(lgraph_t* g, int a, int b) { return g->end[a] < g->start[b]; } /* operation.go:12-14 */
static void chk_add(lgraph_t* g, int o) {                 /* checker.go:21-33 */
  int i;
  if (lg_has(g, o)) return;
  lg_add(g, o);
  for (i = 0; i < g->norder; i++) {
    int v = g->order[i];
    if (happen_before(g, v, o)) lg_edge(g, v, o);
  }
}
/* graph.go:180-193 visit; returns 1 if a cycle is found, gray marks the stack */
static int lg_visit(lgraph_t* g, int v, unsigned char* color) {
  int i;
  color[v] = 1;
  for (i = 0; i < g->norder; i++) {
    int u = g->order[i];
    if (!g->adj[v * g->n + u]) continue;
    if (color[u] == 1) return 1;
    if (color[u] == 0 && lg_visit(g, u, color)) return 1;
  }
  color[v] = 2;
  return 0;
}

int oracle_linearizable(const int64_t* ops, int n) {
  lgraph_t g;
  int *idx, i, j, anomalies = 0;
  unsigned char* color;
  if (n <= 0) return 0;
  memset(&g, 0, sizeof g);
  g.n = n;
  g.hin = (int64_t*)malloc(6 * (size_t)n * sizeof(int64_t));
  if (!g.hin) return -1;
  g.in = g.hin + n; g.hout = g.in + n; g.out = g.hout + n; g.start = g.out + n; g.end = g.start + n;
  g.present = (unsigned char*)calloc((size_t)n, 1);
  g.order = (int*)malloc((size_t)n * sizeof(int));
  g.adj = (unsigned char*)calloc((size_t)n * n, 1);
  idx = (int*)malloc((size_t)n * sizeof(int));
  color = (unsigned char*)malloc((size_t)n);
  /* sort.Sort(byTime(history)): stable by start (insertion sort for small n) */
  for (i = 0; i < n; i++) idx[i] = i;
  for (i = 1; i < n; i++) {
    int v = idx[i], k = i - 1;
    while (k >= 0 && ops[6 * idx[k] + 4] > ops[6 * v + 4]) { idx[k + 1] = idx[k]; k--; }
    idx[k + 1] = v;
  }
  for (i = 0; i < n; i++) {
    const int64_t* o = &ops[6 * idx[i]];
    g.hin[i] = o[0]; g.in[i] = o[1]; g.hout[i] = o[2]; g.out[i] = o[3]; g.start[i] = o[4]; g.end[i] = o[5];
  }
  for (i = 0; i < n; i++) {                                 /* checker.go:73-102 */
    chk_add(&g, i);
    if (!g.hin[i]) {                                        /* read */
      int match = -1, k;
      for (j = i + 1; j < n && !happen_before(&g, i, j) && !happen_before(&g, j, i); j++)
        if (!g.hout[j]) chk_add(&g, j);                     /* look-ahead concurrent writes */
      for (k = 0; k < g.norder; k++) {                      /* match: checker.go:44-52 */
        int v = g.order[k];
        if (g.hin[v] == g.hout[i] && (!g.hout[i] || g.in[v] == g.out[i])) { match = v; break; }
      }
      if (match >= 0) {                                     /* merge: checker.go:55-67 */
        for (k = 0; k < g.norder; k++) {
          int s2 = g.order[k];
          if (g.adj[s2 * n + i] && s2 != match) lg_edge(&g, s2, match);
        }
        if (g.end[i] < g.end[match]) g.end[match] = g.end[i];
        lg_remove(&g, i);
      }
      {                                                     /* Cycle: graph.go:212-232 */
        int found = 0;
        memset(color, 0, (size_t)n);
        for (k = 0; k < g.norder && !found; k++)
          if (color[g.order[k]] == 0 && lg_visit(&g, g.order[k], color)) found = 1;
        if (found) {
          int a, b;
          anomalies++;
          for (a = 0; a < g.norder; a++)
            for (b = 0; b < g.norder; b++) {
              int u = g.order[a], v = g.order[b];
              if (color[u] == 1 && color[v] == 1 && g.adj[u * n + v] && g.start[u] > g.end[v])
                g.adj[u * n + v] = 0;
            }
        }
      }
    }
  }
  free(g.hin); free(g.present); free(g.order); free(g.adj); free(idx); free(color);
  return anomalies;
}

/* History.Linearizable (history.go:55-71): run the checker on every
 * (cluster, key) partition of the completed-operation history. */
int oracle_lin_check(oracle_sim* s, uint64_t* anomalies, uint64_t* ops) {
  uint64_t i, a = 0, n = 0;
  uint32_t k, j;
  int64_t* buf = NULL;
  size_t cap = 0;
  if (!s || !anomalies) return fail(PAXISIM_EINVAL, "null argument");
  for (i = 0; i < s->C; i++) {
    const cluster_t* c = &s->cl[i];
    for (k = 0; k < s->cfg.keys; k++) {
      int m = 0, res;
      uint32_t r, nall = 0;
      for (r = 0; r < s->N; r++) nall += c->rep[r].nh;
      for (j = 0, r = 0; r < s->N; r++)
      for (j = 0; j < c->rep[r].nh; j++) {
        const hist_t* h = &c->rep[r].hist[j];
        if (h->key != k) continue;
        if ((size_t)(m + 1) * 6 > cap) {
          cap = cap ? 2 * cap : 6 * 256;
          buf = (int64_t*)realloc(buf, cap * sizeof(int64_t));
        }
        buf[6 * m + 0] = h->is_write ? 1 : 0;
        buf[6 * m + 1] = h->is_write ? h->value : 0;
        buf[6 * m + 2] = h->is_write ? 0 : 1;
        buf[6 * m + 3] = h->is_write ? 0 : h->value;
        buf[6 * m + 4] = h->start;
        buf[6 * m + 5] = h->end;
        m++;
      }
      (void)nall;
      n += (uint64_t)m;
      if (m == 0) continue;
      res = oracle_linearizable(buf, m);
      if (res < 0) { free(buf); return fail(PAXISIM_ENOMEM, "checker failed"); }
      a += (uint64_t)res;
    }
  }
  free(buf);
  *anomalies = a;
  if (ops) *ops = n;
  return 0;
}

/* Raw completed-operation history of one cluster: 5 words per op
 * {key, is_write, value, start, end}. */
int oracle_history(oracle_sim* s, uint64_t cl, uint32_t* buf, uint32_t cap_ops, uint32_t* n_out) {
  const cluster_t* c;
  uint32_t r, n = 0;
  if (!s || !n_out || cl >= s->C) return fail(PAXISIM_EINVAL, "bad argument");
  c = &s->cl[cl];
  for (r = 0; r < s->N; r++) {
    uint32_t j;
    for (j = 0; j < c->rep[r].nh; j++, n++)
      if (buf && n < cap_ops) memcpy(buf + 5 * (size_t)n, &c->rep[r].hist[j], sizeof(hist_t));
  }
  *n_out = n;
  return 0;
}

/* History.ReadFile (history.go:115-178): replace replica r's recorded ops of
 * one cluster, 5 words per op as oracle_history returns them. */
int oracle_history_load(oracle_sim* s, uint64_t cl, uint32_t r, const uint32_t* ops, uint32_t n) {
  uint32_t j;
  if (!s || (n && !ops) || cl >= s->C || r >= s->N) return fail(PAXISIM_EINVAL, "bad argument");
  if (s->cfg.protocol != PAXISIM_ABD) return fail(PAXISIM_EUNSUPP, "op history is kept by ABD only");
  if (n > s->cfg.history) return fail(PAXISIM_EINVAL, "%u ops exceed history capacity %u", n, s->cfg.history);
  for (j = 0; j < n; j++) memcpy(&s->cl[cl].rep[r].hist[j], ops + 5 * (size_t)j, sizeof(hist_t));
  s->cl[cl].rep[r].nh = n;
  return 0;
}

/* Database.Get of keys [0, n) of one replica (kv on; ABD: its KV). */
int oracle_read_kv(oracle_sim* s, uint64_t cl, uint32_t r, uint32_t* out, uint32_t n) {
  uint32_t k;
  if (!s || (n && !out) || cl >= s->C || r >= s->N || n > s->cfg.keys) return fail(PAXISIM_EINVAL, "bad argument");
  for (k = 0; k < n; k++) {
    const replica_t* p = &s->cl[cl].rep[r];
    if (s->cfg.protocol == PAXISIM_ABD) out[k] = p->kv_val[k];
    else if (s->kv) out[k] = p->db[k];
    else return fail(PAXISIM_EUNSUPP, "replicas keep no Database (config.kv = 0)");
  }
  return 0;
}

int oracle_read_client(oracle_sim* s, uint64_t cl, paxisim_worker_state* out, uint32_t cap, uint32_t* n_out) {
  uint32_t w, n;
  if (!s || !n_out || cl >= s->C || (cap && !out)) return fail(PAXISIM_EINVAL, "bad argument");
  n = s->wl.outstanding;
  for (w = 0; w < n && w < cap; w++) {
    out[w].cid = s->cl[cl].wk_cur[w];
    out[w].issued = s->cl[cl].wk_issued[w];
    out[w].reply_value = s->cl[cl].wk_rep[w];
    out[w].pad = 0;
  }
  *n_out = n;
  return 0;
}

/* The key and kind of command `cid` of a cluster (test support: the checker
 * recomputes a Database from an execution log). */
int oracle_command(oracle_sim* s, uint64_t cl, uint32_t cid, uint32_t* key, uint32_t* write) {
  if (!s || cl >= s->C || !cid) return fail(PAXISIM_EINVAL, "bad argument");
  if (key) *key = wl_key(s, s->cl[cl].kc, cid);
  if (write) *write = (uint32_t)wl_write(s, s->cl[cl].kc, cid);
  return 0;
}
