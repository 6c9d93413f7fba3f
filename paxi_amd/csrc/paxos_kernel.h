// paxos_kernel.h — Multi-Paxos handlers on gfx950 (a protocol policy of sim_core.h).
//
// One lane = one replica of one cluster.  The handlers follow
// paxos/paxos.go:86-376 and paxos/replica.go:42-66 (cited per function) and the
// node runtime's forward/reply routing node.go:79-172.
//
// Paxos state during a launch:
//   registers: ballot, slot, execute, active, phase-1 acks, pending/forward counts, digest
//   LDS:       log window {ballot, cmd|flags, acks} as [r][W][lane] u32 (regions a, b, c)
//   HBM:       request side table, pending/forward tables, digest checkpoints
#pragma once
#include "sim_core.h"

namespace pxs {

// ---------------------------------------------------------------------------
// log window in LDS: entry of slot s of replica r at [(r*W + (s & (W-1)))*64 + lane]
// ---------------------------------------------------------------------------
struct Ent { uint32_t b, c, a; };

template <int NT>
__device__ __forceinline__ uint32_t eidx(const Params& P, const Rep<NT>& x, int32_t s) {
  return x.e0 + ((uint32_t)s & (P.W - 1u)) * x.es;
}
template <int NT>
__device__ __forceinline__ Ent eget(const Rep<NT>& x, uint32_t i) { return Ent{x.l_a[i], x.l_b[i], x.l_c[i]}; }
template <int NT>
__device__ __forceinline__ void eput(Rep<NT>& x, uint32_t i, const Ent& e) {
  x.l_a[i] = e.b;
  x.l_b[i] = e.c;
  x.l_c[i] = e.a;
}
// request side table slot for LDS entry index i
template <int NT>
__device__ __forceinline__ uint32_t* reqx_at(const Params& P, const Rep<NT>& x, uint32_t i) {
  return &x.reqx[i];
}
template <int NT>
__device__ __forceinline__ uint32_t ereq(const Params& P, const Rep<NT>& x, uint32_t i, uint32_t c) {
  if (c & EF_REQSELF) return mkreq(c & CMD_MASK, PAXISIM_CLIENT_SRC);
  if (c & EF_REQEXT) return ldg(reqx_at(P, x, i));
  return 0u;
}
// attach request q to entry flags c (whose command is cmd)
template <int NT>
__device__ __forceinline__ uint32_t eset_req(const Params& P, const Rep<NT>& x, uint32_t i, uint32_t c, uint32_t q) {
  c &= ~(EF_REQSELF | EF_REQEXT);
  if (!q) return c;
  if (req_origin(q) == PAXISIM_CLIENT_SRC && req_cid(q) == (c & CMD_MASK)) return c | EF_REQSELF;
  *reqx_at(P, x, i) = q;
  return c | EF_REQEXT;
}
// replace the command of an entry, keeping its request (paxos.go:168-171)
template <int NT>
__device__ __forceinline__ uint32_t eset_cmd(const Params& P, const Rep<NT>& x, uint32_t i, uint32_t c, uint32_t cmd) {
  if ((c & EF_REQSELF) && (c & CMD_MASK) != cmd) {
    *reqx_at(P, x, i) = mkreq(c & CMD_MASK, PAXISIM_CLIENT_SRC);
    c = (c & ~EF_REQSELF) | EF_REQEXT;
  }
  return (c & ~CMD_MASK) | cmd;
}

// ---------------------------------------------------------------------------
// Request.Reply routing (node.go:83-97) and node.Forward (node.go:165-172)
// ---------------------------------------------------------------------------
template <int NT>
__device__ __forceinline__ void request_reply(const Params& P, Rep<NT>& x, uint32_t req, uint32_t reply_cmd) {
  const uint32_t o = req_origin(req);
  if (o == PAXISIM_CLIENT_SRC) client_reply<NT>(P, x, req_cid(req));
  else post_unicast<NT>(P, x, o, PAXISIM_MSG_REPLY, 0u, 0u, reply_cmd);
}

// node.Forward (node.go:165-172)
template <int NT>
__device__ __forceinline__ void node_forward(const Params& P, Rep<NT>& x, uint32_t to, uint32_t req) {
  const uint32_t cid = req_cid(req);
  uint32_t i = 0;
  for (; i < x.nfwd; i++)
    if (req_cid(ldg(&P.fwd[krc(P, i, x.r, x.c)])) == cid) break;
  if (i == x.nfwd) {
    if (x.nfwd == FMAX) x.flags |= PAXISIM_F_PEND_OVF | PAXISIM_F_UNFAITHFUL;
    else P.fwd[krc(P, x.nfwd++, x.r, x.c)] = req;
  } else {
    P.fwd[krc(P, i, x.r, x.c)] = req;
  }
  post_unicast<NT>(P, x, to, PAXISIM_MSG_REQUEST, 0u, 0u, cid);
}

// node.recv Reply case (node.go:83-90)
template <int NT>
__device__ __forceinline__ void handle_reply(const Params& P, Rep<NT>& x, uint32_t cid) {
  uint32_t i = 0;
  for (; i < x.nfwd; i++)
    if (req_cid(ldg(&P.fwd[krc(P, i, x.r, x.c)])) == cid) break;
  if (i == x.nfwd) {
    x.flags |= PAXISIM_F_UNFAITHFUL;
    return;
  }
  const uint32_t req = ldg(&P.fwd[krc(P, i, x.r, x.c)]);
  x.nfwd--;
  P.fwd[krc(P, i, x.r, x.c)] = ldg(&P.fwd[krc(P, x.nfwd, x.r, x.c)]);
  request_reply<NT>(P, x, req, cid);
}

// ---------------------------------------------------------------------------
// Multi-Paxos handlers
// ---------------------------------------------------------------------------
// WOVF / GHOST: raised on the replica and remembered per instance
template <int NT>
__device__ __forceinline__ void raise_win(Rep<NT>& x, uint32_t f) {
  x.flags |= f;
  x.iflags |= f & (PAXISIM_F_WOVF | PAXISIM_F_GHOST);
}

// Entries below execute ("ghosts").  exec() deletes an
// executed entry (paxos.go:366); update() (173-177), HandleP2a (254-258) and
// HandleP3 (326) re-create one when a message for an executed slot arrives,
// and Go keeps it.  Only HandleP2b (270-310) reads it: a P2b for the slot
// adopts a higher ballot, or panics on the nil quorum when the ballot is this
// replica's own and equals the entry's.  Such a P2b answers a P2a this replica
// sent while the slot was >= execute, so it arrives within 2 + 2*max_delay
// steps of the execution: a ghost lives that long after it is (re)created,
// in a per-instance table in HBM {slot, ballot, until | commit << 31} touched
// only on these paths.  iflags GHOST = the table may hold a live entry.
template <int NT>
__device__ __forceinline__ size_t gidx(const Params& P, const Rep<NT>& x, uint32_t g) {
  return ((size_t)g * P.NI + x.inst) * P.C + x.c;
}
template <int NT>
__device__ __forceinline__ uint32_t ghost_find(const Params& P, Rep<NT>& x, int32_t s, uint4& e) {
  if (!(x.iflags & PAXISIM_F_GHOST)) return GMAX;
  uint32_t live = 0, hit = GMAX;
  for (uint32_t g = 0; g < GMAX; g++) {
    const uint4 v = ldg(&P.gst[gidx<NT>(P, x, g)]);
    const bool l = (v.z & 0x7FFFFFFFu) > x.t;
    live |= l;
    if (l && v.x == (uint32_t)s && hit == GMAX) { e = v; hit = g; }
  }
  if (!live) x.iflags &= ~PAXISIM_F_GHOST;               // every ghost has expired
  return hit;
}
template <int NT>
__device__ __forceinline__ uint32_t ghost_alloc(const Params& P, Rep<NT>& x) {
  x.flags |= PAXISIM_F_GHOST;
  for (uint32_t g = 0; g < GMAX; g++) {
    const uint32_t until = ldg(&P.gst[gidx<NT>(P, x, g)]).z & 0x7FFFFFFFu;
    if (!(x.iflags & PAXISIM_F_GHOST) || until <= x.t) {
      x.iflags |= PAXISIM_F_GHOST;
      return g;
    }
  }
  x.flags |= PAXISIM_F_UNFAITHFUL;                       // cannot keep this ghost
  return GMAX;
}
template <int NT>
__device__ __forceinline__ uint32_t ghost_until(const Params& P, const Rep<NT>& x) {
  return x.t + 3u + 2u * P.max_delay;
}
// update() / HandleP2a on a slot below execute: create, or raise an uncommitted ballot
template <int NT>
__device__ __forceinline__ void ghost(const Params& P, Rep<NT>& x, int32_t s, uint32_t b) {
  uint4 e;
  uint32_t g = ghost_find<NT>(P, x, s, e);
  if (g < GMAX) {
    if (!(e.z >> 31) && b > e.y) P.gst[gidx<NT>(P, x, g)] = make_uint4(e.x, b, e.z, 0u);
    return;
  }
  if ((g = ghost_alloc<NT>(P, x)) < GMAX) P.gst[gidx<NT>(P, x, g)] = make_uint4((uint32_t)s, b, ghost_until<NT>(P, x), 0u);
}
// HandleP3 on a slot below execute: the entry exists and is committed (paxos.go:326-331)
template <int NT>
__device__ __forceinline__ void ghost_commit(const Params& P, Rep<NT>& x, int32_t s) {
  uint4 e;
  uint32_t g = ghost_find<NT>(P, x, s, e);
  if (g < GMAX) {
    P.gst[gidx<NT>(P, x, g)] = make_uint4(e.x, e.y, e.z | 0x80000000u, 0u);
    return;
  }
  if ((g = ghost_alloc<NT>(P, x)) < GMAX)
    P.gst[gidx<NT>(P, x, g)] = make_uint4((uint32_t)s, 0u, ghost_until<NT>(P, x) | 0x80000000u, 0u);
}
// HandleP2b (paxos.go:270-310) for a slot below execute
template <int NT>
__device__ __forceinline__ void ghost_p2b(const Params& P, Rep<NT>& x, int32_t ms, uint32_t mb) {
  uint4 e;
  if (ghost_find<NT>(P, x, ms, e) == GMAX || mb < e.y || (e.z >> 31)) return;
  if (mb > x.ballot) {
    x.ballot = mb;
    x.active = 0;
  }
  if (bal_id(mb) == x.r && mb == e.y) {                  // nil quorum: Go panics
    x.flags |= PAXISIM_F_POISON;
    x.stop = true;
  }
}

template <int NT>
__device__ __forceinline__ bool in_window(const Params& P, const Rep<NT>& x, int32_t s) {
  return s >= x.execute && s < x.execute + (int32_t)P.W;
}

template <int NT>
__device__ __forceinline__ void paxos_forward(const Params& P, Rep<NT>& x) {     // paxos.go:371-376
  for (uint32_t i = 0; i < x.npend; i++) node_forward<NT>(P, x, bal_id(x.ballot), ldg(&x.pend[(size_t)i * x.pstride]));
  x.npend = 0;
}

template <int NT>
__device__ __forceinline__ void paxos_p1a(const Params& P, Rep<NT>& x) {      // paxos.go:100-108
  if (x.active) return;
  if ((x.ballot >> 4) + 1u >= (1u << 27)) x.flags |= PAXISIM_F_BALLOT_OVF | PAXISIM_F_UNFAITHFUL;
  x.ballot = bal_next(x.ballot, x.r);
  x.p1mask = 1u << x.r;
  post_broadcast<NT>(P, x, PAXISIM_MSG_P1A | x.ktag, x.ballot, 0u, 0u);
}

template <int NT>
__device__ __forceinline__ void paxos_p2a(const Params& P, Rep<NT>& x, uint32_t req) {  // paxos.go:111-131
  x.slot++;
  const uint32_t cid = req_cid(req);
  if (in_window<NT>(P, x, x.slot)) {
    const uint32_t i = eidx<NT>(P, x, x.slot);
    const uint32_t c = eset_req<NT>(P, x, i, cid | EF_EXISTS | EF_QUORUM, req);
    eput<NT>(x, i, Ent{x.ballot, c, 1u << x.r});
  } else {
    raise_win(x, PAXISIM_F_WOVF | PAXISIM_F_UNFAITHFUL);
  }
  if (P.thrifty) {                                   // MulticastQuorum(N/2+1) (socket.go:132-145), ring order
    const uint32_t N = nrep<NT>(P);
    uint32_t sent = 0;
    intent_flush<NT>(P, x);
#pragma nounroll
    for (uint32_t i = 1; i < N && sent < N / 2 + 1; i++, sent++)
      send1<NT>(P, x, (x.r + i) % N, PAXISIM_MSG_P2A | x.ktag, x.ballot, (uint32_t)x.slot, cid);
  } else {
    post_broadcast<NT>(P, x, PAXISIM_MSG_P2A | x.ktag, x.ballot, (uint32_t)x.slot, cid);
  }
}

template <int NT>
__device__ __forceinline__ void paxos_handle_request(const Params& P, Rep<NT>& x, uint32_t req) {  // paxos.go:86-97
  if (!x.active) {
    if (x.npend == PMAX) x.flags |= PAXISIM_F_PEND_OVF | PAXISIM_F_UNFAITHFUL;
    else x.pend[(size_t)x.npend++ * x.pstride] = req;
    if (bal_id(x.ballot) != x.r) paxos_p1a<NT>(P, x);
  } else {
    paxos_p2a<NT>(P, x, req);
  }
}

template <int NT>
__device__ __forceinline__ void handle_request(const Params& P, Rep<NT>& x, uint32_t req) {  // replica.go:42-66
  const bool leader = x.active || bal_id(x.ballot) == x.r;
  if (P.ephemeral || leader || x.ballot == 0) paxos_handle_request<NT>(P, x, req);
  else node_forward<NT>(P, x, bal_id(x.ballot), req);
}

// Agreement ring (client.go:279-320 Consensus, restated as a running check):
// the first replica to reach digest checkpoint k records it, every later one
// compares (a 64-bit CAS, so concurrent arrivals in one step agree on who was
// first; whether some pair disagrees does not depend on that order).
static __device__ __noinline__ void agree_arrive(unsigned long long* a, uint32_t* st0, size_t sstride, uint32_t k,
                                         uint64_t digest) {
  const unsigned long long want = ((unsigned long long)k << 40) | ((digest ^ (digest >> 24)) & 0xFFFFFFFFFFull);
  unsigned long long v = atomicCAS(a, 0ull, want);
  uint32_t st = 0;                                       // 0: first to arrive, recorded
  while (v != 0ull) {
    const uint32_t tv = (uint32_t)(v >> 40);
    if (tv == k) { st = v == want ? ST_AGC : ST_AGB; break; }
    if (tv > k) { st = ST_AGM; break; }                  // the first digest has left the ring
    const unsigned long long o = atomicCAS(a, v, want);  // an older checkpoint: claim the slot
    if (o == v) break;
    v = o;
  }
  if (st == ST_AGB) st0[ST_AGC * sstride] += 1;          // a mismatch was compared too
  if (st) st0[st * sstride] += 1;
}

// Database.Execute (db.go:103-114) when replicas keep the KV: a write's value
// (its command id) goes to its key and database.version counts it (put,
// db.go:123-134); a read changes nothing.  The previous value Execute returns
// is what the key holds at this point of the executed log.
template <int NT>
__device__ __forceinline__ void kv_exec(const Params& P, Rep<NT>& x, uint32_t cmd) {
  if (!wl_write(P, x.kc, cmd)) return;
  P.kv_val[((size_t)wl_key(P, x.kc, cmd) * nrep<NT>(P) + x.r) * P.C + x.c] = cmd;
  x.kvver++;
}

template <int NT>
__device__ __forceinline__ void paxos_exec(const Params& P, Rep<NT>& x) {     // paxos.go:345-369
  for (;;) {
    const uint32_t i = eidx<NT>(P, x, x.execute);
    const uint32_t c = x.l_b[i];
    if ((c & (EF_EXISTS | EF_COMMIT)) != (EF_EXISTS | EF_COMMIT)) break;
    if (x.iflags & PAXISIM_F_WOVF) x.flags |= PAXISIM_F_UNFAITHFUL;
    const uint32_t cmd = c & CMD_MASK;
    if (c & (EF_REQSELF | EF_REQEXT)) request_reply<NT>(P, x, ereq<NT>(P, x, i, c), cmd);
    x.digest = mix64(x.digest ^ (((uint64_t)(uint32_t)x.execute << 32) | cmd));
    if (P.kv) kv_exec<NT>(P, x, cmd);                              // p.Execute(e.command), paxos.go:352
    x.l_b[i] = 0u;                                                 // delete(p.log, execute)
    x.execute++;
    if ((uint32_t)x.execute % CKI == 0) {
      const uint32_t k = ((uint32_t)x.execute / CKI) % CKR;
      const size_t ci = ((size_t)k * P.NI + x.inst) * P.C + x.c;
      P.ck_e[ci] = (uint32_t)x.execute;
      P.ck_d[ci] = x.digest;
      if (P.AR) {
        const uint32_t kk = (uint32_t)x.execute / CKI;
        agree_arrive(&P.agr[((size_t)(kk % P.AR) * P.NK + x.key) * P.C + x.c], &P.stats[rc(P, x.r, x.c)],
                     (size_t)P.N * P.C, kk, x.digest);
      }
    }
  }
}

template <int NT>
__device__ __forceinline__ void paxos_handle_p1a(const Params& P, Rep<NT>& x, uint32_t mb) {  // paxos.go:134-162
  if (mb > x.ballot) {
    x.ballot = mb;
    x.active = 0;
    paxos_forward<NT>(P, x);
  }
  if (x.iflags & PAXISIM_F_WOVF) x.flags |= PAXISIM_F_UNFAITHFUL;
  int32_t hi = x.slot;
  if (hi > x.execute + (int32_t)P.W - 1) hi = x.execute + (int32_t)P.W - 1;
  uint32_t n = 0;
  for (int32_t s = x.execute; s <= hi; s++) {
    const uint32_t c = x.l_b[eidx<NT>(P, x, s)];
    n += (c & EF_EXISTS) && !(c & EF_COMMIT);
  }
  uint32_t ri;
  intent_flush<NT>(P, x);                                                    // keep per-link order
  if (!send_begin<NT>(P, x, bal_id(mb), 1u + n, ri)) return;
  x.rec[ri] = make_uint4(PAXISIM_MSG_P1B | (n << 8) | x.ktag, x.ballot, 0u, 0u);
  for (int32_t s = x.execute; s <= hi; s++) {
    const Ent e = eget<NT>(x, eidx<NT>(P, x, s));
    if (!(e.c & EF_EXISTS) || (e.c & EF_COMMIT)) continue;
    ri += LANES;
    x.rec[ri] = make_uint4(PAXISIM_MSG_P1B_ENTRY, e.b, (uint32_t)s, e.c & CMD_MASK);
  }
}

// P1b with its CommandBallot payload in the records after ri0
template <int NT>
__device__ __forceinline__ void paxos_handle_p1b(const Params& P, Rep<NT>& x, uint32_t src, uint32_t mb, uint32_t ri0,
                                              uint32_t n) {                   // paxos.go:164-230
  if (mb < x.ballot || x.active) return;
  for (uint32_t k = 0; k < n; k++) {                                          // update(): 164-180
    const uint4 cb = ldg(&x.rec[ri0 + (k + 1u) * LANES]);
    const int32_t s = (int32_t)cb.z;
    if (s > x.slot) x.slot = s;
    if (in_window<NT>(P, x, s)) {
      const uint32_t i = eidx<NT>(P, x, s);
      Ent e = eget<NT>(x, i);
      if (e.c & EF_EXISTS) {
        if (!(e.c & EF_COMMIT) && cb.y > e.b) {
          e.b = cb.y;
          e.c = eset_cmd<NT>(P, x, i, e.c, cb.w);
          eput<NT>(x, i, e);
        }
      } else {
        eput<NT>(x, i, Ent{cb.y, cb.w | EF_EXISTS, 0u});                      // quorum nil
      }
    } else if (s < x.execute) {
      ghost<NT>(P, x, s, cb.y);
    } else {
      raise_win(x, PAXISIM_F_WOVF);
    }
  }
  if (mb > x.ballot) {
    x.ballot = mb;
    x.active = 0;
    paxos_forward<NT>(P, x);
  }
  if (bal_id(mb) == x.r && mb == x.ballot) {
    x.p1mask |= 1u << src;
    if (quorum_ok(P, P.q1, x.p1mask)) {
      x.active = 1;
      if (x.iflags & PAXISIM_F_WOVF) x.flags |= PAXISIM_F_UNFAITHFUL;
      int32_t hi = x.slot;
      if (hi > x.execute + (int32_t)P.W - 1) hi = x.execute + (int32_t)P.W - 1;
      for (int32_t s = x.execute; s <= hi; s++) {
        const uint32_t i = eidx<NT>(P, x, s);
        const uint32_t c = x.l_b[i];
        if (!(c & EF_EXISTS) || (c & EF_COMMIT)) continue;                   // nil gap (G5)
        x.l_a[i] = x.ballot;
        x.l_b[i] = c | EF_QUORUM;
        x.l_c[i] = 1u << x.r;
        post_broadcast<NT>(P, x, PAXISIM_MSG_P2A | x.ktag, x.ballot, (uint32_t)s, c & CMD_MASK);
      }
      const uint32_t np = x.npend;
      x.npend = 0;
      for (uint32_t k = 0; k < np; k++) paxos_p2a<NT>(P, x, ldg(&x.pend[(size_t)k * x.pstride]));
    }
  }
}

template <int NT>
__device__ __forceinline__ void paxos_handle_p2a(const Params& P, Rep<NT>& x, uint32_t mb, int32_t ms,
                                                 uint32_t mcid) {             // paxos.go:233-267
  if (mb >= x.ballot) {
    x.ballot = mb;
    x.active = 0;
    if (ms > x.slot) x.slot = ms;
    if (in_window<NT>(P, x, ms)) {
      const uint32_t i = eidx<NT>(P, x, ms);
      Ent e = eget<NT>(x, i);
      if (e.c & EF_EXISTS) {
        if (!(e.c & EF_COMMIT) && mb > e.b) {
          if ((e.c & CMD_MASK) != mcid && (e.c & (EF_REQSELF | EF_REQEXT))) {
            node_forward<NT>(P, x, bal_id(mb), ereq<NT>(P, x, i, e.c));
            e.c &= ~(EF_REQSELF | EF_REQEXT);
          }
          e.c = eset_cmd<NT>(P, x, i, e.c, mcid);
          e.b = mb;
          x.l_a[i] = e.b;
          x.l_b[i] = e.c;
        }
      } else {
        eput<NT>(x, i, Ent{mb, mcid | EF_EXISTS, 0u});
      }
    } else if (ms < x.execute) {
      ghost<NT>(P, x, ms, mb);
    } else {
      raise_win(x, PAXISIM_F_WOVF);
    }
  }
  post_unicast<NT>(P, x, bal_id(mb), PAXISIM_MSG_P2B | x.ktag, x.ballot, (uint32_t)ms, 0u);
}

template <int NT>
__device__ __forceinline__ void paxos_handle_p2b(const Params& P, Rep<NT>& x, uint32_t src, uint32_t mb,
                                                 int32_t ms) {                // paxos.go:270-310
  if (!in_window<NT>(P, x, ms)) {
    if (ms < x.execute) ghost_p2b<NT>(P, x, ms, mb);
    else if (x.iflags & PAXISIM_F_WOVF) x.flags |= PAXISIM_F_UNFAITHFUL;
    return;
  }
  const uint32_t i = eidx<NT>(P, x, ms);
  const uint32_t c = x.l_b[i];
  const uint32_t eb = x.l_a[i];
  if (!(c & EF_EXISTS) || mb < eb || (c & EF_COMMIT)) return;
  if (mb > x.ballot) {
    x.ballot = mb;
    x.active = 0;
  }
  if (bal_id(mb) == x.r && mb == eb) {
    if (!(c & EF_QUORUM)) {                                                   // nil quorum: Go panics
      x.flags |= PAXISIM_F_POISON;
      x.stop = true;
      return;
    }
    const uint32_t ack = x.l_c[i] | (1u << src);
    x.l_c[i] = ack;
    if (quorum_ok(P, P.q2, ack)) {
      x.l_b[i] = c | EF_COMMIT;
      x.commits++;
      post_broadcast<NT>(P, x, PAXISIM_MSG_P3 | x.ktag, mb, (uint32_t)ms, c & CMD_MASK);
      if (P.rwc) {
        const uint32_t q = ereq<NT>(P, x, i, c);
        if (!q) { x.flags |= PAXISIM_F_POISON; x.stop = true; return; }   // nil r.Reply
        request_reply<NT>(P, x, q, req_cid(q));
      } else {
        paxos_exec<NT>(P, x);
      }
    }
  }
}

template <int NT>
__device__ __forceinline__ void paxos_handle_p3(const Params& P, Rep<NT>& x, uint32_t mb, int32_t ms,
                                                uint32_t mcid) {              // paxos.go:313-343
  if (ms > x.slot) x.slot = ms;
  if (in_window<NT>(P, x, ms)) {
    const uint32_t i = eidx<NT>(P, x, ms);
    uint32_t c = x.l_b[i];
    if (c & EF_EXISTS) {
      if ((c & CMD_MASK) != mcid && (c & (EF_REQSELF | EF_REQEXT))) {
        node_forward<NT>(P, x, bal_id(mb), ereq<NT>(P, x, i, c));
        c &= ~(EF_REQSELF | EF_REQEXT);
      }
    } else {
      c = EF_EXISTS;                                                          // &entry{} (G6)
      x.l_a[i] = 0u;
      x.l_c[i] = 0u;
    }
    c = eset_cmd<NT>(P, x, i, c, mcid) | EF_COMMIT;
    x.l_b[i] = c;
    if (P.rwc) {
      if (c & (EF_REQSELF | EF_REQEXT)) {
        const uint32_t q = ereq<NT>(P, x, i, c);
        request_reply<NT>(P, x, q, req_cid(q));
      }
      return;
    }
  } else if (ms < x.execute) {
    ghost_commit<NT>(P, x, ms);
  } else {
    raise_win(x, PAXISIM_F_WOVF);
  }
  if (!P.rwc) paxos_exec<NT>(P, x);
}

// ---------------------------------------------------------------------------
// protocol policy
// ---------------------------------------------------------------------------
struct PaxosProto {
  static constexpr uint32_t kind = PAXISIM_PAXOS;
  template <int NT>
  __device__ static __forceinline__ void load(const Params& P, Rep<NT>& x) {
    const size_t i = rc(P, x.r, x.c);
    x.ballot = P.ballot[i];
    x.slot = (int32_t)P.slot[i];
    x.execute = (int32_t)P.execute[i];
    const uint32_t meta = P.meta[i];
    x.active = meta & 1u;
    x.p1mask = meta >> 16;
    x.npend = P.npend[i];
    x.nfwd = P.nfwd[i];
    x.digest = P.digest[i];
    // the replica's one instance: LDS log window [r][W][lane], SoA pending table
    x.iflags = x.flags & (PAXISIM_F_WOVF | PAXISIM_F_GHOST);
    x.inst = x.r;
    x.key = 0;
    x.ktag = 0;
    x.e0 = ((x.r * P.W) << 6) | x.lane;
    x.es = LANES;
    x.reqx = P.reqx + (size_t)x.blk * (P.N * P.W * LANES);
    x.pend = P.pend + i;
    x.pstride = P.NI * (uint32_t)P.C;
  }
  template <int NT>
  __device__ static __forceinline__ void store(const Params& P, const Rep<NT>& x) {
    const size_t i = rc(P, x.r, x.c);
    P.ballot[i] = x.ballot;
    P.slot[i] = (uint32_t)x.slot;
    P.execute[i] = (uint32_t)x.execute;
    P.meta[i] = (x.active & 1u) | (x.p1mask << 16);
    P.npend[i] = x.npend;
    P.nfwd[i] = x.nfwd;
    P.digest[i] = x.digest;
  }
  template <int NT>
  __device__ static __forceinline__ void client_request(const Params& P, Rep<NT>& x, uint32_t cid) {
    handle_request<NT>(P, x, mkreq(cid, PAXISIM_CLIENT_SRC));
  }
  // HandleP2b (paxos.go:270-310) for a P2b that neither completes a quorum
  // nor poisons: returns true after applying it exactly as paxos_handle_p2b
  // would (ignored: no entry (G7), m.Ballot < e.ballot, committed, or outside
  // the window where no flag can be raised; else adopt a higher ballot and
  // record the ack).  Returns false, with no effect, for every other message.
  template <int NT>
  __device__ static __forceinline__ bool absorb(const Params& P, Rep<NT>& x, uint32_t src, const uint4& m) {
    if (hdr_type(m.x) != PAXISIM_MSG_P2B) return false;
    const int32_t ms = (int32_t)m.z;
    const uint32_t mb = m.y;
    if (!in_window<NT>(P, x, ms))
      return ms < x.execute ? !(x.iflags & PAXISIM_F_GHOST) : !(x.iflags & PAXISIM_F_WOVF);
    const uint32_t i = eidx<NT>(P, x, ms);
    const uint32_t c = x.l_b[i];
    const uint32_t eb = x.l_a[i];
    if (!(c & EF_EXISTS) || mb < eb || (c & EF_COMMIT)) return true;
    if (bal_id(mb) == x.r && mb == eb) {
      if (!(c & EF_QUORUM)) return false;                 // nil quorum: the full handler poisons
      const uint32_t ack = x.l_c[i] | (1u << src);
      if (quorum_ok(P, P.q2, ack)) return false;          // commit: the full handler
      x.l_c[i] = ack;
    }
    if (mb > x.ballot) {
      x.ballot = mb;
      x.active = 0;
    }
    return true;
  }
  // node.handle dispatch (node.go:104-115; registrations paxos/replica.go:33-38)
  template <int NT>
  __device__ static __forceinline__ void dispatch(const Params& P, Rep<NT>& x, uint32_t src, const uint4& m,
                                                  uint32_t ri) {
    switch (hdr_type(m.x)) {
      case PAXISIM_MSG_REQUEST: dv_inc<NT>(x, PAXISIM_MSG_REQUEST); handle_request<NT>(P, x, mkreq(m.w, src)); break;
      case PAXISIM_MSG_REPLY: dv_inc<NT>(x, PAXISIM_MSG_REPLY); handle_reply<NT>(P, x, m.w); break;
      case PAXISIM_MSG_P1A: dv_inc<NT>(x, PAXISIM_MSG_P1A); paxos_handle_p1a<NT>(P, x, m.y); break;
      case PAXISIM_MSG_P1B: dv_inc<NT>(x, PAXISIM_MSG_P1B); paxos_handle_p1b<NT>(P, x, src, m.y, ri, hdr_n(m.x)); break;
      case PAXISIM_MSG_P2A: dv_inc<NT>(x, PAXISIM_MSG_P2A); paxos_handle_p2a<NT>(P, x, m.y, (int32_t)m.z, m.w); break;
      case PAXISIM_MSG_P2B: dv_inc<NT>(x, PAXISIM_MSG_P2B); paxos_handle_p2b<NT>(P, x, src, m.y, (int32_t)m.z); break;
      case PAXISIM_MSG_P3: dv_inc<NT>(x, PAXISIM_MSG_P3); paxos_handle_p3<NT>(P, x, m.y, (int32_t)m.z, m.w); break;
      default: break;
    }
  }
};

}  // namespace pxs
