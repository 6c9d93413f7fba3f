// paxos_kernel.h — Multi-Paxos replica step on gfx950 (LDS-resident workgroup).
//
// One lane = one replica of one cluster.  The handlers follow
// paxos/paxos.go:86-376 and paxos/replica.go:42-66 (cited per function), the
// socket filter socket.go:66-109 and the node runtime node.go:79-172, under
// the delivery schedule of DESIGN.md §3.
//
// Memory map during a launch:
//   registers: replica scalars (ballot, slot, execute, active, p1 acks, flags,
//              digest, counters) and the socket fault state of the N links
//   LDS:       log windows {ballot, cmd|flags, acks} [r][W][lane], mailbox
//              counts [bucket][dst][src][lane], client workers, poison step
//   HBM:       message records (block-contiguous, prefetched one ahead),
//              request side table, pending/forward tables, checkpoints
#pragma once
#include "paxisim_dev.h"

namespace pxs {

template <int NT>
struct Rep {
  static constexpr uint32_t NL = NT ? (uint32_t)NT : (uint32_t)PAXISIM_MAX_N;  // link registers
  uint64_t c, gid;                      // global lane / cluster id
  uint32_t lane, r, t, b0, hs, kc, blk;
  uint32_t ballot;
  int32_t slot, execute;
  uint32_t active, p1mask, flags, npend, nfwd;
  uint64_t digest;
  uint32_t du[NL], su[NL];              // link fault state: drop_until; slow_until | delay << 28
  uint32_t dv[9];                       // delivered by type (REQUEST..P3)
  uint32_t client, sent, dropped, discarded, commits, replies;
  uint32_t send_seq;
  bool stop, crashed;
  // LDS views
  uint32_t *l_bal, *l_cmd, *l_ack, *l_wcur, *l_wiss, *l_poison;
  uint8_t* l_cnt;
  uint4* rec;                           // this block's record region
};

template <int NT>
__device__ __forceinline__ uint32_t nrep(const Params& P) { return NT ? (uint32_t)NT : P.N; }

// register-array select / update with a runtime index (unrolled: no scratch)
// (the empty asm keeps LLVM from folding the select chain back into an
// alloca + dynamic index, which would put the array in scratch memory)
__device__ __forceinline__ uint32_t opaque(uint32_t v) {
  asm volatile("" : "+v"(v));
  return v;
}
template <int NT>
__device__ __forceinline__ uint32_t lsel(const uint32_t (&a)[Rep<NT>::NL], uint32_t i) {
  uint32_t v = opaque(a[0]);
#pragma unroll
  for (uint32_t k = 1; k < Rep<NT>::NL; k++) v = (i == k) ? opaque(a[k]) : v;
  return v;
}

// ---------------------------------------------------------------------------
// log window in LDS: entry of slot s of replica r at [(r*W + (s & (W-1)))*64 + lane]
// ---------------------------------------------------------------------------
struct Ent { uint32_t b, c, a; };

template <int NT>
__device__ __forceinline__ uint32_t eidx(const Params& P, const Rep<NT>& x, int32_t s) {
  return ((x.r * P.W + ((uint32_t)s & (P.W - 1u))) << 6) | x.lane;
}
template <int NT>
__device__ __forceinline__ Ent eget(const Rep<NT>& x, uint32_t i) { return Ent{x.l_bal[i], x.l_cmd[i], x.l_ack[i]}; }
template <int NT>
__device__ __forceinline__ void eput(Rep<NT>& x, uint32_t i, const Ent& e) {
  x.l_bal[i] = e.b;
  x.l_cmd[i] = e.c;
  x.l_ack[i] = e.a;
}
// request side table slot for LDS entry index i
template <int NT>
__device__ __forceinline__ uint32_t* reqx_at(const Params& P, const Rep<NT>& x, uint32_t i) {
  return &P.reqx[(size_t)x.blk * (P.N * P.W * LANES) + i];
}
template <int NT>
__device__ __forceinline__ uint32_t ereq(const Params& P, const Rep<NT>& x, uint32_t i, uint32_t c) {
  if (c & EF_REQSELF) return mkreq(c & CMD_MASK, PAXISIM_CLIENT_SRC);
  if (c & EF_REQEXT) return *reqx_at(P, x, i);
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
// socket.Send (socket.go:66-109): crash -> drop -> flaky -> slow, then the
// bounded (link, arrival-step) bucket.  Returns the record index to write.
// ---------------------------------------------------------------------------
template <int NT>
__device__ __forceinline__ bool send_begin(const Params& P, Rep<NT>& x, uint32_t to, uint32_t nrec, uint32_t& ri) {
  const uint32_t N = nrep<NT>(P);
  const uint32_t seq = x.send_seq++;
  x.sent++;
  if (to >= N || x.crashed) { x.dropped++; return false; }
  if (x.t < lsel<NT>(x.du, to) || (P.nfaults && scripted(P, PAXISIM_FAULT_DROP, x.gid, x.r, to, x.t, nullptr))) {
    x.dropped++;
    return false;
  }
  uint32_t delay = 0;
  if (P.nfaults) {
    uint32_t p = 0;
    if (scripted(P, PAXISIM_FAULT_FLAKY, x.gid, x.r, to, x.t, &p) && p > 0 &&
        ppm_hit(draw(x.hs, tag(PUR_FLAKY, x.r, seq)), p)) {
      x.dropped++;
      return false;
    }
  }
  const uint32_t su = lsel<NT>(x.su, to);
  if (x.t < (su & (T_MAX - 1u))) delay = su >> 28;
  if (P.nfaults) scripted(P, PAXISIM_FAULT_SLOW, x.gid, x.r, to, x.t, &delay);
  if (delay > P.max_delay) delay = P.max_delay;
  uint32_t b = x.b0 + 1u + delay;
  if (b >= P.D) b -= P.D;
  const uint32_t box = (b * N + to) * P.NS + x.r;
  uint8_t* cp = &x.l_cnt[(box << 6) | x.lane];
  const uint32_t k = *cp;
  if (k + nrec > P.M) {
    x.flags |= PAXISIM_F_MBOX_OVF | PAXISIM_F_UNFAITHFUL;
    x.dropped++;
    return false;
  }
  *cp = (uint8_t)(k + nrec);
  ri = ((box * P.M + k) << 6) | x.lane;
  return true;
}

template <int NT>
__device__ __forceinline__ void send1(const Params& P, Rep<NT>& x, uint32_t to, uint32_t type, uint32_t ballot,
                                      uint32_t slot, uint32_t cid) {
  uint32_t ri;
  if (send_begin<NT>(P, x, to, 1, ri)) x.rec[ri] = make_uint4(type, ballot, slot, cid);
}

// Broadcast: every peer except self, IDs.Less order (socket.go:147-155; G1, G2)
template <int NT>
__device__ __forceinline__ void broadcast1(const Params& P, Rep<NT>& x, uint32_t type, uint32_t ballot,
                                           uint32_t slot, uint32_t cid) {
  const uint32_t N = nrep<NT>(P);
#pragma nounroll
  for (uint32_t d = 0; d < N; d++)
    if (d != x.r) send1<NT>(P, x, d, type, ballot, slot, cid);
}

// ---------------------------------------------------------------------------
// client (benchmark.go:246-275) and Request.Reply routing (node.go:83-97)
// ---------------------------------------------------------------------------
template <int NT>
__device__ __forceinline__ void client_reply(const Params& P, Rep<NT>& x, uint32_t cid) {
  const uint32_t w = (cid - 1u) % P.WK;
  const uint32_t wi = (w << 6) | x.lane;
  if (x.l_wcur[wi] != cid) return;              // duplicate reply: the worker moved on
  x.replies++;
  const uint32_t issued = x.l_wiss[wi];
  if (P.max_requests == 0 || issued < P.max_requests) {
    const uint64_t nc = 1ull + w + (uint64_t)P.WK * issued;
    if (nc > CMD_MASK) {
      x.flags |= PAXISIM_F_PEND_OVF | PAXISIM_F_UNFAITHFUL;
      x.l_wcur[wi] = 0;
      return;
    }
    x.l_wiss[wi] = issued + 1u;
    x.l_wcur[wi] = (uint32_t)nc;
    // the next request reaches the worker's target next step (client source N)
    uint32_t b = x.b0 + 1u;
    if (b >= P.D) b -= P.D;
    const uint32_t box = (b * nrep<NT>(P) + P.target[w]) * P.NS + nrep<NT>(P);
    uint8_t* cp = &x.l_cnt[(box << 6) | x.lane];
    const uint32_t k = *cp;
    if (k >= P.M) {
      x.flags |= PAXISIM_F_MBOX_OVF | PAXISIM_F_UNFAITHFUL;
      return;
    }
    x.rec[((box * P.M + k) << 6) | x.lane] = make_uint4(PAXISIM_MSG_REQUEST, 0u, 0u, (uint32_t)nc);
    *cp = (uint8_t)(k + 1u);
  } else {
    x.l_wcur[wi] = 0;
  }
}

template <int NT>
__device__ __forceinline__ void request_reply(const Params& P, Rep<NT>& x, uint32_t req, uint32_t reply_cmd) {
  const uint32_t o = req_origin(req);
  if (o == PAXISIM_CLIENT_SRC) client_reply<NT>(P, x, req_cid(req));
  else send1<NT>(P, x, o, PAXISIM_MSG_REPLY, 0u, 0u, reply_cmd);
}

// node.Forward (node.go:165-172)
template <int NT>
__device__ __forceinline__ void node_forward(const Params& P, Rep<NT>& x, uint32_t to, uint32_t req) {
  const uint32_t cid = req_cid(req);
  uint32_t i = 0;
  for (; i < x.nfwd; i++)
    if (req_cid(P.fwd[krc(P, i, x.r, x.c)]) == cid) break;
  if (i == x.nfwd) {
    if (x.nfwd == FMAX) x.flags |= PAXISIM_F_PEND_OVF | PAXISIM_F_UNFAITHFUL;
    else P.fwd[krc(P, x.nfwd++, x.r, x.c)] = req;
  } else {
    P.fwd[krc(P, i, x.r, x.c)] = req;
  }
  send1<NT>(P, x, to, PAXISIM_MSG_REQUEST, 0u, 0u, cid);
}

// node.recv Reply case (node.go:83-90)
template <int NT>
__device__ __forceinline__ void handle_reply(const Params& P, Rep<NT>& x, uint32_t cid) {
  uint32_t i = 0;
  for (; i < x.nfwd; i++)
    if (req_cid(P.fwd[krc(P, i, x.r, x.c)]) == cid) break;
  if (i == x.nfwd) {
    x.flags |= PAXISIM_F_UNFAITHFUL;
    return;
  }
  const uint32_t req = P.fwd[krc(P, i, x.r, x.c)];
  x.nfwd--;
  P.fwd[krc(P, i, x.r, x.c)] = P.fwd[krc(P, x.nfwd, x.r, x.c)];
  request_reply<NT>(P, x, req, cid);
}

// ---------------------------------------------------------------------------
// Multi-Paxos handlers
// ---------------------------------------------------------------------------
template <int NT>
__device__ __forceinline__ bool in_window(const Params& P, const Rep<NT>& x, int32_t s) {
  return s >= x.execute && s < x.execute + (int32_t)P.W;
}

template <int NT>
__device__ __forceinline__ void paxos_forward(const Params& P, Rep<NT>& x) {     // paxos.go:371-376
  for (uint32_t i = 0; i < x.npend; i++) node_forward<NT>(P, x, bal_id(x.ballot), P.pend[krc(P, i, x.r, x.c)]);
  x.npend = 0;
}

template <int NT>
__device__ __forceinline__ void paxos_p1a(const Params& P, Rep<NT>& x) {      // paxos.go:100-108
  if (x.active) return;
  if ((x.ballot >> 4) + 1u >= (1u << 27)) x.flags |= PAXISIM_F_BALLOT_OVF | PAXISIM_F_UNFAITHFUL;
  x.ballot = bal_next(x.ballot, x.r);
  x.p1mask = 1u << x.r;
  broadcast1<NT>(P, x, PAXISIM_MSG_P1A, x.ballot, 0u, 0u);
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
    x.flags |= PAXISIM_F_WOVF | PAXISIM_F_UNFAITHFUL;
  }
  if (P.thrifty) {                                   // MulticastQuorum(N/2+1) (socket.go:132-145)
    const uint32_t N = nrep<NT>(P);
    uint32_t sent = 0;
#pragma nounroll
    for (uint32_t i = 1; i < N && sent < N / 2 + 1; i++, sent++)
      send1<NT>(P, x, (x.r + i) % N, PAXISIM_MSG_P2A, x.ballot, (uint32_t)x.slot, cid);
  } else {
    broadcast1<NT>(P, x, PAXISIM_MSG_P2A, x.ballot, (uint32_t)x.slot, cid);
  }
}

template <int NT>
__device__ __forceinline__ void paxos_handle_request(const Params& P, Rep<NT>& x, uint32_t req) {  // paxos.go:86-97
  if (!x.active) {
    if (x.npend == PMAX) x.flags |= PAXISIM_F_PEND_OVF | PAXISIM_F_UNFAITHFUL;
    else P.pend[krc(P, x.npend++, x.r, x.c)] = req;
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

template <int NT>
__device__ __forceinline__ void paxos_exec(const Params& P, Rep<NT>& x) {     // paxos.go:345-369
  for (;;) {
    const uint32_t i = eidx<NT>(P, x, x.execute);
    const uint32_t c = x.l_cmd[i];
    if ((c & (EF_EXISTS | EF_COMMIT)) != (EF_EXISTS | EF_COMMIT)) break;
    if (x.flags & PAXISIM_F_WOVF) x.flags |= PAXISIM_F_UNFAITHFUL;
    const uint32_t cmd = c & CMD_MASK;
    if (c & (EF_REQSELF | EF_REQEXT)) request_reply<NT>(P, x, ereq<NT>(P, x, i, c), cmd);
    x.digest = mix64(x.digest ^ (((uint64_t)(uint32_t)x.execute << 32) | cmd));
    x.l_cmd[i] = 0u;                                                 // delete(p.log, execute)
    x.execute++;
    if ((uint32_t)x.execute % CKI == 0) {
      const uint32_t k = ((uint32_t)x.execute / CKI) % CKR;
      P.ck_e[krc(P, k, x.r, x.c)] = (uint32_t)x.execute;
      P.ck_d[krc(P, k, x.r, x.c)] = x.digest;
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
  if (x.flags & PAXISIM_F_WOVF) x.flags |= PAXISIM_F_UNFAITHFUL;
  int32_t hi = x.slot;
  if (hi > x.execute + (int32_t)P.W - 1) hi = x.execute + (int32_t)P.W - 1;
  uint32_t n = 0;
  for (int32_t s = x.execute; s <= hi; s++) {
    const uint32_t c = x.l_cmd[eidx<NT>(P, x, s)];
    n += (c & EF_EXISTS) && !(c & EF_COMMIT);
  }
  uint32_t ri;
  if (!send_begin<NT>(P, x, bal_id(mb), 1u + n, ri)) return;
  x.rec[ri] = make_uint4(PAXISIM_MSG_P1B | (n << 8), x.ballot, 0u, 0u);
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
    const uint4 cb = x.rec[ri0 + (k + 1u) * LANES];
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
      x.flags |= PAXISIM_F_GHOST;
    } else {
      x.flags |= PAXISIM_F_WOVF;
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
      if (x.flags & PAXISIM_F_WOVF) x.flags |= PAXISIM_F_UNFAITHFUL;
      int32_t hi = x.slot;
      if (hi > x.execute + (int32_t)P.W - 1) hi = x.execute + (int32_t)P.W - 1;
      for (int32_t s = x.execute; s <= hi; s++) {
        const uint32_t i = eidx<NT>(P, x, s);
        const uint32_t c = x.l_cmd[i];
        if (!(c & EF_EXISTS) || (c & EF_COMMIT)) continue;                   // nil gap (G5)
        x.l_bal[i] = x.ballot;
        x.l_cmd[i] = c | EF_QUORUM;
        x.l_ack[i] = 1u << x.r;
        broadcast1<NT>(P, x, PAXISIM_MSG_P2A, x.ballot, (uint32_t)s, c & CMD_MASK);
      }
      const uint32_t np = x.npend;
      x.npend = 0;
      for (uint32_t k = 0; k < np; k++) paxos_p2a<NT>(P, x, P.pend[krc(P, k, x.r, x.c)]);
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
          x.l_bal[i] = e.b;
          x.l_cmd[i] = e.c;
        }
      } else {
        eput<NT>(x, i, Ent{mb, mcid | EF_EXISTS, 0u});
      }
    } else if (ms < x.execute) {
      x.flags |= PAXISIM_F_GHOST;
    } else {
      x.flags |= PAXISIM_F_WOVF;
    }
  }
  send1<NT>(P, x, bal_id(mb), PAXISIM_MSG_P2B, x.ballot, (uint32_t)ms, 0u);
}

template <int NT>
__device__ __forceinline__ void paxos_handle_p2b(const Params& P, Rep<NT>& x, uint32_t src, uint32_t mb,
                                                 int32_t ms) {                // paxos.go:270-310
  if (!in_window<NT>(P, x, ms)) {
    if ((ms < x.execute && (x.flags & PAXISIM_F_GHOST)) || (ms >= x.execute && (x.flags & PAXISIM_F_WOVF)))
      x.flags |= PAXISIM_F_UNFAITHFUL;
    return;
  }
  const uint32_t i = eidx<NT>(P, x, ms);
  const uint32_t c = x.l_cmd[i];
  const uint32_t eb = x.l_bal[i];
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
    const uint32_t ack = x.l_ack[i] | (1u << src);
    x.l_ack[i] = ack;
    if (quorum_ok(P, P.q2, ack)) {
      x.l_cmd[i] = c | EF_COMMIT;
      x.commits++;
      broadcast1<NT>(P, x, PAXISIM_MSG_P3, mb, (uint32_t)ms, c & CMD_MASK);
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
    uint32_t c = x.l_cmd[i];
    if (c & EF_EXISTS) {
      if ((c & CMD_MASK) != mcid && (c & (EF_REQSELF | EF_REQEXT))) {
        node_forward<NT>(P, x, bal_id(mb), ereq<NT>(P, x, i, c));
        c &= ~(EF_REQSELF | EF_REQEXT);
      }
    } else {
      c = EF_EXISTS;                                                          // &entry{} (G6)
      x.l_bal[i] = 0u;
      x.l_ack[i] = 0u;
    }
    c = eset_cmd<NT>(P, x, i, c, mcid) | EF_COMMIT;
    x.l_cmd[i] = c;
    if (P.rwc) {
      if (c & (EF_REQSELF | EF_REQEXT)) {
        const uint32_t q = ereq<NT>(P, x, i, c);
        request_reply<NT>(P, x, q, req_cid(q));
      }
      return;
    }
  } else if (ms < x.execute) {
    x.flags |= PAXISIM_F_GHOST;
  } else {
    x.flags |= PAXISIM_F_WOVF;
  }
  if (!P.rwc) paxos_exec<NT>(P, x);
}

// ---------------------------------------------------------------------------
// One replica, one step
// ---------------------------------------------------------------------------
template <int NT>
__device__ __forceinline__ void fault_process(const Params& P, Rep<NT>& x) {
  if (P.drop_ppm == 0 && P.slow_ppm == 0) return;
#pragma unroll
  for (uint32_t d = 0; d < Rep<NT>::NL; d++) {
    if (d >= nrep<NT>(P) || d == x.r) continue;
    const uint32_t u = draw(x.hs, tag(PUR_LINK, x.r, d));
    if (P.drop_ppm && x.t >= x.du[d] && ppm_hit16(u & 0xFFFFu, P.drop_ppm)) x.du[d] = x.t + P.drop_len;
    if (P.slow_ppm && x.t >= (x.su[d] & (T_MAX - 1u)) && ppm_hit16(u >> 16, P.slow_ppm)) {
      const uint32_t span = P.slow_max - P.slow_min + 1u;
      const uint32_t v = draw(x.hs, tag(PUR_SLOWD, x.r, d));
      x.su[d] = (x.t + P.slow_len) | ((P.slow_min + __umulhi(v, span)) << 28);
    }
  }
}

template <int NT>
__device__ __forceinline__ void paxos_replica_step(const Params& P, Rep<NT>& x) {
  constexpr uint32_t NSMAX = NT ? (uint32_t)NT + 1u : (uint32_t)PAXISIM_MAX_N + 1u;
  const uint32_t N = nrep<NT>(P), NS = N + 1u;
  x.send_seq = 0;
  x.stop = false;
  x.hs = step_key(x.kc, x.t);
  fault_process<NT>(P, x);
  x.crashed = P.nfaults && scripted(P, PAXISIM_FAULT_CRASH, x.gid, x.r, 0u, x.t, nullptr);

  const uint32_t box0 = (x.b0 * N + x.r) * NS;          // inbox boxes: box0 + src
  uint32_t rem[NSMAX], pos[NSMAX], total = 0;
#pragma unroll
  for (uint32_t s = 0; s < NSMAX; s++) {
    rem[s] = 0;
    pos[s] = 0;
    if (s < NS) {
      uint32_t n = x.l_cnt[((box0 + s) << 6) | x.lane];
      if (x.crashed && s < N && n) {                    // socket.Recv discards (socket.go:111-118)
        for (uint32_t k = 0; k < n;) {
          const uint32_t h = x.rec[(((box0 + s) * P.M + k) << 6) | x.lane].x;
          x.discarded++;
          k += 1u + (hdr_type(h) == PAXISIM_MSG_P1B ? hdr_n(h) : 0u);
        }
        n = 0;
      }
      rem[s] = n;
      total += n;
    }
  }

  // merge order: weighted pick among sources, two 16-bit picks per draw;
  // the next message's record is loaded before the current one is handled
  uint32_t u = 0, i = 0, src = 0, ri = 0;
  uint4 m = make_uint4(0u, 0u, 0u, 0u);
  auto pick = [&](uint32_t idx, uint32_t& psrc, uint32_t& pri) {
    if (!(idx & 1u)) u = draw(x.hs, tag(PUR_ORDER, x.r, idx >> 1));
    uint32_t pk = (((idx & 1u) ? (u >> 16) : (u & 0xFFFFu)) * total) >> 16;
    bool found = false;
    psrc = 0;
    uint32_t p0 = 0;
#pragma unroll
    for (uint32_t s = 0; s < NSMAX; s++) {
      const uint32_t rs = opaque(rem[s]);
      const bool here = !found && pk < rs;
      if (here) { psrc = s; p0 = opaque(pos[s]); found = true; }
      else if (!found) pk -= rs;
    }
    pri = (((box0 + psrc) * P.M + p0) << 6) | x.lane;
  };
  if (total) {
    pick(0, src, ri);
    m = x.rec[ri];
  }
  while (total && !x.stop) {
    const uint32_t type = hdr_type(m.x);
    const uint32_t len = 1u + (type == PAXISIM_MSG_P1B ? hdr_n(m.x) : 0u);
#pragma unroll
    for (uint32_t s = 0; s < NSMAX; s++) {
      const bool hit = s == src;
      pos[s] = opaque(pos[s]) + (hit ? len : 0u);
      rem[s] = opaque(rem[s]) - (hit ? len : 0u);
    }
    total -= len;
    uint32_t nsrc = 0, nri = 0;
    uint4 nm = make_uint4(0u, 0u, 0u, 0u);
    if (total) {
      pick(i + 1u, nsrc, nri);
      nm = x.rec[nri];                                  // prefetch
    }
    if (src == N) {
      x.client++;
      handle_request<NT>(P, x, mkreq(m.w, PAXISIM_CLIENT_SRC));
    } else {
      switch (type) {                                   // node.handle dispatch (node.go:104-115)
        case PAXISIM_MSG_REQUEST: x.dv[1]++; handle_request<NT>(P, x, mkreq(m.w, src)); break;
        case PAXISIM_MSG_REPLY: x.dv[2]++; handle_reply<NT>(P, x, m.w); break;
        case PAXISIM_MSG_P1A: x.dv[3]++; paxos_handle_p1a<NT>(P, x, m.y); break;
        case PAXISIM_MSG_P1B: x.dv[4]++; paxos_handle_p1b<NT>(P, x, src, m.y, ri, hdr_n(m.x)); break;
        case PAXISIM_MSG_P2A: x.dv[6]++; paxos_handle_p2a<NT>(P, x, m.y, (int32_t)m.z, m.w); break;
        case PAXISIM_MSG_P2B: x.dv[7]++; paxos_handle_p2b<NT>(P, x, src, m.y, (int32_t)m.z); break;
        case PAXISIM_MSG_P3: x.dv[8]++; paxos_handle_p3<NT>(P, x, m.y, (int32_t)m.z, m.w); break;
        default: break;
      }
    }
    src = nsrc;
    ri = nri;
    m = nm;
    i++;
  }
#pragma unroll
  for (uint32_t s = 0; s < NSMAX; s++)
    if (s < NS) x.l_cnt[((box0 + s) << 6) | x.lane] = 0;
  if (x.stop) atomicMin(&x.l_poison[x.lane], x.t);
}

// ---------------------------------------------------------------------------
// The step kernel: workgroup = N waves (replicas) x 64 lanes (clusters)
// ---------------------------------------------------------------------------
template <int NT>
__global__ void __launch_bounds__(NT ? NT * 64 : 1024) paxos_steps(Params P, uint32_t t0, uint32_t nsteps) {
  extern __shared__ uint4 lds[];
  const uint32_t N = nrep<NT>(P);
  const uint32_t blk = blockIdx.x;
  // stage the workgroup's HBM image into LDS
  {
    const uint4* g = reinterpret_cast<const uint4*>(P.image + (size_t)blk * P.img.bytes);
    for (uint32_t k = threadIdx.x; k < P.img.bytes / 16u; k += blockDim.x) lds[k] = g[k];
  }
  uint8_t* L = reinterpret_cast<uint8_t*>(lds);
  Rep<NT> x;
  x.lane = threadIdx.x & 63u;
  x.r = threadIdx.x >> 6;
  x.blk = blk;
  x.c = (uint64_t)blk * LANES + x.lane;
  x.gid = P.cluster_base + x.c;
  x.l_bal = reinterpret_cast<uint32_t*>(L + P.img.off_bal);
  x.l_cmd = reinterpret_cast<uint32_t*>(L + P.img.off_cmd);
  x.l_ack = reinterpret_cast<uint32_t*>(L + P.img.off_ack);
  x.l_wcur = reinterpret_cast<uint32_t*>(L + P.img.off_wcur);
  x.l_wiss = reinterpret_cast<uint32_t*>(L + P.img.off_wiss);
  x.l_poison = reinterpret_cast<uint32_t*>(L + P.img.off_poison);
  x.l_cnt = L + P.img.off_cnt;
  x.rec = P.rec + (size_t)blk * P.rec_per_block;
  const bool live = x.c < P.clusters && x.r < N;
  if (live) {
    const size_t i = rc(P, x.r, x.c);
    x.kc = P.kc[x.c];
    x.ballot = P.ballot[i];
    x.slot = (int32_t)P.slot[i];
    x.execute = (int32_t)P.execute[i];
    const uint32_t meta = P.meta[i];
    x.active = meta & 1u;
    x.p1mask = meta >> 16;
    x.flags = P.flags[i];
    x.npend = P.npend[i];
    x.nfwd = P.nfwd[i];
    x.digest = P.digest[i];
#pragma unroll
    for (uint32_t d = 0; d < Rep<NT>::NL; d++) {
      x.du[d] = d < N ? P.link_drop[krc(P, d, x.r, x.c)] : 0u;
      x.su[d] = d < N ? P.link_slow[krc(P, d, x.r, x.c)] : 0u;
    }
  }
#pragma unroll
  for (int k = 0; k < 9; k++) x.dv[k] = 0;
  x.client = x.sent = x.dropped = x.discarded = x.commits = x.replies = 0;
  __syncthreads();

  uint32_t b0 = t0 % P.D;
  for (uint32_t t = t0; t < t0 + nsteps; t++) {
    if (live && x.l_poison[x.lane] >= t) {
      x.t = t;
      x.b0 = b0;
      paxos_replica_step<NT>(P, x);
    }
    if (++b0 == P.D) b0 = 0;
    __syncthreads();
  }

  // write back: LDS image, registers, counters
  {
    uint4* g = reinterpret_cast<uint4*>(P.image + (size_t)blk * P.img.bytes);
    for (uint32_t k = threadIdx.x; k < P.img.bytes / 16u; k += blockDim.x) g[k] = lds[k];
  }
  if (live) {
    const uint32_t r = x.r;
    const uint64_t c = x.c;
    const size_t i = rc(P, r, c);
    P.ballot[i] = x.ballot;
    P.slot[i] = (uint32_t)x.slot;
    P.execute[i] = (uint32_t)x.execute;
    P.meta[i] = (x.active & 1u) | (x.p1mask << 16);
    P.flags[i] = x.flags;
    P.npend[i] = x.npend;
    P.nfwd[i] = x.nfwd;
    P.digest[i] = x.digest;
#pragma unroll
    for (uint32_t d = 0; d < Rep<NT>::NL; d++) {
      if (d < N) {
        P.link_drop[krc(P, d, r, c)] = x.du[d];
        P.link_slow[krc(P, d, r, c)] = x.su[d];
      }
    }
#pragma unroll
    for (int k = 1; k < 9; k++)
      if (x.dv[k]) P.stats[krc(P, ST_DELIV0 + k, r, c)] += x.dv[k];
    P.stats[krc(P, ST_CLIENT, r, c)] += x.client;
    P.stats[krc(P, ST_SENT, r, c)] += x.sent;
    P.stats[krc(P, ST_DROPPED, r, c)] += x.dropped;
    P.stats[krc(P, ST_DISCARDED, r, c)] += x.discarded;
    P.stats[krc(P, ST_COMMITS, r, c)] += x.commits;
    P.stats[krc(P, ST_REPLIES, r, c)] += x.replies;
  }
}

}  // namespace pxs
