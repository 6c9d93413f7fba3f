// paxos_kernel.h — Multi-Paxos replica step on gfx950.
//
// One lane = one replica of one cluster.  The handlers follow
// paxos/paxos.go:86-376 and paxos/replica.go:42-66 (cited per function), the
// socket filter socket.go:66-109 and the node runtime node.go:79-172, under
// the delivery schedule of DESIGN.md §3.  Replica scalars live in registers
// for the whole launch; the log window, pending/forward tables and the
// mailboxes are SoA in HBM with the cluster index fastest.
#pragma once
#include "paxisim_dev.h"

namespace pxs {

struct Rep {
  uint64_t c, gid, kc;
  uint32_t r, t;
  uint32_t ballot;
  int32_t slot, execute;
  uint32_t active, p1mask, flags, npend, nfwd;
  uint64_t digest;
  uint32_t dv[9];                       // delivered by type (REQUEST..P3)
  uint32_t client, sent, dropped, discarded, commits, replies;
  uint32_t send_seq;
  bool stop, crashed;
};

template <int NT>
__device__ __forceinline__ uint32_t nrep(const Params& P) { return NT ? (uint32_t)NT : P.N; }

// ---------------------------------------------------------------------------
// socket.Send (socket.go:66-109): crash -> drop -> flaky -> slow, then the
// bounded (link, arrival-step) bucket.  Returns the bucket/slot to write.
// ---------------------------------------------------------------------------
template <int NT>
__device__ __forceinline__ bool send_begin(const Params& P, Rep& x, uint32_t to, uint32_t nrec,
                                           size_t& bx, uint32_t& k) {
  const uint32_t N = nrep<NT>(P);
  const uint32_t seq = x.send_seq++;
  x.sent++;
  if (to >= N || x.crashed) { x.dropped++; return false; }
  const size_t li = krc(P, to, x.r, x.c);
  if (x.t < P.drop_until[li] || (P.nfaults && scripted(P, PAXISIM_FAULT_DROP, x.gid, x.r, to, x.t, nullptr))) {
    x.dropped++;
    return false;
  }
  uint32_t delay = 0;
  if (P.nfaults) {
    uint32_t p = 0;
    if (scripted(P, PAXISIM_FAULT_FLAKY, x.gid, x.r, to, x.t, &p) && p > 0) {
      const uint32_t u = (uint32_t)(draw(x.kc, x.t, tag(PUR_FLAKY, x.r, seq)) >> 32);
      if (ppm_hit(u, p)) { x.dropped++; return false; }
    }
  }
  if (x.t < P.slow_until[li]) delay = P.slow_delay[li];
  if (P.nfaults) scripted(P, PAXISIM_FAULT_SLOW, x.gid, x.r, to, x.t, &delay);
  if (delay > P.max_delay) delay = P.max_delay;
  const uint32_t b = (x.t + 1u + delay) % P.D;
  bx = box(P, b, to, x.r);
  uint8_t* cp = cnt_at(P, bx, x.c);
  k = *cp;
  if (k + nrec > P.M) {
    x.flags |= PAXISIM_F_MBOX_OVF | PAXISIM_F_UNFAITHFUL;
    x.dropped++;
    return false;
  }
  *cp = (uint8_t)(k + nrec);
  return true;
}

template <int NT>
__device__ __forceinline__ void send1(const Params& P, Rep& x, uint32_t to, uint32_t type, uint32_t ballot,
                                      uint32_t slot, uint32_t cid) {
  size_t bx;
  uint32_t k;
  if (send_begin<NT>(P, x, to, 1, bx, k)) *rec_at(P, bx, k, x.c) = make_uint4(type, ballot, slot, cid);
}

// Broadcast excludes self, IDs.Less order (socket.go:147-155)
template <int NT>
__device__ __forceinline__ void broadcast1(const Params& P, Rep& x, uint32_t type, uint32_t ballot,
                                           uint32_t slot, uint32_t cid) {
  const uint32_t N = nrep<NT>(P);
  for (uint32_t d = 0; d < N; d++)
    if (d != x.r) send1<NT>(P, x, d, type, ballot, slot, cid);
}

// ---------------------------------------------------------------------------
// client (benchmark.go:246-275) and Request.Reply routing (node.go:83-97)
// ---------------------------------------------------------------------------
template <int NT>
__device__ __forceinline__ void client_reply(const Params& P, Rep& x, uint32_t cid) {
  const uint32_t WK = P.WK, w = (cid - 1u) % WK;
  uint32_t* cur = &P.wk_cur[(size_t)w * P.C + x.c];
  if (*cur != cid) return;                     // duplicate reply: the worker moved on
  x.replies++;
  uint32_t* iss = &P.wk_issued[(size_t)w * P.C + x.c];
  const uint32_t issued = *iss;
  if (P.max_requests == 0 || issued < P.max_requests) {
    const uint64_t nc = 1ull + w + (uint64_t)WK * issued;
    if (nc > 0x07FFFFFFull) {
      x.flags |= PAXISIM_F_PEND_OVF | PAXISIM_F_UNFAITHFUL;
      *cur = 0;
      return;
    }
    *iss = issued + 1u;
    *cur = (uint32_t)nc;
    // the next request reaches the worker's target (this replica) next step
    const size_t bx = box(P, (x.t + 1u) % P.D, P.target[w], nrep<NT>(P));
    uint8_t* cp = cnt_at(P, bx, x.c);
    const uint32_t k = *cp;
    if (k >= P.M) {
      x.flags |= PAXISIM_F_MBOX_OVF | PAXISIM_F_UNFAITHFUL;
      return;
    }
    *rec_at(P, bx, k, x.c) = make_uint4(PAXISIM_MSG_REQUEST, 0u, 0u, (uint32_t)nc);
    *cp = (uint8_t)(k + 1u);
  } else {
    *cur = 0;
  }
}

template <int NT>
__device__ __forceinline__ void request_reply(const Params& P, Rep& x, uint32_t req, uint32_t reply_cmd) {
  const uint32_t o = req_origin(req);
  if (o == PAXISIM_CLIENT_SRC) client_reply<NT>(P, x, req_cid(req));
  else send1<NT>(P, x, o, PAXISIM_MSG_REPLY, 0u, 0u, reply_cmd);
}

// node.Forward (node.go:165-172)
template <int NT>
__device__ __forceinline__ void node_forward(const Params& P, Rep& x, uint32_t to, uint32_t req) {
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
__device__ __forceinline__ void handle_reply(const Params& P, Rep& x, uint32_t cid) {
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
__device__ __forceinline__ bool in_window(const Params& P, const Rep& x, int32_t s) {
  return s >= x.execute && s < x.execute + (int32_t)P.W;
}

template <int NT>
__device__ __forceinline__ void paxos_forward(const Params& P, Rep& x) {     // paxos.go:371-376
  for (uint32_t i = 0; i < x.npend; i++) node_forward<NT>(P, x, bal_id(x.ballot), P.pend[krc(P, i, x.r, x.c)]);
  x.npend = 0;
}

template <int NT>
__device__ __forceinline__ void paxos_p1a(const Params& P, Rep& x) {          // paxos.go:100-108
  if (x.active) return;
  if ((x.ballot >> 4) + 1u >= (1u << 27)) x.flags |= PAXISIM_F_BALLOT_OVF | PAXISIM_F_UNFAITHFUL;
  x.ballot = bal_next(x.ballot, x.r);
  x.p1mask = 1u << x.r;
  broadcast1<NT>(P, x, PAXISIM_MSG_P1A, x.ballot, 0u, 0u);
}

template <int NT>
__device__ __forceinline__ void paxos_p2a(const Params& P, Rep& x, uint32_t req) {  // paxos.go:111-131
  x.slot++;
  const uint32_t cid = req_cid(req);
  if (in_window(P, x, x.slot)) {
    *log_at(P, x.r, x.c, x.slot) = make_uint4(x.ballot, cid, req, E_EXISTS | E_QUORUM | ((1u << x.r) << 16));
  } else {
    x.flags |= PAXISIM_F_WOVF | PAXISIM_F_UNFAITHFUL;
  }
  if (P.thrifty) {                                   // MulticastQuorum(N/2+1) (socket.go:132-145)
    const uint32_t N = nrep<NT>(P);
    uint32_t sent = 0;
    for (uint32_t i = 1; i < N && sent < N / 2 + 1; i++, sent++)
      send1<NT>(P, x, (x.r + i) % N, PAXISIM_MSG_P2A, x.ballot, (uint32_t)x.slot, cid);
  } else {
    broadcast1<NT>(P, x, PAXISIM_MSG_P2A, x.ballot, (uint32_t)x.slot, cid);
  }
}

template <int NT>
__device__ __forceinline__ void paxos_handle_request(const Params& P, Rep& x, uint32_t req) {  // paxos.go:86-97
  if (!x.active) {
    if (x.npend == PMAX) x.flags |= PAXISIM_F_PEND_OVF | PAXISIM_F_UNFAITHFUL;
    else P.pend[krc(P, x.npend++, x.r, x.c)] = req;
    if (bal_id(x.ballot) != x.r) paxos_p1a<NT>(P, x);
  } else {
    paxos_p2a<NT>(P, x, req);
  }
}

template <int NT>
__device__ __forceinline__ void handle_request(const Params& P, Rep& x, uint32_t req) {  // replica.go:42-66
  const bool leader = x.active || bal_id(x.ballot) == x.r;
  if (P.ephemeral || leader || x.ballot == 0) paxos_handle_request<NT>(P, x, req);
  else node_forward<NT>(P, x, bal_id(x.ballot), req);
}

template <int NT>
__device__ __forceinline__ void paxos_exec(const Params& P, Rep& x) {                         // paxos.go:345-369
  for (;;) {
    uint4* ep = log_at(P, x.r, x.c, x.execute);
    uint4 e = *ep;
    if (!(e.w & E_EXISTS) || !(e.w & E_COMMIT)) break;
    if (x.flags & PAXISIM_F_WOVF) x.flags |= PAXISIM_F_UNFAITHFUL;
    if (e.z) request_reply<NT>(P, x, e.z, e.y);
    x.digest = mix64(x.digest ^ (((uint64_t)(uint32_t)x.execute << 32) | e.y));
    ep->w = 0u;                                                      // delete(p.log, execute)
    x.execute++;
    if ((uint32_t)x.execute % CKI == 0) {
      const uint32_t k = ((uint32_t)x.execute / CKI) % CKR;
      P.ck_e[krc(P, k, x.r, x.c)] = (uint32_t)x.execute;
      P.ck_d[krc(P, k, x.r, x.c)] = x.digest;
    }
  }
}

template <int NT>
__device__ __forceinline__ void paxos_handle_p1a(const Params& P, Rep& x, uint32_t mb) {  // paxos.go:134-162
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
    const uint32_t m = log_at(P, x.r, x.c, s)->w;
    n += (m & E_EXISTS) && !(m & E_COMMIT);
  }
  size_t bx;
  uint32_t k;
  if (!send_begin<NT>(P, x, bal_id(mb), 1u + n, bx, k)) return;
  *rec_at(P, bx, k, x.c) = make_uint4(PAXISIM_MSG_P1B | (n << 8), x.ballot, 0u, 0u);
  for (int32_t s = x.execute; s <= hi; s++) {
    const uint4 e = *log_at(P, x.r, x.c, s);
    if (!(e.w & E_EXISTS) || (e.w & E_COMMIT)) continue;
    *rec_at(P, bx, ++k, x.c) = make_uint4(PAXISIM_MSG_P1B_ENTRY, e.x, (uint32_t)s, e.y);
  }
}

// P1b with its CommandBallot payload at records [k0+1, k0+1+n) of bucket bx
template <int NT>
__device__ __forceinline__ void paxos_handle_p1b(const Params& P, Rep& x, uint32_t src, uint32_t mb, size_t bx, uint32_t k0,
                                 uint32_t n) {                                // paxos.go:164-230
  if (mb < x.ballot || x.active) return;
  for (uint32_t i = 0; i < n; i++) {                                          // update(): 164-180
    const uint4 cb = *rec_at(P, bx, k0 + 1u + i, x.c);
    const int32_t s = (int32_t)cb.z;
    if (s > x.slot) x.slot = s;
    if (in_window(P, x, s)) {
      uint4* ep = log_at(P, x.r, x.c, s);
      uint4 e = *ep;
      if (e.w & E_EXISTS) {
        if (!(e.w & E_COMMIT) && cb.y > e.x) { e.x = cb.y; e.y = cb.w; *ep = e; }
      } else {
        *ep = make_uint4(cb.y, cb.w, 0u, E_EXISTS);
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
      for (int32_t i = x.execute; i <= hi; i++) {
        uint4* ep = log_at(P, x.r, x.c, i);
        uint4 e = *ep;
        if (!(e.w & E_EXISTS) || (e.w & E_COMMIT)) continue;                 // nil gap (G5)
        e.x = x.ballot;
        e.w = (e.w & (E_EXISTS | E_COMMIT)) | E_QUORUM | ((1u << x.r) << 16);
        *ep = e;
        broadcast1<NT>(P, x, PAXISIM_MSG_P2A, x.ballot, (uint32_t)i, e.y);
      }
      const uint32_t np = x.npend;
      x.npend = 0;
      for (uint32_t k = 0; k < np; k++) paxos_p2a<NT>(P, x, P.pend[krc(P, k, x.r, x.c)]);
    }
  }
}

template <int NT>
__device__ __forceinline__ void paxos_handle_p2a(const Params& P, Rep& x, uint32_t mb, int32_t ms,
                                                 uint32_t mcid) {             // paxos.go:233-267
  if (mb >= x.ballot) {
    x.ballot = mb;
    x.active = 0;
    if (ms > x.slot) x.slot = ms;
    if (in_window(P, x, ms)) {
      uint4* ep = log_at(P, x.r, x.c, ms);
      uint4 e = *ep;
      if (e.w & E_EXISTS) {
        if (!(e.w & E_COMMIT) && mb > e.x) {
          if (e.y != mcid && e.z) {
            node_forward<NT>(P, x, bal_id(mb), e.z);
            e.z = 0;
          }
          e.y = mcid;
          e.x = mb;
          *ep = e;
        }
      } else {
        *ep = make_uint4(mb, mcid, 0u, E_EXISTS);
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
__device__ __forceinline__ void paxos_handle_p2b(const Params& P, Rep& x, uint32_t src, uint32_t mb,
                                                 int32_t ms) {                // paxos.go:270-310
  if (!in_window(P, x, ms)) {
    if ((ms < x.execute && (x.flags & PAXISIM_F_GHOST)) || (ms >= x.execute && (x.flags & PAXISIM_F_WOVF)))
      x.flags |= PAXISIM_F_UNFAITHFUL;
    return;
  }
  uint4* ep = log_at(P, x.r, x.c, ms);
  uint4 e = *ep;
  if (!(e.w & E_EXISTS) || mb < e.x || (e.w & E_COMMIT)) return;
  if (mb > x.ballot) {
    x.ballot = mb;
    x.active = 0;
  }
  if (bal_id(mb) == x.r && mb == e.x) {
    if (!(e.w & E_QUORUM)) {                                                  // nil quorum: Go panics
      x.flags |= PAXISIM_F_POISON;
      x.stop = true;
      return;
    }
    e.w |= (1u << src) << 16;
    if (quorum_ok(P, P.q2, e.w >> 16)) {
      e.w |= E_COMMIT;
      *ep = e;
      x.commits++;
      broadcast1<NT>(P, x, PAXISIM_MSG_P3, mb, (uint32_t)ms, e.y);
      if (P.rwc) {
        if (!e.z) { x.flags |= PAXISIM_F_POISON; x.stop = true; return; }
        request_reply<NT>(P, x, e.z, req_cid(e.z));
      } else {
        paxos_exec<NT>(P, x);
      }
    } else {
      ep->w = e.w;
    }
  }
}

template <int NT>
__device__ __forceinline__ void paxos_handle_p3(const Params& P, Rep& x, uint32_t mb, int32_t ms,
                                                uint32_t mcid) {              // paxos.go:313-343
  if (ms > x.slot) x.slot = ms;
  if (in_window(P, x, ms)) {
    uint4* ep = log_at(P, x.r, x.c, ms);
    uint4 e = *ep;
    if (e.w & E_EXISTS) {
      if (e.y != mcid && e.z) {
        node_forward<NT>(P, x, bal_id(mb), e.z);
        e.z = 0;
      }
    } else {
      e = make_uint4(0u, 0u, 0u, E_EXISTS);                                   // &entry{} (G6)
    }
    e.y = mcid;
    e.w |= E_COMMIT;
    *ep = e;
    if (P.rwc) {
      if (e.z) request_reply<NT>(P, x, e.z, req_cid(e.z));
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
__device__ __forceinline__ void fault_process(const Params& P, Rep& x) {
  if (P.drop_ppm == 0 && P.slow_ppm == 0) return;
  const uint32_t N = nrep<NT>(P);
  for (uint32_t d = 0; d < N; d++) {
    if (d == x.r) continue;
    const uint64_t u = draw(x.kc, x.t, tag(PUR_LINK, x.r, d));
    const size_t li = krc(P, d, x.r, x.c);
    if (P.drop_ppm && x.t >= P.drop_until[li] && ppm_hit((uint32_t)u, P.drop_ppm)) P.drop_until[li] = x.t + P.drop_len;
    if (P.slow_ppm && x.t >= P.slow_until[li] && ppm_hit((uint32_t)(u >> 32), P.slow_ppm)) {
      const uint32_t span = P.slow_max - P.slow_min + 1u;
      const uint32_t v = (uint32_t)(draw(x.kc, x.t, tag(PUR_SLOWD, x.r, d)) >> 32);
      P.slow_until[li] = x.t + P.slow_len;
      P.slow_delay[li] = P.slow_min + __umulhi(v, span);
    }
  }
}

template <int NT>
__device__ __forceinline__ void paxos_replica_step(const Params& P, Rep& x) {
  constexpr uint32_t NSMAX = NT ? (uint32_t)NT + 1u : (uint32_t)PAXISIM_MAX_N + 1u;
  const uint32_t N = nrep<NT>(P), NS = N + 1u;
  const uint32_t b = x.t % P.D;
  x.send_seq = 0;
  x.stop = false;
  fault_process<NT>(P, x);
  x.crashed = P.nfaults && scripted(P, PAXISIM_FAULT_CRASH, x.gid, x.r, 0u, x.t, nullptr);

  uint32_t rem[NSMAX], pos[NSMAX], total = 0;
#pragma unroll
  for (uint32_t s = 0; s < NSMAX; s++) {
    rem[s] = 0;
    pos[s] = 0;
    if (s < NS) {
      const size_t bx = box(P, b, x.r, s);
      uint32_t n = *cnt_at(P, bx, x.c);
      if (x.crashed && s < N && n) {                  // socket.Recv discards (socket.go:111-118)
        for (uint32_t k = 0; k < n;) {
          const uint32_t h = rec_at(P, bx, k, x.c)->x;
          x.discarded++;
          k += 1u + (hdr_type(h) == PAXISIM_MSG_P1B ? hdr_n(h) : 0u);
        }
        n = 0;
      }
      rem[s] = n;
      total += n;
    }
  }

  for (uint32_t i = 0; total > 0 && !x.stop; i++) {
    const uint32_t u = (uint32_t)(draw(x.kc, x.t, tag(PUR_ORDER, x.r, i)) >> 32);
    uint32_t pick = __umulhi(u, total), src = 0, p0 = 0;
    bool found = false;
#pragma unroll
    for (uint32_t s = 0; s < NSMAX; s++) {
      const bool here = !found && pick < rem[s];
      if (here) { src = s; p0 = pos[s]; found = true; }
      else if (!found) pick -= rem[s];
    }
    const size_t bx = box(P, b, x.r, src);
    const uint4 m = *rec_at(P, bx, p0, x.c);
    const uint32_t type = hdr_type(m.x);
    const uint32_t len = 1u + (type == PAXISIM_MSG_P1B ? hdr_n(m.x) : 0u);
#pragma unroll
    for (uint32_t s = 0; s < NSMAX; s++)
      if (s == src) { pos[s] += len; rem[s] -= len; }
    total -= len;
    if (src == N) {
      x.client++;
      handle_request<NT>(P, x, mkreq(m.w, PAXISIM_CLIENT_SRC));
      continue;
    }
    switch (type) {                                   // node.handle dispatch (node.go:104-115)
      case PAXISIM_MSG_REQUEST: x.dv[1]++; handle_request<NT>(P, x, mkreq(m.w, src)); break;
      case PAXISIM_MSG_REPLY: x.dv[2]++; handle_reply<NT>(P, x, m.w); break;
      case PAXISIM_MSG_P1A: x.dv[3]++; paxos_handle_p1a<NT>(P, x, m.y); break;
      case PAXISIM_MSG_P1B: x.dv[4]++; paxos_handle_p1b<NT>(P, x, src, m.y, bx, p0, hdr_n(m.x)); break;
      case PAXISIM_MSG_P2A: x.dv[6]++; paxos_handle_p2a<NT>(P, x, m.y, (int32_t)m.z, m.w); break;
      case PAXISIM_MSG_P2B: x.dv[7]++; paxos_handle_p2b<NT>(P, x, src, m.y, (int32_t)m.z); break;
      case PAXISIM_MSG_P3: x.dv[8]++; paxos_handle_p3<NT>(P, x, m.y, (int32_t)m.z, m.w); break;
      default: break;
    }
  }
#pragma unroll
  for (uint32_t s = 0; s < NSMAX; s++)
    if (s < NS) *cnt_at(P, box(P, b, x.r, s), x.c) = 0;
  if (x.stop) atomicMin(&P.poison[x.c], x.t);
}

// ---------------------------------------------------------------------------
// The step kernel: workgroup = N waves (replicas) x 64 lanes (clusters)
// ---------------------------------------------------------------------------
template <int NT>
__global__ void __launch_bounds__(1024) paxos_steps(Params P, uint32_t t0, uint32_t nsteps) {
  const uint32_t r = threadIdx.x >> 6;
  const uint64_t c = (uint64_t)blockIdx.x * LANES + (threadIdx.x & 63u);
  const bool live = c < P.clusters;
  Rep x;
  x.r = r;
  x.c = c;
  x.gid = P.cluster_base + c;
  if (live) {
    const size_t i = rc(P, r, c);
    x.kc = P.kc[c];
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
  }
#pragma unroll
  for (int k = 0; k < 9; k++) x.dv[k] = 0;
  x.client = x.sent = x.dropped = x.discarded = x.commits = x.replies = 0;

  for (uint32_t t = t0; t < t0 + nsteps; t++) {
    if (live && P.poison[c] >= t) {
      x.t = t;
      paxos_replica_step<NT>(P, x);
    }
    __syncthreads();
  }

  if (live) {
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
