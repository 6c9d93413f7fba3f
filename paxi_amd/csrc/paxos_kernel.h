// paxos_kernel.h — Multi-Paxos handlers on gfx950 (a protocol policy of sim_core.h).
//
// One lane = one replica of one cluster.  The handlers follow
// paxos/paxos.go:86-376 and paxos/replica.go:42-66 (cited per function) and the
// node runtime's forward/reply routing node.go:79-172.
//
// Paxos state during a launch:
//   registers: ballot, slot, execute, active, phase-1 acks, pending/forward counts, digest
//   log window {ballot, cmd|flags, acks} as [r][W][lane] u32 (regions a, b, c of
//              the tile image): in the HBM image for the serial kernels (the
//              product, sim_serial*), in LDS for the rounds-1-2 sim_steps kernel
//   HBM:       request side table, pending/forward tables, digest checkpoints
#pragma once
#include "sim_core.h"

namespace pxs {

// ---------------------------------------------------------------------------
// log window (HBM image, or LDS in sim_steps): entry of slot s of replica r at [(r*W + (s & (W-1)))*64 + lane]
// ---------------------------------------------------------------------------
struct Ent { uint32_t b, c, a; };

// PXS_TALLY (paxisim_dev.h): the handlers below see only x
#ifdef PXS_TALLY
#define PXS_TALLY_X(x, cls, ptr, st) tally_at((x).tdbg, (x).blk, (cls), (const void*)(ptr), (st))
#else
#define PXS_TALLY_X(x, cls, ptr, st)
#endif

// Two layouts share these handlers.  Multi-Paxos keeps each replica's window
// in LDS as three u32 planes (l_a / l_b / l_c, entry stride es = 64 lanes) and
// the request side table in HBM (reqx).  The per-key instances of WPaxos keep
// theirs in HBM as one 16-B entry {ballot, cmd|flags, acks, request} per slot
// (es = 4 words): reads go through a one-entry register cache that the
// dispatcher fills before the handler runs (its load overlaps the instance
// bind), and writes go through to HBM.  es is a compile-time constant of each
// kernel instance (sim_steps sets it before any use), so the branch folds.
template <int NT>
__device__ __forceinline__ uint32_t eidx(const Params& P, const Rep<NT>& x, int32_t s) {
  return x.e0 + ((uint32_t)s & (P.W - 1u)) * x.es;
}
template <int NT>
__device__ __forceinline__ bool hbm_log(const Rep<NT>& x) { return x.es == 4u; }
template <int NT>
__device__ __forceinline__ void ecache(Rep<NT>& x, uint32_t i) {
  if (x.ci != i) {
    PXS_TALLY_X(x, TC_ENT_LD, x.l_a + i, false);
    x.ce = *reinterpret_cast<const uint4*>(x.l_a + i);
    x.ci = i;
  }
}
template <int NT>
__device__ __forceinline__ uint32_t ea(Rep<NT>& x, uint32_t i) {
  if (hbm_log(x)) { ecache(x, i); return x.ce.x; }
  PXS_TALLY_X(x, TC_ENT_LD, x.l_a + i, false);
  return x.l_a[i];
}
template <int NT>
__device__ __forceinline__ uint32_t eb(Rep<NT>& x, uint32_t i) {
  if (hbm_log(x)) { ecache(x, i); return x.ce.y; }
  PXS_TALLY_X(x, TC_ENT_LD, x.l_b + i, false);
  return x.l_b[i];
}
template <int NT>
__device__ __forceinline__ uint32_t ec(Rep<NT>& x, uint32_t i) {
  if (hbm_log(x)) { ecache(x, i); return x.ce.z; }
  if (wb_on(x) && x.ci == i) return x.ce.z;
  PXS_TALLY_X(x, TC_ENT_LD, x.l_c + i, false);
  return x.l_c[i];
}
template <int NT>
__device__ __forceinline__ void set_a(Rep<NT>& x, uint32_t i, uint32_t v) {
  PXS_TALLY_X(x, TC_ENT_ST, x.l_a + i, true);
  if (hbm_log(x)) { x.l_a[i] = v; if (x.ci == i) x.ce.x = v; return; }
  x.l_a[i] = v;
}
// committed-entry bits of an HBM-resident window: exec() stops at the first
// clear bit without reading the entry (W <= 16; wider windows read it)
template <int NT>
__device__ __forceinline__ void cm_note(Rep<NT>& x, uint32_t i, uint32_t c) {
  const uint32_t bit = 1u << ((i >> 2) & 31u);
  x.cmask = (c & EF_COMMIT) ? (x.cmask | bit) : (x.cmask & ~bit);
}
template <int NT>
__device__ __forceinline__ void set_b(Rep<NT>& x, uint32_t i, uint32_t v) {
  PXS_TALLY_X(x, TC_ENT_ST, hbm_log(x) ? x.l_a + i + 1u : x.l_b + i, true);
  if (hbm_log(x)) { x.l_a[i + 1u] = v; if (x.ci == i) x.ce.y = v; cm_note(x, i, v); return; }
  x.l_b[i] = v;
}
template <int NT>
__device__ __forceinline__ void set_c(Rep<NT>& x, uint32_t i, uint32_t v) {
  PXS_TALLY_X(x, TC_ENT_ST, hbm_log(x) ? x.l_a + i + 2u : x.l_c + i, true);
  if (hbm_log(x)) { x.l_a[i + 2u] = v; if (x.ci == i) x.ce.z = v; return; }
  if (wb_on(x)) {
    if (x.ci != i) wb_flush(x);
    x.ci = i;
    x.ce.z = v;
    return;
  }
  x.l_c[i] = v;
}
template <int NT>
__device__ __forceinline__ Ent eget(Rep<NT>& x, uint32_t i) { return Ent{ea(x, i), eb(x, i), ec(x, i)}; }
template <int NT>
__device__ __forceinline__ void eput(Rep<NT>& x, uint32_t i, const Ent& e) {
  if (hbm_log(x)) {                                  // one 12-B store
    uint32_t* q = x.l_a + i;
    PXS_TALLY_X(x, TC_ENT_ST, q, true);
    *reinterpret_cast<uint2*>(q) = make_uint2(e.b, e.c);
    q[2] = e.a;
    if (x.ci == i) { x.ce.x = e.b; x.ce.y = e.c; x.ce.z = e.a; }
    cm_note(x, i, e.c);
    return;
  }
  if (wb_on(x) && x.ci == i) x.ci = ~0u;            // superseded by this write
  PXS_TALLY_X(x, TC_ENT_ST, x.l_a + i, true);
  PXS_TALLY_X(x, TC_ENT_ST, x.l_b + i, true);
  PXS_TALLY_X(x, TC_ENT_ST, x.l_c + i, true);
  x.l_a[i] = e.b;
  x.l_b[i] = e.c;
  x.l_c[i] = e.a;
}
// request side table entry for log entry index i
template <int NT>
__device__ __forceinline__ uint32_t rq_get(Rep<NT>& x, uint32_t i) {
  if (hbm_log(x)) { ecache(x, i); return x.ce.w; }
  PXS_TALLY_X(x, TC_OTHER, &x.reqx[i], false);
  return ldg(&x.reqx[i]);
}
template <int NT>
__device__ __forceinline__ void rq_set(Rep<NT>& x, uint32_t i, uint32_t q) {
  PXS_TALLY_X(x, hbm_log(x) ? TC_ENT_ST : TC_OTHER, hbm_log(x) ? x.l_a + i + 3u : &x.reqx[i], true);
  if (hbm_log(x)) { x.l_a[i + 3u] = q; if (x.ci == i) x.ce.w = q; return; }
  x.reqx[i] = q;
}
template <int NT>
__device__ __forceinline__ uint32_t ereq(const Params& P, Rep<NT>& x, uint32_t i, uint32_t c) {
  if (c & EF_REQSELF) return mkreq(c & CMD_MASK, PAXISIM_CLIENT_SRC);
  if (c & EF_REQEXT) return rq_get(x, i);
  return 0u;
}
// attach request q to entry flags c (whose command is cmd)
template <int NT>
__device__ __forceinline__ uint32_t eset_req(const Params& P, Rep<NT>& x, uint32_t i, uint32_t c, uint32_t q) {
  c &= ~(EF_REQSELF | EF_REQEXT);
  if (!q) return c;
  if (req_origin(q) == PAXISIM_CLIENT_SRC && req_cid(q) == (c & CMD_MASK)) return c | EF_REQSELF;
  rq_set(x, i, q);
  return c | EF_REQEXT;
}
// replace the command of an entry, keeping its request (paxos.go:168-171)
template <int NT>
__device__ __forceinline__ uint32_t eset_cmd(const Params& P, Rep<NT>& x, uint32_t i, uint32_t c, uint32_t cmd) {
  if ((c & EF_REQSELF) && (c & CMD_MASK) != cmd) {
    rq_set(x, i, mkreq(c & CMD_MASK, PAXISIM_CLIENT_SRC));
    c = (c & ~EF_REQSELF) | EF_REQEXT;
  }
  return (c & ~CMD_MASK) | cmd;
}

// ---------------------------------------------------------------------------
// Request.Reply routing (node.go:83-97) and node.Forward (node.go:165-172)
// ---------------------------------------------------------------------------
// The Reply's Value (0 = nil) rides in the record's ballot word.
template <int NT>
__device__ __forceinline__ void request_reply(const Params& P, Rep<NT>& x, uint32_t req, uint32_t reply_cmd,
                                              uint32_t value) {
  const uint32_t o = req_origin(req);
  if (o == PAXISIM_CLIENT_SRC) client_reply<NT>(P, x, req_cid(req), value);
  else post_unicast<NT>(P, x, o, PAXISIM_MSG_REPLY, value, 0u, reply_cmd);
}

// node.Forward (node.go:165-172)
// index of cid in the forwards table, or nfwd: four probes per round trip
template <int NT>
__device__ __forceinline__ uint32_t fwd_find(const Params& P, const Rep<NT>& x, uint32_t cid) {
  if (!hbm_log(x)) {                                     // (A/B r2: the LDS-window kernels keep one probe per trip)
    uint32_t i = 0;
    for (; i < x.nfwd; i++) {
      PXS_TALLY_AT(P, x.blk, TC_FWD, &P.fwd[krc(P, i, x.r, x.c)], false);
      if (req_cid(ldg(&P.fwd[krc(P, i, x.r, x.c)])) == cid) break;
    }
    return i;
  }
  for (uint32_t i = 0; i < x.nfwd; i += 4u) {
    uint32_t f[4];
#ifdef PXS_TALLY
#pragma unroll
    for (uint32_t k = 0; k < 4u; k++)
      if (i + k < x.nfwd) PXS_TALLY_AT(P, x.blk, TC_FWD, &P.fwd[krc(P, i + k, x.r, x.c)], false);
#endif
#pragma unroll
    for (uint32_t k = 0; k < 4u; k++) f[k] = i + k < x.nfwd ? P.fwd[krc(P, i + k, x.r, x.c)] : 0u;
#pragma unroll
    for (uint32_t k = 0; k < 4u; k++)
      if (i + k < x.nfwd && req_cid(f[k]) == cid) return i + k;
  }
  return x.nfwd;
}

template <int NT>
__device__ __forceinline__ void node_forward(const Params& P, Rep<NT>& x, uint32_t to, uint32_t req) {
  const uint32_t cid = req_cid(req);
  const uint32_t i = fwd_find<NT>(P, x, cid);
  if (i == x.nfwd) {
    if (x.nfwd == FMAX) x.flags |= PAXISIM_F_PEND_OVF | PAXISIM_F_UNFAITHFUL;
    else {
      PXS_TALLY_AT(P, x.blk, TC_FWD, &P.fwd[krc(P, x.nfwd, x.r, x.c)], true);
      P.fwd[krc(P, x.nfwd++, x.r, x.c)] = req;
    }
  } else {
    PXS_TALLY_AT(P, x.blk, TC_FWD, &P.fwd[krc(P, i, x.r, x.c)], true);
    P.fwd[krc(P, i, x.r, x.c)] = req;
  }
  post_unicast<NT>(P, x, to, PAXISIM_MSG_REQUEST, 0u, 0u, cid);
}

// node.recv Reply case (node.go:83-90).  With the table in HBM (the per-key
// kernels) the probe keeps the four entries it loaded: the request found is
// one of them, and so is the table's last entry (moved into the freed place)
// whenever it lies in the same group - one round trip where the LDS-window
// kernels' probe-then-reload path takes three.
template <int NT>
__device__ __forceinline__ void handle_reply(const Params& P, Rep<NT>& x, uint32_t cid, uint32_t value) {
  if (hbm_log(x)) {
    const uint32_t last = x.nfwd - 1u;
    for (uint32_t i0 = 0; i0 < x.nfwd; i0 += 4u) {
      uint32_t f[4];
#ifdef PXS_TALLY
#pragma unroll
    for (uint32_t k = 0; k < 4u; k++)
      if (i0 + k < x.nfwd) PXS_TALLY_AT(P, x.blk, TC_FWD, &P.fwd[krc(P, i0 + k, x.r, x.c)], false);
#endif
#pragma unroll
      for (uint32_t k = 0; k < 4u; k++) f[k] = i0 + k < x.nfwd ? P.fwd[krc(P, i0 + k, x.r, x.c)] : 0u;
#pragma unroll
      for (uint32_t k = 0; k < 4u; k++) {
        if (!(i0 + k < x.nfwd && req_cid(f[k]) == cid)) continue;
        uint32_t lv = 0;
#pragma unroll
        for (uint32_t q = 0; q < 4u; q++) lv = last == i0 + q ? f[q] : lv;
        if (last >= i0 + 4u) {
          PXS_TALLY_AT(P, x.blk, TC_FWD, &P.fwd[krc(P, last, x.r, x.c)], false);
          lv = ldg(&P.fwd[krc(P, last, x.r, x.c)]);
        }
        x.nfwd = last;
        PXS_TALLY_AT(P, x.blk, TC_FWD, &P.fwd[krc(P, i0 + k, x.r, x.c)], true);
        P.fwd[krc(P, i0 + k, x.r, x.c)] = lv;
        request_reply<NT>(P, x, f[k], cid, value);
        return;
      }
    }
    x.flags |= PAXISIM_F_UNFAITHFUL;
    return;
  }
  const uint32_t i = fwd_find<NT>(P, x, cid);
  if (i == x.nfwd) {
    x.flags |= PAXISIM_F_UNFAITHFUL;
    return;
  }
  PXS_TALLY_AT(P, x.blk, TC_FWD, &P.fwd[krc(P, i, x.r, x.c)], false);
  PXS_TALLY_AT(P, x.blk, TC_FWD, &P.fwd[krc(P, x.nfwd, x.r, x.c)], false);
  PXS_TALLY_AT(P, x.blk, TC_FWD, &P.fwd[krc(P, i, x.r, x.c)], true);
  const uint32_t req = ldg(&P.fwd[krc(P, i, x.r, x.c)]);
  x.nfwd--;
  P.fwd[krc(P, i, x.r, x.c)] = ldg(&P.fwd[krc(P, x.nfwd, x.r, x.c)]);
  request_reply<NT>(P, x, req, cid, value);
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
// Ghost table addressing.  Per-key instances (HBM log) keep a lane's GMAX
// ghosts of one instance in one 128-B line ([NI][C][GMAX]), so the probes
// after the first hit in cache; Multi-Paxos keeps [GMAX][NI][C] (A/B r2: the
// line layout costs its LDS-window kernels registers).  The probes stay
// serial (ldg): eight in flight at once would cost 32 registers.
template <int NT>
__device__ __forceinline__ uint4* gref(const Params& P, const Rep<NT>& x, uint32_t g) {
  uint4* q = hbm_log(x) ? &P.gst[((size_t)x.inst * P.C + x.c) * GMAX + g] : &P.gst[((size_t)g * P.NI + x.inst) * P.C + x.c];
  PXS_TALLY_AT(P, x.blk, TC_GHOST, q, false);   // (every use of a ghost reference counted as a line)
  return q;
}
template <int NT>
__device__ __forceinline__ uint32_t ghost_find(const Params& P, Rep<NT>& x, int32_t s, uint4& e) {
  if (!(x.iflags & PAXISIM_F_GHOST)) return GMAX;
  uint32_t live = 0, hit = GMAX;
  for (uint32_t g = 0; g < GMAX; g++) {
    const uint4 v = ldg(gref<NT>(P, x, g));
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
    const uint32_t until = ldg(gref<NT>(P, x, g)).z & 0x7FFFFFFFu;
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
    if (!(e.z >> 31) && b > e.y) *gref<NT>(P, x, g) = make_uint4(e.x, b, e.z, 0u);
    return;
  }
  if ((g = ghost_alloc<NT>(P, x)) < GMAX) *gref<NT>(P, x, g) = make_uint4((uint32_t)s, b, ghost_until<NT>(P, x), 0u);
}
// HandleP3 on a slot below execute: the entry exists and is committed (paxos.go:326-331)
template <int NT>
__device__ __forceinline__ void ghost_commit(const Params& P, Rep<NT>& x, int32_t s) {
  uint4 e;
  uint32_t g = ghost_find<NT>(P, x, s, e);
  if (g < GMAX) {
    *gref<NT>(P, x, g) = make_uint4(e.x, e.y, e.z | 0x80000000u, 0u);
    return;
  }
  if ((g = ghost_alloc<NT>(P, x)) < GMAX)
    *gref<NT>(P, x, g) = make_uint4((uint32_t)s, 0u, ghost_until<NT>(P, x) | 0x80000000u, 0u);
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

#ifndef PXS_P2B_EAGER
#define PXS_P2B_EAGER 0   // 1: HandleP2b reads the entry's ack word with its ballot and flags (A/B)
#endif
template <int NT>
__device__ __forceinline__ bool in_window(const Params& P, const Rep<NT>& x, int32_t s) {
  return s >= x.execute && s < x.execute + (int32_t)P.W;
}

template <int NT>
__device__ __forceinline__ void paxos_forward(const Params& P, Rep<NT>& x) {     // paxos.go:371-376
  for (uint32_t i = 0; i < x.npend; i++) {
    PXS_TALLY_AT(P, x.blk, TC_PEND, &x.pend[(size_t)i * x.pstride], false);
    node_forward<NT>(P, x, bal_id(x.ballot), ldg(&x.pend[(size_t)i * x.pstride]));
  }
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
    else {
      PXS_TALLY_AT(P, x.blk, TC_PEND, &x.pend[(size_t)x.npend * x.pstride], true);
      x.pend[(size_t)x.npend++ * x.pstride] = req;
    }
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

// Database.Execute (db.go:103-114) when replicas keep the KV: a write's value
// (its command id) goes to its key and database.version counts it (put,
// db.go:123-134); a read changes nothing.  The previous value Execute returns
// is what the key holds at this point of the executed log.
// Database.Execute's return value (db.go:103-114): the key's value before cmd.
// A plain load: only the reply's store consumes it, so the wait for it lands
// there rather than here (PXS_KV_LDG=1: wait at once, A/B).
#ifndef PXS_KV_LDG
#define PXS_KV_LDG 0
#endif
#ifndef PXS_AGREE_POST
#define PXS_AGREE_POST 1    // 0: no agreement-ring arrivals (A/B attribution only)
#endif
#ifndef PXS_REPLY_VALUE
#define PXS_REPLY_VALUE 1   // 0: replies carry no value (A/B attribution only; not the reference's behaviour)
#endif
// (the key is computed once per executed command: kv_key)
template <int NT>
__device__ __forceinline__ uint32_t kv_key(const Params& P, Rep<NT>& x, uint32_t h, uint32_t cmd) {
  // a per-key instance (HBM log: WPaxos, M2Paxos, KPaxos) only executes commands of its own key
  return hbm_log(x) ? x.key : key_fit<NT>(P, x, wl_key_h(P, h, cmd));
}
template <int NT>
__device__ __forceinline__ uint32_t kv_get(const Params& P, Rep<NT>& x, uint32_t key) {
  if (!PXS_REPLY_VALUE) return 0u;
  const uint32_t* a = &P.kv_val[((size_t)key * nrep<NT>(P) + x.r) * P.C + x.c];
  PXS_TALLY_AT(P, x.blk, TC_KV_LD, a, false);
  return PXS_KV_LDG ? ldg(a) : *a;
}
template <int NT>
__device__ __forceinline__ void kv_exec(const Params& P, Rep<NT>& x, uint32_t h, uint32_t key, uint32_t cmd) {
  if (!wl_write_h(P, h)) return;
  PXS_TALLY_AT(P, x.blk, TC_KV_ST, &P.kv_val[((size_t)key * nrep<NT>(P) + x.r) * P.C + x.c], true);
  P.kv_val[((size_t)key * nrep<NT>(P) + x.r) * P.C + x.c] = cmd;
  x.kvver++;
}

// hi / hc: the entry index and flags the caller has just written, which exec
// then does not read back.  With the window in HBM (three planes, the serial
// kernel) each slot's iteration loads the next slot's flags before it issues
// its own stores (PXS_EXEC_AHEAD), so the loop's exit test does not wait for
// them (vmcnt retires loads and stores in issue order).
// A WPaxos bind (wlds) does not load the instance's digest: exec, its only
// reader, loads it on first use, and the unbind stores it only if exec changed it.
template <int NT>
__device__ __forceinline__ void digest_need(const Params& P, Rep<NT>& x) {
  if (hbm_log(x) && P.wlds && x.dig_st == 0u) {
    PXS_TALLY_AT(P, x.blk, TC_CKPT, &P.wdig[wp_si(P, x.blk, x.key, x.r, x.lane)], false);
    x.digest = P.wdig[wp_si(P, x.blk, x.key, x.r, x.lane)];
    x.dig_st = 1u;
  }
}
#ifndef PXS_EXEC_AHEAD
#define PXS_EXEC_AHEAD 1
#endif
template <int NT>
__device__ __forceinline__ void paxos_exec(const Params& P, Rep<NT>& x, uint32_t hi = ~0u,
                                           uint32_t hc = 0u) {     // paxos.go:345-369
  uint32_t ni = ~0u, nc = 0u;                                      // the next slot's entry, loaded ahead
  for (;;) {
    if (hbm_log(x)) {                                              // skip the HBM read of an uncommitted entry
      if (P.W <= 16u ? !((x.cmask >> ((uint32_t)x.execute & (P.W - 1u))) & 1u) : x.execute > x.slot) break;
    }
    const uint32_t i = eidx<NT>(P, x, x.execute);
    const uint32_t c = i == hi ? hc : (i == ni ? nc : eb(x, i));
    hi = ~0u;
    if ((c & (EF_EXISTS | EF_COMMIT)) != (EF_EXISTS | EF_COMMIT)) break;
    if (PXS_EXEC_AHEAD && x.hw && !hbm_log(x)) {
      ni = eidx<NT>(P, x, x.execute + 1);
      nc = x.l_b[ni];
    }
    if (x.iflags & PAXISIM_F_WOVF) x.flags |= PAXISIM_F_UNFAITHFUL;
    digest_need<NT>(P, x);
    const uint32_t cmd = c & CMD_MASK;
    const uint32_t h = P.kv ? wl_hash(x.kc, cmd) : 0u;
    const uint32_t key = P.kv ? kv_key<NT>(P, x, h, cmd) : 0u;
    if (c & (EF_REQSELF | EF_REQEXT))                             // Reply{Value: p.Execute(cmd)}, paxos.go:352-362
      request_reply<NT>(P, x, ereq<NT>(P, x, i, c), cmd, P.kv ? kv_get<NT>(P, x, key) : 0u);
    x.digest = mix64(x.digest ^ (((uint64_t)(uint32_t)x.execute << 32) | cmd));
    x.dig_st = 2u;
    if (P.kv) kv_exec<NT>(P, x, h, key, cmd);                      // p.Execute(e.command), paxos.go:352
    set_b(x, i, 0u);                                               // delete(p.log, execute)
    x.execute++;
    if ((uint32_t)x.execute % CKI == 0) {
      const uint32_t k = ((uint32_t)x.execute / CKI) % CKR;
      const size_t ci = ((size_t)k * P.NI + x.inst) * P.C + x.c;
      PXS_TALLY_AT(P, x.blk, TC_CKPT, &P.ck_e[ci], true);
      PXS_TALLY_AT(P, x.blk, TC_CKPT, &P.ck_d[ci], true);
      P.ck_e[ci] = (uint32_t)x.execute;
      P.ck_d[ci] = x.digest;
      if (P.AR && PXS_AGREE_POST) agree_post<NT>(P, x, (uint32_t)x.execute / CKI);
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
    const uint32_t c = eb(x, eidx<NT>(P, x, s));
    n += (c & EF_EXISTS) && !(c & EF_COMMIT);
  }
  uint32_t ri;
  intent_flush<NT>(P, x);                                                    // keep per-link order
  if (!send_begin<NT>(P, x, bal_id(mb), 1u + n, ri)) return;
  PXS_TALLY_AT(P, x.blk, TC_REC_ST, &x.rec[ri], true);
  x.rec[ri] = make_uint4(PAXISIM_MSG_P1B | (n << 8) | x.ktag, x.ballot, 0u, 0u);
  for (int32_t s = x.execute; s <= hi; s++) {
    const Ent e = eget<NT>(x, eidx<NT>(P, x, s));
    if (!(e.c & EF_EXISTS) || (e.c & EF_COMMIT)) continue;
    ri += LANES;
    PXS_TALLY_AT(P, x.blk, TC_REC_ST, &x.rec[ri], true);
    x.rec[ri] = make_uint4(PAXISIM_MSG_P1B_ENTRY, e.b, (uint32_t)s, e.c & CMD_MASK);
  }
}

// P1b with its CommandBallot payload in the records after ri0
template <int NT>
__device__ __forceinline__ void paxos_handle_p1b(const Params& P, Rep<NT>& x, uint32_t src, uint32_t mb, uint32_t ri0,
                                              uint32_t n) {                   // paxos.go:164-230
  if (mb < x.ballot || x.active) return;
  for (uint32_t k = 0; k < n; k++) {                                          // update(): 164-180
    PXS_TALLY_AT(P, x.blk, TC_REC_LD, &x.rec[ri0 + (k + 1u) * LANES], false);
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
        const uint32_t c = eb(x, i);
        if (!(c & EF_EXISTS) || (c & EF_COMMIT)) continue;                   // nil gap (G5)
        eput<NT>(x, i, Ent{x.ballot, c | EF_QUORUM, 1u << x.r});
        post_broadcast<NT>(P, x, PAXISIM_MSG_P2A | x.ktag, x.ballot, (uint32_t)s, c & CMD_MASK);
      }
      const uint32_t np = x.npend;
      x.npend = 0;
      for (uint32_t k = 0; k < np; k++) {
        PXS_TALLY_AT(P, x.blk, TC_PEND, &x.pend[(size_t)k * x.pstride], false);
        paxos_p2a<NT>(P, x, ldg(&x.pend[(size_t)k * x.pstride]));
      }
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
          set_a(x, i, e.b);
          set_b(x, i, e.c);
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
  PXS_SUB_T0(pxs_e0)
  const uint32_t i = eidx<NT>(P, x, ms);
  const uint32_t c = eb(x, i);
  const uint32_t eb0 = ea(x, i);
  const uint32_t ea0 = PXS_P2B_EAGER ? ec(x, i) : 0u;   // (HBM window: the three words in one round trip)
  if (!(c & EF_EXISTS) || mb < eb0 || (c & EF_COMMIT)) return;
  PXS_SUB_T1(pxs_e0, 10)
  if (mb > x.ballot) {
    x.ballot = mb;
    x.active = 0;
  }
  if (bal_id(mb) == x.r && mb == eb0) {
    if (!(c & EF_QUORUM)) {                                                   // nil quorum: Go panics
      x.flags |= PAXISIM_F_POISON;
      x.stop = true;
      return;
    }
    PXS_SUB_T0(pxs_a0)
    const uint32_t ack = (PXS_P2B_EAGER ? ea0 : ec(x, i)) | (1u << src);
    set_c(x, i, ack);
    PXS_SUB_T1(pxs_a0, 11)
    if (quorum_ok(P, P.q2, ack)) {
      set_b(x, i, c | EF_COMMIT);
      x.commits++;
      post_broadcast<NT>(P, x, PAXISIM_MSG_P3 | x.ktag, mb, (uint32_t)ms, c & CMD_MASK);
      if (P.rwc) {
        const uint32_t q = ereq<NT>(P, x, i, c);
        if (!q) { x.flags |= PAXISIM_F_POISON; x.stop = true; return; }   // nil r.Reply
        request_reply<NT>(P, x, q, req_cid(q), 0u);   // Reply{Command}: no Value
      } else {
        PXS_SUB_T0(pxs_x0)
        paxos_exec<NT>(P, x, i, c | EF_COMMIT);
        PXS_SUB_T1(pxs_x0, 9)
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
    uint32_t c = eb(x, i);
    if (c & EF_EXISTS) {
      if ((c & CMD_MASK) != mcid && (c & (EF_REQSELF | EF_REQEXT))) {
        node_forward<NT>(P, x, bal_id(mb), ereq<NT>(P, x, i, c));
        c &= ~(EF_REQSELF | EF_REQEXT);
      }
    } else {
      c = EF_EXISTS;                                                          // &entry{} (G6)
      set_a(x, i, 0u);
      set_c(x, i, 0u);
    }
    c = eset_cmd<NT>(P, x, i, c, mcid) | EF_COMMIT;
    set_b(x, i, c);
    if (P.rwc) {
      if (c & (EF_REQSELF | EF_REQEXT)) {
        const uint32_t q = ereq<NT>(P, x, i, c);
        request_reply<NT>(P, x, q, req_cid(q), 0u);   // Reply{Command}: no Value
      }
      return;
    }
    PXS_SUB_T0(pxs_x1)
    paxos_exec<NT>(P, x, i, c);
    PXS_SUB_T1(pxs_x1, 5)
    return;
  } else if (ms < x.execute) {
    ghost_commit<NT>(P, x, ms);
  } else {
    raise_win(x, PAXISIM_F_WOVF);
  }
  if (!P.rwc) paxos_exec<NT>(P, x);
}

// HandleP2b (paxos.go:270-310) for a P2b that neither completes a quorum nor
// poisons, on the bound instance: returns true after applying it exactly as
// paxos_handle_p2b would (ignored: no entry (G7), m.Ballot < e.ballot,
// committed, or outside the window where no flag can be raised; else adopt a
// higher ballot and record the ack).  Returns false, with no effect, for every
// other P2b.
template <int NT>
__device__ __forceinline__ bool p2b_absorb(const Params& P, Rep<NT>& x, uint32_t src, const uint4& m) {
  const int32_t ms = (int32_t)m.z;
  const uint32_t mb = m.y;
  if (!in_window<NT>(P, x, ms))
    return ms < x.execute ? !(x.iflags & PAXISIM_F_GHOST) : !(x.iflags & PAXISIM_F_WOVF);
  const uint32_t i = eidx<NT>(P, x, ms);
  const uint32_t c = eb(x, i);
  const uint32_t eb0 = ea(x, i);
  const uint32_t ea0 = PXS_P2B_EAGER ? ec(x, i) : 0u;
  if (!(c & EF_EXISTS) || mb < eb0 || (c & EF_COMMIT)) return true;
  if (bal_id(mb) == x.r && mb == eb0) {
    if (!(c & EF_QUORUM)) return false;                 // nil quorum: the full handler poisons
    const uint32_t ack = (PXS_P2B_EAGER ? ea0 : ec(x, i)) | (1u << src);
    if (quorum_ok(P, P.q2, ack)) return false;          // commit: the full handler
    set_c(x, i, ack);
  }
  if (mb > x.ballot) {
    x.ballot = mb;
    x.active = 0;
  }
  return true;
}

// ---------------------------------------------------------------------------
// protocol policy
// ---------------------------------------------------------------------------
struct PaxosProto {
  static constexpr uint32_t kind = PAXISIM_PAXOS;
  static constexpr bool step_scratch = false;   // (no per-replica-step LDS scratch: sim_core.h sim_serial)
  template <int NT>
  __device__ static __forceinline__ void load(const Params& P, Rep<NT>& x) {
    const size_t i = rc(P, x.r, x.c);
#ifdef PXS_TALLY
    PXS_TALLY_AT(P, x.blk, TC_ROW_LD, &P.ballot[i], false);
    PXS_TALLY_AT(P, x.blk, TC_ROW_LD, &P.slot[i], false);
    PXS_TALLY_AT(P, x.blk, TC_ROW_LD, &P.execute[i], false);
    PXS_TALLY_AT(P, x.blk, TC_ROW_LD, &P.meta[i], false);
    PXS_TALLY_AT(P, x.blk, TC_ROW_LD, &P.npend[i], false);
    PXS_TALLY_AT(P, x.blk, TC_ROW_LD, &P.nfwd[i], false);
    PXS_TALLY_AT(P, x.blk, TC_ROW_LD, &P.digest[i], false);
#endif
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
#ifdef PXS_TALLY
    PXS_TALLY_AT(P, x.blk, TC_ROW_ST, &P.ballot[i], true);
    PXS_TALLY_AT(P, x.blk, TC_ROW_ST, &P.slot[i], true);
    PXS_TALLY_AT(P, x.blk, TC_ROW_ST, &P.execute[i], true);
    PXS_TALLY_AT(P, x.blk, TC_ROW_ST, &P.meta[i], true);
    PXS_TALLY_AT(P, x.blk, TC_ROW_ST, &P.npend[i], true);
    PXS_TALLY_AT(P, x.blk, TC_ROW_ST, &P.nfwd[i], true);
    PXS_TALLY_AT(P, x.blk, TC_ROW_ST, &P.digest[i], true);
#endif
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
  // a P2b that completes no quorum is handled in the trip before it (sim_core.h)
  template <int NT>
  __device__ static __forceinline__ bool absorb(const Params& P, Rep<NT>& x, uint32_t src, const uint4& m) {
    return hdr_type(m.x) == PAXISIM_MSG_P2B && p2b_absorb<NT>(P, x, src, m);
  }
  // node.handle dispatch (node.go:104-115; registrations paxos/replica.go:33-38)
  template <int NT>
  __device__ static __forceinline__ void dispatch(const Params& P, Rep<NT>& x, uint32_t src, const uint4& m,
                                                  uint32_t ri) {
    switch (hdr_type(m.x)) {
      case PAXISIM_MSG_REQUEST: { PXS_CASE_T0 dv_inc<NT>(x, PAXISIM_MSG_REQUEST); handle_request<NT>(P, x, mkreq(m.w, src)); PXS_CASE_T1(PAXISIM_MSG_REQUEST) } break;
      case PAXISIM_MSG_REPLY: { PXS_CASE_T0 dv_inc<NT>(x, PAXISIM_MSG_REPLY); handle_reply<NT>(P, x, m.w, m.y); PXS_CASE_T1(PAXISIM_MSG_REPLY) } break;
      case PAXISIM_MSG_P1A: { PXS_CASE_T0 dv_inc<NT>(x, PAXISIM_MSG_P1A); paxos_handle_p1a<NT>(P, x, m.y); PXS_CASE_T1(PAXISIM_MSG_P1A) } break;
      case PAXISIM_MSG_P1B: { PXS_CASE_T0 dv_inc<NT>(x, PAXISIM_MSG_P1B); paxos_handle_p1b<NT>(P, x, src, m.y, ri, hdr_n(m.x)); PXS_CASE_T1(PAXISIM_MSG_P1B) } break;
      case PAXISIM_MSG_P2A: { PXS_CASE_T0 dv_inc<NT>(x, PAXISIM_MSG_P2A); paxos_handle_p2a<NT>(P, x, m.y, (int32_t)m.z, m.w); PXS_CASE_T1(PAXISIM_MSG_P2A) } break;
      case PAXISIM_MSG_P2B: { PXS_CASE_T0 dv_inc<NT>(x, PAXISIM_MSG_P2B); paxos_handle_p2b<NT>(P, x, src, m.y, (int32_t)m.z); PXS_CASE_T1(PAXISIM_MSG_P2B) } break;
      case PAXISIM_MSG_P3: { PXS_CASE_T0 dv_inc<NT>(x, PAXISIM_MSG_P3); paxos_handle_p3<NT>(P, x, m.y, (int32_t)m.z, m.w); PXS_CASE_T1(PAXISIM_MSG_P3) } break;
      default: break;
    }
  }
};

}  // namespace pxs
