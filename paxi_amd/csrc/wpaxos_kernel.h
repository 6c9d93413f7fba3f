// wpaxos_kernel.h — WPaxos handlers on gfx950 (a protocol policy of sim_core.h).
//
// Follows wpaxos/replica.go:42-108 and wpaxos/kpaxos.go:15-74 (cited per
// function).  A WPaxos replica holds one paxos.Paxos ("kpaxos") per key,
// created on first use (Replica.init, replica.go:36-40), with Q1/Q2 =
// GridRow/GridColumn (fz = 0) or FGridQ1/Q2(fz) (kpaxos.go:15-27).  The kpaxos
// Broadcast/Send wrappers (kpaxos.go:51-74) tag P1a..P3 with the key; here the
// tag rides in the record header (x.ktag = key << 16).  Leaders migrate by the
// consecutive policy (policy.go:49-69): after `threshold` consecutive requests
// forwarded by one node of another zone, the leader sends that node a
// LeaderChange and it steals the key with a phase-1 (replica.go:101-108).
//
// The Paxos handlers are paxos_kernel.h's, run on the bound instance: a
// dispatch loads the key's instance registers from HBM, runs the handler and
// writes them back.  Instance state of 64 clusters x 9 replicas x K keys does
// not fit a workgroup's LDS, so it stays in HBM, laid out per (block, key,
// replica, lane) so that one lane's state, window and pending list are each
// contiguous:
//   wst   [blk][K][N][64] x 32 B  {ballot, slot, execute, active|exists<<1|wovf,ghost<<2|p1acks<<16,
//                                   npend, digest, policy last|hits<<8 | committed window slots<<16}
//   wlog  [blk][K][N][64][W] x 16 B {ballot, cmd|flags, acks, request}
//   wpend [blk][K][N][64][PMAX] x 4 B
#pragma once
#include "paxos_kernel.h"

namespace pxs {

// The majority / ema policies run only on a leader's request path; built out
// of line (PXS_POLICY_NOINLINE=1) they stay out of the merge loop's registers.
#if defined(PXS_POLICY_NOINLINE) && PXS_POLICY_NOINLINE
#define PXS_POLICY_FN __device__ __attribute__((noinline))
#else
#define PXS_POLICY_FN __device__ __forceinline__
#endif

template <int NT>
__device__ __forceinline__ size_t wp_slot(const Params& P, const Rep<NT>& x, uint32_t key) {
  if (PXS_WP_LANEMAJOR) return (((size_t)x.blk * nrep<NT>(P) + x.r) * LANES + x.lane) * P.keys + key;
  return (((size_t)x.blk * P.keys + key) * nrep<NT>(P) + x.r) * LANES + x.lane;
}

// bind the kpaxos of `key`: its registers, its window and pending list.  The
// scalars come from LDS (LDS: the tile image holds them, wlds) or from the HBM
// table; the digest, which only exec() reads, from HBM either way.
template <int NT, bool LDS>
__device__ __forceinline__ void wp_bind(const Params& P, Rep<NT>& x, uint32_t key) {
  const size_t si = wp_slot<NT>(P, x, key);
  uint4 a, b;
  if constexpr (LDS) {
    const uint32_t* w = x.l_inst + key * x.ikst + x.iro + x.lane;
    a = make_uint4(w[0], w[64], w[128], w[192]);
    b.w = w[256];
    b.x = (a.w >> 4) & 0x3Fu;
    a.w &= 0xFFFF000Fu;
    b.y = b.z = 0u;                  // the digest: loaded by exec when it needs it (digest_need)
    x.dig_st = 0u;
  } else {
    PXS_TALLY_AT(P, x.blk, TC_INST_LD, &P.wst[(size_t)P.wst_str * si], false);
    a = P.wst[(size_t)P.wst_str * si];
    b = P.wst[(size_t)P.wst_str * si + 1];
  }
  x.key = key;
  x.ktag = key << 16;
  x.inst = key * nrep<NT>(P) + x.r;
  x.ballot = a.x;
  x.slot = (int32_t)a.y;
  x.execute = (int32_t)a.z;
  x.active = a.w & 1u;
  x.exists = (a.w >> 1) & 1u;
  x.iflags = (a.w >> 2) & (PAXISIM_F_WOVF | PAXISIM_F_GHOST);
  x.p1mask = a.w >> 16;
  x.npend = b.x;
  x.digest = (uint64_t)b.y | ((uint64_t)b.z << 32);
  if constexpr (!LDS) x.dig_st = 1u;
  x.pol = b.w & 0xFFFFu;
  x.cmask = b.w >> 16;
  uint32_t* lb = P.wlog + si * P.wlog_str;
  x.l_a = lb;
  x.l_b = lb + 1;
  x.l_c = lb + 2;
  x.reqx = lb + 3;
  x.pend = P.wpend + si * PMAX;
  x.ci = ~0u;                        // the entry cache belongs to the bound window
}
template <int NT, bool LDS>
__device__ __forceinline__ void wp_unbind(const Params& P, const Rep<NT>& x) {
  const size_t si = wp_slot<NT>(P, x, x.key);
  const uint32_t meta = (x.active & 1u) | (x.exists << 1) | (x.iflags << 2) | (x.p1mask << 16);
  if constexpr (LDS) {
    uint32_t* w = x.l_inst + x.key * x.ikst + x.iro + x.lane;
    w[0] = x.ballot;
    w[64] = (uint32_t)x.slot;
    w[128] = (uint32_t)x.execute;
    w[192] = meta | (x.npend << 4);
    w[256] = x.pol | (x.cmask << 16);
    if (x.dig_st == 2u) P.wdig[si] = x.digest;
  } else {
    PXS_TALLY_AT(P, x.blk, TC_INST_ST, &P.wst[(size_t)P.wst_str * si], true);
    P.wst[(size_t)P.wst_str * si] = make_uint4(x.ballot, (uint32_t)x.slot, (uint32_t)x.execute, meta);
    P.wst[(size_t)P.wst_str * si + 1] = make_uint4(x.npend, (uint32_t)x.digest, (uint32_t)(x.digest >> 32), x.pol | (x.cmask << 16));
  }
}

// r.paxi[m.Key] without a prior init: a nil *kpaxos, whose use panics in Go
template <int NT>
__device__ __forceinline__ bool wp_get(Rep<NT>& x) {
  if (x.exists) return true;
  x.flags |= PAXISIM_F_POISON;
  x.stop = true;
  return false;
}

// Replica.init (replica.go:36-40): a new kpaxos gets a new policy, whose
// majority interval starts now (policy.go:35, NewPolicy)
template <int NT>
__device__ __forceinline__ void wp_create(const Params& P, Rep<NT>& x) {
  if (!x.exists && P.policy == PAXISIM_POLICY_MAJORITY)
    PXS_TALLY_AT(P, x.blk, TC_OTHER, &P.wpx[3 * wp_slot<NT>(P, x, x.key) + 2], true);
  if (!x.exists && P.policy == PAXISIM_POLICY_MAJORITY)
    P.wpx[3 * wp_slot<NT>(P, x, x.key) + 2] = make_uint4(0u, x.t, 0u, 0u);
  x.exists = 1;
}

// majority.Hit (policy.go:79-93), the step as the clock; ids visited in index
// order where Go ranges over a map, so the highest qualifying index wins
template <int NT>
PXS_POLICY_FN uint32_t majority_hit(uint4* q, uint32_t t, uint32_t id, uint32_t n, uint32_t interval) {
  const uint4 h0 = q[0], h1 = q[1];
  uint4 m = q[2];
  uint32_t w[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
  const uint32_t sh = (id & 1u) * 16u;
#pragma unroll
  for (uint32_t k = 0; k < 8; k++)
    if (k == (id >> 1) && ((w[k] >> sh) & 0xFFFFu) < 0xFFFFu) w[k] += 1u << sh;   // saturating u16
  m.x++;
  uint32_t res = POL_NONE;
  if (m.x > 1u && t - m.y >= interval) {
#pragma unroll
    for (uint32_t i = 0; i < 16; i++)
      if (i < n && ((w[i >> 1] >> ((i & 1u) * 16u)) & 0xFFFFu) >= m.x / 2u) res = i;
#pragma unroll
    for (uint32_t k = 0; k < 8; k++) w[k] = 0;                                   // reset (policy.go:95-101)
    m.x = 0;
    m.y = t;
  }
  q[0] = make_uint4(w[0], w[1], w[2], w[3]);
  q[1] = make_uint4(w[4], w[5], w[6], w[7]);
  q[2] = m;
  return res;
}

// ema.Hit (policy.go:111-130): every operation rounded on its own, as the
// oracle computes it.  Measured: __dmul_rn/__dadd_rn alone still let the
// compiler fuse the product into the sum (1-ulp parity failures), so the
// products go through an asm barrier.  Returns the new settled zone
// (1-based), or 0.
template <int NT>
PXS_POLICY_FN uint32_t ema_hit(uint4* q, double alpha, double zid) {
  uint4 m = q[2];
  double s = __hiloint2double((int)m.y, (int)m.x);
  uint32_t res = 0;
  if (s == 0.0) {
    s = zid;
  } else {
#pragma clang fp contract(off)
    double t1 = alpha * zid;
    double t3 = (1.0 - alpha) * s;
    asm volatile("" : "+v"(t1), "+v"(t3));   // the products are rounded before the sum: no FMA
    s = t1 + t3;
    if (!(fabs(s - round(s)) > 0.1)) {
      const uint32_t z = (uint32_t)(int32_t)round(s);
      if (z != m.z) {
        m.z = z;
        res = z;
      }
    }
  }
  m.x = (uint32_t)__double2loint(s);
  m.y = (uint32_t)__double2hiint(s);
  q[2] = m;
  return res;
}

// consecutive.Hit (policy.go:55-69); threshold 0 is the null policy (policy.go:18-21)
template <int NT>
__device__ __forceinline__ uint32_t policy_hit(const Params& P, Rep<NT>& x, uint32_t id) {
  if (P.policy == PAXISIM_POLICY_MAJORITY)
    return majority_hit<NT>(P.wpx + 3 * wp_slot<NT>(P, x, x.key), x.t, id, nrep<NT>(P), P.policy_interval);
  if (P.policy == PAXISIM_POLICY_EMA) {
    const uint32_t z = ema_hit<NT>(P.wpx + 3 * wp_slot<NT>(P, x, x.key), P.policy_alpha,
                                   (double)(P.zone_of[id] + 1u));
    return z ? (uint32_t)__ffs(P.zmask[z - 1u]) - 1u : POL_NONE;                 // NewID(z, 1)
  }
  if (P.policy_thr == 0) return POL_NONE;
  uint32_t last = x.pol & 0xFFu, hits = x.pol >> 8;
  if (id == last) {
    hits++;
  } else {
    last = id;
    hits = 1;
  }
  uint32_t res = POL_NONE;
  if (hits >= P.policy_thr) {
    res = last;
    last = POL_NONE;
    hits = 0;
  }
  x.pol = last | (hits << 8);
  return res;
}

// KPaxos index() (kpaxos/replica.go:32-44): the static leader of a key is
// "z.1" with z = 1 + key / 200 (at most 5); an ID that is not in the
// configuration is an unknown address, whose sends are dropped (socket.go:86-88).
template <int NT>
__device__ __forceinline__ uint32_t kp_leader(const Params& P, uint32_t key) {
  const uint32_t z = key < 800u ? key / 200u : 4u;
  return z < P.Z ? P.zfirst[z] : NO_ID;
}

template <int NT>
__device__ __forceinline__ void wp_handle_request(const Params& P, Rep<NT>& x, uint32_t req) {  // replica.go:42-66
  wp_create<NT>(P, x);                                                 // r.init(key)
  if (P.variant == PAXISIM_KPAXOS) {                                   // kpaxos/replica.go:52-62
    const uint32_t leader = kp_leader<NT>(P, key_value(P, x.key));
    if (leader == x.r) paxos_handle_request<NT>(P, x, req);
    else node_forward<NT>(P, x, leader, req);                          // `go r.Forward(leader, m)`
    return;
  }
  if (!P.adaptive) {
    paxos_handle_request<NT>(P, x, req);
    return;
  }
  if (x.active || bal_id(x.ballot) == x.r || x.ballot == 0) {        // p.IsLeader() || p.Ballot() == 0
    paxos_handle_request<NT>(P, x, req);
    // m.NodeID: the receiving node for an HTTP request (http.go:96), the forwarder otherwise (node.go:167)
    const uint32_t o = req_origin(req);
    const uint32_t to = policy_hit<NT>(P, x, o == PAXISIM_CLIENT_SRC ? x.r : o);
    if (to != POL_NONE && P.zone_of[to] != P.zone_of[x.r])            // LeaderChange{Key, To, From, Ballot}
      post_unicast<NT>(P, x, to, PAXISIM_MSG_LEADERCHG | x.ktag, x.ballot, to, x.r);
  } else {
    node_forward<NT>(P, x, bal_id(x.ballot), req);                     // `go r.Forward(p.Leader(), m)`
  }
}

// Same-trip absorption of a P2b for the kpaxos still bound.
//   0: off (default).
//   1: the round-4 r4l experiment as DESIGN.md §5.6 describes it: the next
//      P2b of the bound key runs p2b_absorb on the bound registers after the
//      dispatch's unbind, and nothing writes them back again; nor is "bound"
//      checked (load() leaves key 0 with another instance's registers).  A
//      diagnostic build only: it loses HandleP2b's ballot adoption
//      (paxos.go:281-284) whenever the absorbed P2b carries a higher ballot.
//   2: the same absorption with an explicit bound key (none after load()) and
//      the instance written back when the absorbed P2b changed ballot/active.
// (the macro is defined in sim_core.h, whose merge loop calls absorb)
constexpr uint32_t WP_UNBOUND = 0xFFFFu;   // x.key before the first bind of a replica-step (PXS_WP_ABSORB=2)

// LDS: the instance scalars live in the tile's LDS image (wlds); else in HBM
template <bool LDS>
struct WPaxosProtoT {
  static constexpr uint32_t kind = PAXISIM_WPAXOS;
  template <int NT>
  __device__ static __forceinline__ void load(const Params& P, Rep<NT>& x) {
    PXS_TALLY_AT(P, x.blk, TC_ROW_LD, &P.nfwd[rc(P, x.r, x.c)], false);
    x.l_inst = x.l_a;                // image region a: the instance scalars (LDS layout)
    x.ikst = (nrep<NT>(P) * WP_WORDS) << 6;
    x.iro = (x.r * WP_WORDS) << 6;
    x.nfwd = P.nfwd[rc(P, x.r, x.c)];
    x.e0 = 0;                        // entry of slot s: word 4*(s & (W-1)) of the lane's window
    x.es = 4;
    x.pstride = 1;
    x.key = PXS_WP_ABSORB >= 2 ? WP_UNBOUND : 0u;
    x.ktag = 0;
  }
  // HandleP2b (paxos.go:270-310) of a next message in the same trip, without
  // a bind: only a P2b of the kpaxos whose registers are bound, and only when
  // it completes no quorum (p2b_absorb).  handleAccepted (replica.go:90-93)
  // first dereferences r.paxi[m.Key]: a nil kpaxos goes to the full handler,
  // which poisons.
  template <int NT>
  __device__ static __forceinline__ bool absorb(const Params& P, Rep<NT>& x, uint32_t src, const uint4& m) {
    if (hdr_type(m.x) != PAXISIM_MSG_P2B || hdr_key(m.x) != x.key || !x.exists) return false;
    const uint32_t b0 = x.ballot, a0 = x.active;
    if (!p2b_absorb<NT>(P, x, src, m)) return false;
    if (PXS_WP_ABSORB >= 2 && (x.ballot != b0 || x.active != a0)) wp_unbind<NT, LDS>(P, x);
    return true;
  }
  template <int NT>
  __device__ static __forceinline__ void store(const Params& P, const Rep<NT>& x) {
    PXS_TALLY_AT(P, x.blk, TC_ROW_ST, &P.nfwd[rc(P, x.r, x.c)], true);
    P.nfwd[rc(P, x.r, x.c)] = x.nfwd;
  }
  // The serial kernel (sim_core.h) runs one replica at a time: the instance
  // scalars of that replica's K kpaxos move from the HBM image into an LDS
  // scratch [key][word][lane] for its replica-step (one coalesced copy each
  // way), so a bind / unbind is LDS traffic rather than eight keys' worth of
  // scattered HBM rows per wave.
  static constexpr bool step_scratch = LDS && PXS_WP_SCRATCH;
  template <int NT>
  __device__ static __forceinline__ void step_begin(const Params& P, Rep<NT>& x, uint8_t* scr) {
    uint32_t* s = reinterpret_cast<uint32_t*>(scr);
    const uint32_t* g = reinterpret_cast<const uint32_t*>(P.image + (size_t)x.blk * P.img.bytes + P.img.off_a) +
                        ((x.r * WP_WORDS) << 6) + x.lane;
    const uint32_t gk = (nrep<NT>(P) * WP_WORDS) << 6;
    for (uint32_t k = 0; k < P.keys; k++)
#pragma unroll
      for (uint32_t w = 0; w < WP_WORDS; w++) s[((k * WP_WORDS + w) << 6) + x.lane] = g[k * gk + (w << 6)];
    x.l_inst = s;
    x.ikst = WP_WORDS << 6;
    x.iro = 0;
  }
  template <int NT>
  __device__ static __forceinline__ void step_end(const Params& P, const Rep<NT>& x) {
    const uint32_t* s = x.l_inst;
    uint32_t* g = reinterpret_cast<uint32_t*>(P.image + (size_t)x.blk * P.img.bytes + P.img.off_a) +
                  ((x.r * WP_WORDS) << 6) + x.lane;
    const uint32_t gk = (nrep<NT>(P) * WP_WORDS) << 6;
    for (uint32_t k = 0; k < P.keys; k++)
#pragma unroll
      for (uint32_t w = 0; w < WP_WORDS; w++) g[k * gk + (w << 6)] = s[((k * WP_WORDS + w) << 6) + x.lane];
  }
  template <int NT>
  __device__ static __forceinline__ void client_request(const Params& P, Rep<NT>& x, uint32_t cid) {
    PXS_CASE_T0
    wp_bind<NT, LDS>(P, x, key_fit<NT>(P, x, wl_key(P, x.kc, cid)));
    wp_handle_request<NT>(P, x, mkreq(cid, PAXISIM_CLIENT_SRC));
    wp_unbind<NT, LDS>(P, x);
    PXS_CASE_T1(0)
  }
  // registrations replica.go:25-32
  template <int NT>
  __device__ static __forceinline__ void dispatch(const Params& P, Rep<NT>& x, uint32_t src, const uint4& m,
                                                  uint32_t ri) {
    const uint32_t type = hdr_type(m.x);
    if (type == PAXISIM_MSG_REPLY) {                                   // node.recv (node.go:83-90)
      PXS_CASE_T0
      dv_inc<NT>(x, PAXISIM_MSG_REPLY);
      handle_reply<NT>(P, x, m.w, m.y);
      PXS_CASE_T1(PAXISIM_MSG_REPLY)
      return;
    }
    {
      PXS_CASE_T0
      wp_bind<NT, LDS>(P, x, type == PAXISIM_MSG_REQUEST ? key_fit<NT>(P, x, wl_key(P, x.kc, m.w)) : hdr_key(m.x));
      // the entry of the message's slot (P2a / P2b / P3; harmless for the
      // others: any slot indexes the window): its load goes out with the bind's
      ecache<NT>(x, (m.z & (P.W - 1u)) * 4u);
      PXS_CASE_T1(14)
    }
    bool clean = false;                                                // instance state unchanged
    switch (type) {
      case PAXISIM_MSG_REQUEST:
        { PXS_CASE_T0
        dv_inc<NT>(x, PAXISIM_MSG_REQUEST);
        wp_handle_request<NT>(P, x, mkreq(m.w, src));
        PXS_CASE_T1(PAXISIM_MSG_REQUEST) }
        break;
      case PAXISIM_MSG_P1A:                                            // handlePrepare 72-76
        { PXS_CASE_T0
        dv_inc<NT>(x, PAXISIM_MSG_P1A);
        wp_create<NT>(P, x);
        paxos_handle_p1a<NT>(P, x, m.y);
        PXS_CASE_T1(PAXISIM_MSG_P1A) }
        break;
      case PAXISIM_MSG_P1B:                                            // handlePromise 78-82
        { PXS_CASE_T0
        dv_inc<NT>(x, PAXISIM_MSG_P1B);
        if (wp_get<NT>(x)) paxos_handle_p1b<NT>(P, x, src, m.y, ri, hdr_n(m.x));
        PXS_CASE_T1(PAXISIM_MSG_P1B) }
        break;
      case PAXISIM_MSG_P2A:                                            // handleAccept 84-88
        { PXS_CASE_T0
        dv_inc<NT>(x, PAXISIM_MSG_P2A);
        wp_create<NT>(P, x);
        paxos_handle_p2a<NT>(P, x, m.y, (int32_t)m.z, m.w);
        PXS_CASE_T1(PAXISIM_MSG_P2A) }
        break;
      case PAXISIM_MSG_P2B:                                            // handleAccepted 90-93
        { PXS_CASE_T0
        dv_inc<NT>(x, PAXISIM_MSG_P2B);
        // most P2bs change only their entry (an ack, or nothing): the instance
        // state then needs no write-back
        const uint32_t b0 = x.ballot, e0 = (uint32_t)x.execute, f0 = x.iflags, m0 = x.cmask;
        if (wp_get<NT>(x)) paxos_handle_p2b<NT>(P, x, src, m.y, (int32_t)m.z);
        clean = !x.stop && x.ballot == b0 && (uint32_t)x.execute == e0 && x.iflags == f0 && x.cmask == m0;
        PXS_CASE_T1(PAXISIM_MSG_P2B) }
        break;
      case PAXISIM_MSG_P3:                                             // handleCommit 95-99
        { PXS_CASE_T0
        dv_inc<NT>(x, PAXISIM_MSG_P3);
        wp_create<NT>(P, x);
        paxos_handle_p3<NT>(P, x, m.y, (int32_t)m.z, m.w);
        PXS_CASE_T1(PAXISIM_MSG_P3) }
        break;
      case PAXISIM_MSG_LEADERCHG:                                      // handleLeaderChange 101-108
        { PXS_CASE_T0
        dv_inc<NT>(x, PAXISIM_MSG_LEADERCHG);
        if (wp_get<NT>(x) && m.y == x.ballot && m.z == x.r) paxos_p1a<NT>(P, x);
        PXS_CASE_T1(PAXISIM_MSG_LEADERCHG) }
        break;
      default: break;
    }
    {
      PXS_CASE_T0
      if (!clean) wp_unbind<NT, LDS>(P, x);
      PXS_CASE_T1(15)
    }
  }
};

using WPaxosProto = WPaxosProtoT<false>;
using WPaxosProtoL = WPaxosProtoT<true>;

}  // namespace pxs
