// sim_core.h — protocol-independent machinery of one replica-step on gfx950.
//
// A workgroup is N waves x 64 lanes: wave r plays replica r, lane l plays
// cluster 64*blk + l.  This file holds what every protocol shares: the
// replica's register state, the socket fault filter (socket.go:66-109), the
// bucketed mailboxes, the PRNG-driven merge of per-source FIFO inboxes with
// a one-message-ahead record prefetch, the closed-loop client
// (benchmark.go:246-275) and the launch skeleton that stages the workgroup's
// LDS image.  A protocol plugs in as a policy class with
//   static void load(P, x) / store(P, x)        registers <-> HBM per launch
//   static void dispatch(P, x, src, m, ri)      node.handle (node.go:104-115)
//   static void client_request(P, x, cid)       the HTTP request path (http.go:99)
#pragma once
#include "paxisim_dev.h"

namespace pxs {

template <int NT>
struct Rep {
  static constexpr uint32_t NL = NT ? (uint32_t)NT : (uint32_t)PAXISIM_MAX_N;  // link registers
  uint64_t c, gid;                      // global lane / cluster id
  uint32_t lane, r, t, b0, hs, kc, blk;
  // protocol registers (Paxos: ballot..digest; ABD: slot = op counter, execute = history length)
  uint32_t ballot;
  int32_t slot, execute;
  uint32_t active, p1mask, flags, npend, nfwd;
  uint64_t digest;
  // the bound Paxos instance (Multi-Paxos: the replica's one; WPaxos: one kpaxos per key)
  uint32_t inst;                        // instance index in [NI] tables (key * N + r)
  uint32_t ktag;                        // WPaxos: key << 16, tagged onto P1a..P3 records
  uint32_t key, exists, pol;            // WPaxos: key, r.paxi[key] != nil, policy last | hits << 8
  uint32_t iflags;                      // WOVF / GHOST of the bound instance
  uint32_t e0, es;                      // log entry i of slot s: e0 + (s & (W-1)) * es
  uint4 ce;                             // HBM-resident window (es = 4): entry at word ci, cached (paxos_kernel.h)
  uint32_t ci;
  uint32_t cmask;                       // HBM-resident window: committed entries, one bit per window slot (W <= 16)
  bool hw;                              // the log window is in HBM (a kernel constant: sim_serial)
  uint32_t* reqx;                       // request side table, indexed like the log
  uint32_t* pend;                       // pending request k at pend[k * pstride]
  uint32_t pstride;
  uint32_t dvp[PAXISIM_NMSG / 2];       // delivered by type, two 16-bit counts per word (constant-indexed)
  uint32_t client, sent, dropped, discarded, commits, replies;
  uint32_t kvver;                       // database.version (P.kv)
  uint32_t send_seq;
  uint32_t rw, rv;                      // a client reply's value not yet stored: worker + 1 (0 = none), value
  uint32_t dmask, fmask;                // per-step: dropped / flaky destinations
  uint32_t im;                          // pending send intent: destination mask (0 = none)
  uint32_t iw0, iw1, iw2, iw3;          // pending send intent: the record
  uint64_t dly;                         // per-step: 4-bit delay per destination
  bool stop, crashed;
  // LDS views
  uint32_t *l_a, *l_b, *l_c, *l_wcur, *l_wiss, *l_poison;
  uint8_t* l_cnt;
  uint8_t* l_agn;                       // agreement-ring arrivals this step, [parity][r][lane] (agree_post)
#ifdef PXS_TALLY
  unsigned long long* tdbg;             // PXS_TALLY: P.dbg, for the handlers that only see x
#endif
  uint32_t* l_inst;                     // WPaxos (wlds): instance scalars in LDS (wpaxos_kernel.h)
  uint32_t ikst, iro;                   // WPaxos (wlds): word offsets of key k / this replica in l_inst
  uint32_t dig_st;                      // WPaxos (wlds): bound instance's digest 0 not loaded, 1 loaded, 2 changed
  uint4* rec;                           // this block's record region
};

template <int NT>
__device__ __forceinline__ uint32_t nrep(const Params& P) { return NT ? (uint32_t)NT : P.N; }

// delivered-by-type counters: 16 bits each, two per register (a launch's
// steps are capped so that no count can reach 2^16, paxisim.hip)
template <int NT>
__device__ __forceinline__ void dv_inc(Rep<NT>& x, uint32_t k) { x.dvp[k >> 1] += (k & 1u) ? 0x10000u : 1u; }
template <int NT>
__device__ __forceinline__ uint32_t dv_get(const Rep<NT>& x, uint32_t k) { return (x.dvp[k >> 1] >> ((k & 1u) * 16u)) & 0xFFFFu; }

// A global load consumed on the spot.  vmcnt counts stores too, so a load
// whose use lies behind a handler's record stores makes the compiler wait for
// those stores; retiring the load inside its own branch keeps that wait off
// the staged (LDS) path that merges with it.
__device__ __forceinline__ uint4 load_now(const uint4* p) { return ldg(p); }

// The empty asm keeps LLVM from folding a select chain back into an alloca +
// dynamic index (which would put the register array in scratch memory).
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
// socket.Send (socket.go:66-109): crash -> drop -> flaky -> slow, then the
// bounded (link, arrival-step) bucket.  Returns the record index to write.
// ---------------------------------------------------------------------------
// One exit (PXS_SEND_ONE_EXIT, on): the filter's verdict is a value and the
// drop is counted once at the end.  The early-return form - a return inside
// the divergent Flaky branch - is the shape LLVM has miscompiled in three
// builds (a register live across the branch held the Flaky
// probability, or another stale value, on the dropping lanes' path to the
// join); with one exit neither reproducer of round 5 diverges
// (gpurun_out/r5l).  0 keeps the early returns (A/B, reproducers).
#ifndef PXS_SEND_ONE_EXIT
#define PXS_SEND_ONE_EXIT 1
#endif
template <int NT>
__device__ __forceinline__ bool send_begin(const Params& P, Rep<NT>& x, uint32_t to, uint32_t nrec, uint32_t& ri) {
  const uint32_t seq = x.send_seq++;
  x.sent++;
  if constexpr (PXS_SEND_ONE_EXIT) {
    // crash, unknown id (socket.go:86-88) and drop were folded into dmask at step start
    bool ok = to < nrep<NT>(P) && !((x.dmask >> to) & 1u);
    if (ok && ((x.fmask >> to) & 1u)) {                // flaky (socket.go:77-81), scripted only
      uint32_t p = 0;
      scripted(P, PAXISIM_FAULT_FLAKY, x.gid, x.r, to, x.t, &p);
      ok = !ppm_hit(draw(x.hs, tag(PUR_FLAKY, x.r, seq)), p);
    }
    // slow (socket.go:99-106); `to & 15` keeps the shift defined for an unknown id,
    // whose bucket is never written
    uint32_t b = x.b0 + 1u + (uint32_t)((x.dly >> (4u * (to & 15u))) & 15u);
    if (b >= P.D) b -= P.D;
    const uint32_t box = (b * nrep<NT>(P) + (ok ? to : 0u)) * P.NS + x.r;
    const uint32_t k = ok ? (uint32_t)x.l_cnt[(box << 6) | x.lane] : 0u;
    const bool ovf = ok && k + nrec > P.M;
    if (ovf) x.flags |= PAXISIM_F_MBOX_OVF | PAXISIM_F_UNFAITHFUL;
    ok = ok && !ovf;
    x.dropped += ok ? 0u : 1u;
    if (ok) x.l_cnt[(box << 6) | x.lane] = (uint8_t)(k + nrec);
    ri = ((box * P.M + k) << 6) | x.lane;
    return ok;
  }
  // crash, unknown id (socket.go:86-88) and drop were folded into dmask at step start
  if (to >= nrep<NT>(P) || ((x.dmask >> to) & 1u)) { x.dropped++; return false; }
  if ((x.fmask >> to) & 1u) {                          // flaky (socket.go:77-81), scripted only
    uint32_t p = 0;
    scripted(P, PAXISIM_FAULT_FLAKY, x.gid, x.r, to, x.t, &p);
    if (ppm_hit(draw(x.hs, tag(PUR_FLAKY, x.r, seq)), p)) { x.dropped++; return false; }
  }
  uint32_t b = x.b0 + 1u + (uint32_t)((x.dly >> (4u * to)) & 15u);   // slow (socket.go:99-106)
  if (b >= P.D) b -= P.D;
  const uint32_t box = (b * nrep<NT>(P) + to) * P.NS + x.r;
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

// The scripted faults of this replica at this step (socket.go:163-199 Drop /
// Slow / Flaky / Crash windows), in one pass over the table: a crash flag and,
// per destination, drop / flaky bits and the largest Slow delay (4 bits each).
// The table is uniform across the wave; its three loads per fault go out
// together (one round trip per fault, not one per (kind, destination) query).
struct ScriptedStep {
  uint32_t drop, flaky;
  uint64_t slow;
  bool crash;
};
template <int NT>
__device__ __forceinline__ ScriptedStep scripted_scan(const Params& P, const Rep<NT>& x) {
  ScriptedStep o = {0u, 0u, 0ull, false};
  const uint32_t N = nrep<NT>(P);
  for (uint32_t i = 0; i < P.nfaults; i++) {
    const uint4 a = P.faults[i].a;                                // kind, src, dst, param
    const uint4 b = P.faults[i].b;                                // cluster_lo, cluster_hi
    const uint4 c = P.faults[i].c;                                // step_from, step_to
    if (a.y != x.r) continue;
    const uint64_t lo = (uint64_t)b.x | ((uint64_t)b.y << 32), hi = (uint64_t)b.z | ((uint64_t)b.w << 32);
    if (x.gid < lo || x.gid >= hi || x.t < c.x || x.t >= c.y) continue;
    if (a.x == PAXISIM_FAULT_CRASH) {
      o.crash = true;
      continue;
    }
    const uint32_t dst = a.z == PAXISIM_ALL_DST ? ((1u << N) - 1u) : (a.z < N ? 1u << a.z : 0u);
    if (a.x == PAXISIM_FAULT_DROP) o.drop |= dst;
    if (a.x == PAXISIM_FAULT_FLAKY && a.w > 0) o.flaky |= dst;
    if (a.x == PAXISIM_FAULT_SLOW) {
#pragma unroll
      for (uint32_t d = 0; d < Rep<NT>::NL; d++) {
        const uint64_t cur = (o.slow >> (4u * d)) & 15u;
        if (((dst >> d) & 1u) && a.w > cur) o.slow = (o.slow & ~(15ull << (4u * d))) | ((uint64_t)a.w << (4u * d));
      }
    }
  }
  return o;
}

// Per step: fold crash / drop / slow / flaky of every outgoing link into masks
// (the filter order crash -> drop -> flaky -> slow is kept by send_begin).
template <int NT>
__device__ __forceinline__ void link_masks(const Params& P, Rep<NT>& x, const uint32_t (&du)[Rep<NT>::NL],
                                           const uint32_t (&su)[Rep<NT>::NL], const ScriptedStep& sc) {
  const uint32_t N = nrep<NT>(P);
  uint32_t dm = 0;
  uint64_t dl = 0;
#pragma unroll
  for (uint32_t d = 0; d < Rep<NT>::NL; d++) {
    if (d >= N) continue;
    uint32_t delay = 0;
    const bool drop = x.t < du[d] || ((sc.drop >> d) & 1u);
    if (x.t < (su[d] & (T_MAX - 1u))) delay = su[d] >> 28;
    const uint32_t sd = (uint32_t)(sc.slow >> (4u * d)) & 15u;
    if (sd > delay) delay = sd;
    if (delay > P.max_delay) delay = P.max_delay;
    dm |= (drop || x.crashed) ? (1u << d) : 0u;
    dl |= (uint64_t)delay << (4u * d);
  }
  x.dmask = dm;
  x.fmask = sc.flaky;
  x.dly = dl;
}

template <int NT>
__device__ __forceinline__ void send1(const Params& P, Rep<NT>& x, uint32_t to, uint32_t w0, uint32_t w1,
                                      uint32_t w2, uint32_t w3) {
  uint32_t ri;
  if (send_begin<NT>(P, x, to, 1, ri)) {
    PXS_TALLY_AT(P, x.blk, TC_REC_ST, &x.rec[ri], true);
    x.rec[ri] = make_uint4(w0, w1, w2, w3);
  }
}

// Broadcast: every peer except self, IDs.Less order (socket.go:147-155; G1, G2)
template <int NT>
__device__ __forceinline__ void broadcast1(const Params& P, Rep<NT>& x, uint32_t w0, uint32_t w1, uint32_t w2,
                                           uint32_t w3) {
  constexpr uint32_t NU = NT ? (uint32_t)NT : (uint32_t)PAXISIM_MAX_N;
#pragma unroll
  for (uint32_t d = 0; d < NU; d++)
    if (d < nrep<NT>(P) && d != x.r) send1<NT>(P, x, d, w0, w1, w2, w3);
}

// ---------------------------------------------------------------------------
// Send intents.  A handler posts at most one pending send (one record to a set
// of destinations); the merge loop emits it after the dispatch switch, so the
// socket-filter / mailbox code runs once per iteration for all lanes instead of
// once per handler branch.  Posting a second send first emits the pending one,
// and emission walks destinations in index order, so every link sees its
// records in exactly the order the handlers issued them.
// ---------------------------------------------------------------------------
#ifndef PXS_FLUSH1_9
#define PXS_FLUSH1_9 0   // 1: 9-replica WPaxos kernel flushes in one pass (A/B r2: +4% at 153 spilled VGPRs, -3% at 101)
#endif
template <int NT>
__device__ __forceinline__ void intent_flush(const Params& P, Rep<NT>& x) {
  if (!x.im) return;
  constexpr uint32_t NU = NT ? (uint32_t)NT : (uint32_t)PAXISIM_MAX_N;
  if (NT == 9 && PXS_FLUSH1_9 && x.es == 4u) {   // (the HBM-log kernel: A/B r2 +, the LDS-window one -)
#pragma unroll
    for (uint32_t d = 0; d < NU; d++) {
      if (!((x.im >> d) & 1u)) continue;
      const uint32_t seq = x.send_seq++;
      x.sent++;
      if ((x.dmask >> d) & 1u) { x.dropped++; continue; }
      if ((x.fmask >> d) & 1u) {
        uint32_t p = 0;
        scripted(P, PAXISIM_FAULT_FLAKY, x.gid, x.r, d, x.t, &p);
        if (ppm_hit(draw(x.hs, tag(PUR_FLAKY, x.r, seq)), p)) { x.dropped++; continue; }
      }
      uint32_t b = x.b0 + 1u + (uint32_t)((x.dly >> (4u * d)) & 15u);
      if (b >= P.D) b -= P.D;
      const uint32_t box = (b * NU + d) * P.NS + x.r;
      const uint32_t k = x.l_cnt[(box << 6) | x.lane];
      if (k + 1u > P.M) {
        x.flags |= PAXISIM_F_MBOX_OVF | PAXISIM_F_UNFAITHFUL;
        x.dropped++;
        continue;
      }
      x.l_cnt[(box << 6) | x.lane] = (uint8_t)(k + 1u);
      PXS_TALLY_AT(P, x.blk, TC_REC_ST, &x.rec[((box * P.M + k) << 6) | x.lane], true);
      x.rec[((box * P.M + k) << 6) | x.lane] = make_uint4(x.iw0, x.iw1, x.iw2, x.iw3);
    }
    x.im = 0;
    return;
  }
  // pass 1: the bucket count of every destination (independent LDS reads:
  // each destination has its own box, so reading them up front is exact)
  uint32_t box[NU], k[NU];
#pragma unroll
  for (uint32_t d = 0; d < NU; d++) {
    box[d] = 0;
    k[d] = 0;
    if (d < nrep<NT>(P) && ((x.im >> d) & 1u)) {
      uint32_t b = x.b0 + 1u + (uint32_t)((x.dly >> (4u * d)) & 15u);
      if (b >= P.D) b -= P.D;
      box[d] = (b * nrep<NT>(P) + d) * P.NS + x.r;
      k[d] = x.l_cnt[(box[d] << 6) | x.lane];
    }
  }
  // pass 2: the socket filter and the append, destinations in index order
#pragma unroll
  for (uint32_t d = 0; d < NU; d++) {
    if (!(d < nrep<NT>(P) && ((x.im >> d) & 1u))) continue;
    const uint32_t seq = x.send_seq++;
    x.sent++;
    if ((x.dmask >> d) & 1u) { x.dropped++; continue; }
    if ((x.fmask >> d) & 1u) {
      uint32_t p = 0;
      scripted(P, PAXISIM_FAULT_FLAKY, x.gid, x.r, d, x.t, &p);
      if (ppm_hit(draw(x.hs, tag(PUR_FLAKY, x.r, seq)), p)) { x.dropped++; continue; }
    }
    if (k[d] + 1u > P.M) {
      x.flags |= PAXISIM_F_MBOX_OVF | PAXISIM_F_UNFAITHFUL;
      x.dropped++;
      continue;
    }
    x.l_cnt[(box[d] << 6) | x.lane] = (uint8_t)(k[d] + 1u);
    PXS_TALLY_AT(P, x.blk, TC_REC_ST, &x.rec[((box[d] * P.M + k[d]) << 6) | x.lane], true);
    x.rec[((box[d] * P.M + k[d]) << 6) | x.lane] = make_uint4(x.iw0, x.iw1, x.iw2, x.iw3);
  }
  x.im = 0;
}
template <int NT>
__device__ __forceinline__ void post_mask(const Params& P, Rep<NT>& x, uint32_t mask, uint32_t w0, uint32_t w1,
                                          uint32_t w2, uint32_t w3) {
  intent_flush<NT>(P, x);
  x.im = mask;
  x.iw0 = w0; x.iw1 = w1; x.iw2 = w2; x.iw3 = w3;
}
// Send(to, m) (socket.go:66)
template <int NT>
__device__ __forceinline__ void post_unicast(const Params& P, Rep<NT>& x, uint32_t to, uint32_t w0, uint32_t w1,
                                             uint32_t w2, uint32_t w3) {
  if (to >= nrep<NT>(P)) {                // unknown id ("0.0"): counted and dropped in order
    intent_flush<NT>(P, x);
    send1<NT>(P, x, to, w0, w1, w2, w3);
    return;
  }
  post_mask<NT>(P, x, 1u << to, w0, w1, w2, w3);
}
// Broadcast(m) (socket.go:147-155)
template <int NT>
__device__ __forceinline__ void post_broadcast(const Params& P, Rep<NT>& x, uint32_t w0, uint32_t w1, uint32_t w2,
                                               uint32_t w3) {
  post_mask<NT>(P, x, ((1u << nrep<NT>(P)) - 1u) & ~(1u << x.r), w0, w1, w2, w3);
}

// ---------------------------------------------------------------------------
// workload (benchmark.go:202-275): key and read/write of command cid
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t wl_hash(uint32_t kc, uint32_t cid) { return fmix32(fmix32(kc ^ 0x5BD1E995u) ^ cid); }
// With locality (WPaxos per-zone clients, benchmark.go:202-213 "conflict"/Min):
// worker w's command is, with P = locality, one of the keys k = z (mod Z) of
// the zone z of its target replica, otherwise uniform over all keys.
// x % d for d >= 1 given m = floor((2^32-1)/d): the quotient estimate is low by at most one
__device__ __forceinline__ uint32_t mod_magic(uint32_t x, uint32_t d, uint32_t m) {
  uint32_t r = x - d * __umulhi(x, m);
  return r >= d ? r - d : r;
}
// "normal" with Bconfig.Move (benchmark.go:137-140): command cid draws from
// the key CDF of the Mu its issue number falls in, e = (cid-1) / move_every;
// past the last table the Mu sequence repeats from move_loop.  Upper bound by
// binary search: the number of thresholds <= u.
__device__ __forceinline__ uint32_t wl_key_moving(const Params& P, uint32_t u, uint32_t cid) {
  uint32_t e = (cid - 1u) / P.move_every;
  if (e >= P.move_tables) e = P.move_loop + (e - P.move_loop) % (P.move_tables - P.move_loop);
  const uint32_t* t = P.move_cdf + (size_t)e * PAXISIM_MAX_KEYS;
  uint32_t lo = 0, hi = P.keys - 1u;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (t[mid] <= u) lo = mid + 1u;
    else hi = mid;
  }
  return lo;
}
// The key index of command cid given h = wl_hash(kc, cid): in [0, keys), or
// keys for a table draw beyond the key space (the unbounded "exponential"
// tail; key_fit flags it where the key is used).
__device__ __forceinline__ uint32_t wl_key_h(const Params& P, uint32_t h, uint32_t cid) {
  if (P.locality_ppm) {
    const uint32_t w = mod_magic(cid - 1u, P.WK, P.wk_magic);        // (cid-1) % WK
    const uint32_t z = P.wzone[w], nk = P.wnk[w];                    // zone_of[target[w]], its key count
    if (nk && ppm_hit(fmix32(h ^ 0x165667B1u), P.locality_ppm)) return z + P.Z * mod_magic(h, nk, P.wnk_magic[w]);
  }
  switch (P.dist) {   // Bconfig.Distribution (benchmark.go:202-233), DESIGN.md §3.8
    case PAXISIM_DIST_ORDER: return mod_magic(cid, P.kspace, P.kspace_magic);
    case PAXISIM_DIST_CONFLICT:   // Go's literal key 0 (benchmark.go:213-214), else the order counter + Min
      return fmix32(h ^ 0x3C6EF372u) % 100u < P.conflicts ? P.conflict_key : mod_magic(cid, P.kspace, P.kspace_magic);
    case PAXISIM_DIST_TABLE: {   // inverse CDF; the table index is uniform, so these are scalar loads
      const uint32_t u = fmix32(h ^ 0x2545F491u);
      if (P.move_every) return wl_key_moving(P, u, cid);
      if (P.key_tail && u >= P.key_tail) return P.keys;
      uint32_t k = 0;
      for (uint32_t i = 0; i + 1u < P.keys; i++) k += u >= P.key_cdf[i] ? 1u : 0u;
      return k;
    }
    default: return mod_magic(h, P.kspace, P.kspace_magic);
  }
}
__device__ __forceinline__ uint32_t wl_key(const Params& P, uint32_t kc, uint32_t cid) {
  return wl_key_h(P, wl_hash(kc, cid), cid);
}
// A key the replica uses: a draw beyond the key space has no state here (Go's
// key would be a new map entry), so the replica raises UNFAITHFUL and uses the
// last index.
template <int NT>
__device__ __forceinline__ uint32_t key_fit(const Params& P, Rep<NT>& x, uint32_t k) {
  if (k >= P.keys) {
    x.flags |= PAXISIM_F_UNFAITHFUL;
    k = P.keys - 1u;
  }
  return k;
}
// The key value the reference's Database sees for index k (paxisim.h)
__device__ __forceinline__ uint32_t key_value(const Params& P, uint32_t k) {
  if (P.dist == PAXISIM_DIST_TABLE) return k;
  if (P.dist == PAXISIM_DIST_CONFLICT && P.key_min && k == P.conflict_key) return 0u;
  return P.key_min + k;
}
__device__ __forceinline__ bool wl_write_h(const Params& P, uint32_t h) {
  return ppm_hit(fmix32(h ^ 0x27D4EB2Fu), P.write_ppm);
}
__device__ __forceinline__ bool wl_write(const Params& P, uint32_t kc, uint32_t cid) {
  return wl_write_h(P, wl_hash(kc, cid));
}

#ifndef PXS_REPLY_STORE
#define PXS_REPLY_STORE 1   // 0: the worker's last Reply.Value is not kept (A/B attribution only)
#endif
#ifndef PXS_REPLY_DEFER
#define PXS_REPLY_DEFER 1   // the Reply.Value store waits until the end of the merge trip
#endif
// The value usually comes from a load issued just before the reply (Execute's
// previous value, paxos_kernel.h kv_get): storing it at the end of the trip
// lets the handler go on without waiting for that load.
template <int NT>
__device__ __forceinline__ void reply_flush(const Params& P, Rep<NT>& x) {
  if (x.rw) {
    PXS_TALLY_AT(P, x.blk, TC_REPLY, &P.wrep[(size_t)(x.rw - 1u) * P.C + x.c], true);
    P.wrep[(size_t)(x.rw - 1u) * P.C + x.c] = x.rv;
    x.rw = 0;
  }
}
// The HTTP response reaches worker w, which keeps its Reply.Value (the value
// a read returned, benchmark.go:259-262) and issues its next request: it
// arrives at the worker's target (client source N) in the next step.
template <int NT>
__device__ __forceinline__ void client_reply(const Params& P, Rep<NT>& x, uint32_t cid, uint32_t value) {
  uint32_t w = (cid - 1u) - P.WK * __umulhi(cid - 1u, P.wk_magic);   // (cid-1) % WK
  if (w >= P.WK) w -= P.WK;
  const uint32_t wi = (w << 6) | x.lane;
  if (x.l_wcur[wi] != cid) return;              // duplicate reply: the worker moved on
  x.replies++;
  if (PXS_REPLY_STORE && PXS_REPLY_DEFER) {
    reply_flush<NT>(P, x);
    x.rw = w + 1u;
    x.rv = value;
  } else if (PXS_REPLY_STORE) {
    P.wrep[(size_t)w * P.C + x.c] = value;
  }
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
    uint32_t b = x.b0 + 1u;
    if (b >= P.D) b -= P.D;
    const uint32_t box = (b * nrep<NT>(P) + P.target[w]) * P.NS + nrep<NT>(P);
    uint8_t* cp = &x.l_cnt[(box << 6) | x.lane];
    const uint32_t k = *cp;
    if (k >= P.M) {
      x.flags |= PAXISIM_F_MBOX_OVF | PAXISIM_F_UNFAITHFUL;
      return;
    }
    PXS_TALLY_AT(P, x.blk, TC_REC_ST, &x.rec[((box * P.M + k) << 6) | x.lane], true);
    x.rec[((box * P.M + k) << 6) | x.lane] = make_uint4(PAXISIM_MSG_REQUEST, 0u, 0u, (uint32_t)nc);
    *cp = (uint8_t)(k + 1u);
  } else {
    x.l_wcur[wi] = 0;
  }
}

// A worker whose first request is due at this step sends it to its target
// now (paxisim_workload.start_step), behind the requests already queued there.
template <int NT>
__device__ __forceinline__ void client_start(const Params& P, Rep<NT>& x) {
  for (uint32_t m = P.late_workers; m; m &= m - 1u) {   // scalar loop: the mask is uniform
    const uint32_t w = (uint32_t)__builtin_ctz(m);
    if (P.start_step[w] != x.t || P.target[w] != x.r) continue;
    const uint32_t wi = (w << 6) | x.lane;
    x.l_wcur[wi] = 1u + w;
    x.l_wiss[wi] = 1u;
    const uint32_t box = (x.b0 * nrep<NT>(P) + x.r) * P.NS + nrep<NT>(P);
    uint8_t* cp = &x.l_cnt[(box << 6) | x.lane];
    const uint32_t k = *cp;
    if (k >= P.M) {
      x.flags |= PAXISIM_F_MBOX_OVF | PAXISIM_F_UNFAITHFUL;
      continue;
    }
    x.rec[((box * P.M + k) << 6) | x.lane] = make_uint4(PAXISIM_MSG_REQUEST, 0u, 0u, 1u + w);
    *cp = (uint8_t)(k + 1u);
  }
}

// ---------------------------------------------------------------------------
// Random fault process: per idle outgoing link, one draw may open a drop and
// / or a slow window.
// ---------------------------------------------------------------------------
// The link state {drop_until, slow_until | delay << 28} of every outgoing link
// lives in HBM ([dst][N][C], lanes coalesced): loaded once per step, written
// back when a window opens; it is not held in registers across the step.
template <int NT>
__device__ __forceinline__ void fault_process(const Params& P, Rep<NT>& x, uint32_t (&du)[Rep<NT>::NL],
                                              uint32_t (&su)[Rep<NT>::NL]) {
  if (P.drop_ppm == 0 && P.slow_ppm == 0) return;
#pragma unroll
  for (uint32_t d = 0; d < Rep<NT>::NL; d++) {
    if (d >= nrep<NT>(P) || d == x.r) continue;
    const uint32_t u = draw(x.hs, tag(PUR_LINK, x.r, d));
    if (P.drop_ppm && x.t >= du[d] && ppm_hit16(u & 0xFFFFu, P.drop_ppm)) {
      du[d] = x.t + P.drop_len;
      PXS_TALLY_AT(P, x.blk, TC_LINK, &P.link_drop[krc(P, d, x.r, x.c)], true);
      P.link_drop[krc(P, d, x.r, x.c)] = du[d];
    }
    if (P.slow_ppm && x.t >= (su[d] & (T_MAX - 1u)) && ppm_hit16(u >> 16, P.slow_ppm)) {
      const uint32_t span = P.slow_max - P.slow_min + 1u;
      const uint32_t v = draw(x.hs, tag(PUR_SLOWD, x.r, d));
      su[d] = (x.t + P.slow_len) | ((P.slow_min + __umulhi(v, span)) << 28);
      PXS_TALLY_AT(P, x.blk, TC_LINK, &P.link_slow[krc(P, d, x.r, x.c)], true);
      P.link_slow[krc(P, d, x.r, x.c)] = su[d];
    }
  }
}

// Same-trip absorption of send-free P2bs (below) in the 9-replica Paxos
// kernel too; 0 builds it without (A/B of register pressure vs trips).
#ifndef PXS_ABSORB9
#define PXS_ABSORB9 1
#endif
#ifndef PXS_ABSORB_MAX
#define PXS_ABSORB_MAX 2   // messages absorbed per trip (A/B: 2 > 3 > 4 > 6 on config 2)
#endif
#ifndef PXS_ABSORB_ABD
#define PXS_ABSORB_ABD 0
#endif
#ifndef PXS_AGR_SLOT
#define PXS_AGR_SLOT 0    // 1: the Multi-Paxos ring indexed by slot too (round 4; diagnostic A/B only - wrong under compaction)
#endif
#ifndef PXS_WP_ABSORB
#define PXS_WP_ABSORB 0   // WPaxos same-key P2b absorption (wpaxos_kernel.h): 0 off, 1 the r4l experiment, 2 fixed
#endif
#ifndef PXS_FLUSH_LATE
#define PXS_FLUSH_LATE 1
#endif
#ifndef PXS_LINK_LATE
#define PXS_LINK_LATE 1   // the unstaged loop issues its first record load before the link state's (replica_step)
#endif
#ifndef PXS_PREFETCH2
#define PXS_PREFETCH2 0   // 1: unstaged loop loads records two messages ahead (A/B r2l: -13% on config 2, more spills)
#endif

// ---------------------------------------------------------------------------
// One replica, one step
// ---------------------------------------------------------------------------
// Records left per source in the merge.  9-replica kernels pack them into
// bytes (four sources a register: counts are at most M <= 255), which frees
// seven registers across the merge loop; the others keep one a source.
#ifndef PXS_PACKREM9
#define PXS_PACKREM9 1
#endif
template <uint32_t NS, bool PACK>
struct RemT {
  uint32_t v[NS];
  __device__ __forceinline__ void clear() {
#pragma unroll
    for (uint32_t s = 0; s < NS; s++) v[s] = 0;
  }
  __device__ __forceinline__ uint32_t get(uint32_t s) const { return opaque(v[s]); }   // s: a constant
  __device__ __forceinline__ void put(uint32_t s, uint32_t n) { v[s] = n; }           // after clear()
  __device__ __forceinline__ void sub(uint32_t src, uint32_t n) {
#pragma unroll
    for (uint32_t s = 0; s < NS; s++) v[s] = opaque(v[s]) - (s == src ? n : 0u);
  }
};
template <uint32_t NS>
struct RemT<NS, true> {
  static constexpr uint32_t NW = (NS + 3u) / 4u;
  uint32_t w[NW];
  __device__ __forceinline__ void clear() {
#pragma unroll
    for (uint32_t k = 0; k < NW; k++) w[k] = 0;
  }
  __device__ __forceinline__ uint32_t get(uint32_t s) const { return (opaque(w[s >> 2]) >> ((s & 3u) * 8u)) & 0xFFu; }
  __device__ __forceinline__ void put(uint32_t s, uint32_t n) { w[s >> 2] |= n << ((s & 3u) * 8u); }
  __device__ __forceinline__ void sub(uint32_t src, uint32_t n) {   // never borrows: n <= the count
    const uint32_t d = n << ((src & 3u) * 8u);
#pragma unroll
    for (uint32_t k = 0; k < NW; k++) w[k] = opaque(w[k]) - ((src >> 2) == k ? d : 0u);
  }
};

#ifdef PXS_STAMPS
struct Stamps { unsigned long long setup, loop, barrier, trips, msgs, steps, pick, disp, wait, flush, stage, tail; };
#endif

template <int NT, class Proto, bool STAGED>
__device__ __forceinline__ void replica_step(const Params& P, Rep<NT>& x
#ifdef PXS_STAMPS
                                             , void* stp
#endif
) {
#ifdef PXS_STAMPS
  Stamps& st = *reinterpret_cast<Stamps*>(stp);
  const unsigned long long s0 = stamp();
#endif
  constexpr uint32_t NSMAX = NT ? (uint32_t)NT + 1u : (uint32_t)PAXISIM_MAX_N + 1u;
  const uint32_t N = nrep<NT>(P), NS = N + 1u;
  x.send_seq = 0;
  x.stop = false;
  x.im = 0;
  x.rw = 0;
  x.hs = step_key(x.kc, x.t);
  if (P.late_workers) client_start<NT>(P, x);
  const ScriptedStep sc = P.nfaults ? scripted_scan<NT>(P, x) : ScriptedStep{0u, 0u, 0ull, false};
  x.crashed = sc.crash;
  // The random fault process and the step's link masks.  Nothing before the
  // first handler's sends reads them, so the unstaged loop runs this after it
  // has issued its first record load: the link state's HBM round trip then
  // overlaps the record's instead of preceding it (PXS_LINK_LATE).
  auto link_step = [&]() {
    // link state exists only under a random fault process (without one it stays 0)
    const bool random_faults = P.drop_ppm || P.slow_ppm;
    uint32_t du[Rep<NT>::NL], su[Rep<NT>::NL];
#pragma unroll
    for (uint32_t d = 0; d < Rep<NT>::NL; d++) {
      du[d] = d < N && random_faults ? P.link_drop[krc(P, d, x.r, x.c)] : 0u;
      su[d] = d < N && random_faults ? P.link_slow[krc(P, d, x.r, x.c)] : 0u;
#ifdef PXS_TALLY
      if (d < N && random_faults) {
        PXS_TALLY_AT(P, x.blk, TC_LINK, &P.link_drop[krc(P, d, x.r, x.c)], false);
        PXS_TALLY_AT(P, x.blk, TC_LINK, &P.link_slow[krc(P, d, x.r, x.c)], false);
      }
#endif
    }
    fault_process<NT>(P, x, du, su);
    link_masks<NT>(P, x, du, su, sc);
  };
  constexpr bool LINK_LATE = !STAGED && PXS_LINK_LATE;
  if constexpr (!LINK_LATE) link_step();

  const uint32_t box0 = (x.b0 * N + x.r) * NS;          // inbox boxes: box0 + src
  // per source: records left (rem) and the step's initial count, packed in
  // bytes (c0w), so a source's FIFO position is c0 - rem without a register each
  constexpr uint32_t NCW = (NSMAX + 3u) / 4u;
  RemT<NSMAX, NT == 9 && PXS_PACKREM9> rem;
  uint32_t c0w[NCW], total = 0;
  rem.clear();
#pragma unroll
  for (uint32_t k = 0; k < NCW; k++) c0w[k] = 0;
#pragma unroll
  for (uint32_t s = 0; s < NSMAX; s++) {
    if (s < NS) {
      uint32_t n = x.l_cnt[((box0 + s) << 6) | x.lane];
      if (x.crashed && s < N && n) {                    // socket.Recv discards (socket.go:111-118)
        for (uint32_t k = 0; k < n;) {
          PXS_TALLY_AT(P, x.blk, TC_REC_LD, &x.rec[(((box0 + s) * P.M + k) << 6) | x.lane], false);
          const uint32_t h = ldg(&x.rec[(((box0 + s) * P.M + k) << 6) | x.lane]).x;
          x.discarded++;
          k += rec_len(h);
        }
        n = 0;
      }
      rem.put(s, n);
      c0w[s >> 2] |= n << ((s & 3u) * 8u);
      total += n;
    }
  }
  if (P.phase_sort)   // this step's load of the cluster, by step residue (serial kernel)
    reinterpret_cast<uint32_t*>(x.l_cnt + P.ph_rel)[((x.t % P.phase_period) << 6) | x.lane] += total;

  // merge order: weighted pick among sources, two 16-bit picks per draw;
  // the next message's record is loaded before the current one is handled
#ifdef PXS_STAMPS
  const unsigned long long s1 = stamp();
  st.setup += s1 - s0;
  {
    uint32_t tot = total;
    for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o, 64);
    st.msgs += tot;   // records (~messages) over the wave's lanes
  }
#endif
  uint32_t u = 0, i = 0, src = 0, ri = 0;
  uint4 m = make_uint4(0u, 0u, 0u, 0u);
  // pick idx: the source of the idx-th message, given the remaining counts
  auto pick_from = [&](uint32_t idx, uint32_t tot, const decltype(rem)& rm, uint32_t& uu, uint32_t& psrc,
                       uint32_t& pri) {
    if (!(idx & 1u)) uu = draw(x.hs, tag(PUR_ORDER, x.r, idx >> 1));
    uint32_t pk = (((idx & 1u) ? (uu >> 16) : (uu & 0xFFFFu)) * tot) >> 16;
    bool found = false;
    psrc = 0;
    uint32_t p0 = 0;
#pragma unroll
    for (uint32_t s = 0; s < NSMAX; s++) {
      const uint32_t rs = rm.get(s);
      const bool here = !found && pk < rs;
      if (here) { psrc = s; p0 = ((c0w[s >> 2] >> ((s & 3u) * 8u)) & 0xFFu) - rs; found = true; }
      else if (!found) pk -= rs;
    }
    pri = (((box0 + psrc) * P.M + p0) << 6) | x.lane;
  };
  auto pick = [&](uint32_t idx, uint32_t& psrc, uint32_t& pri) { pick_from(idx, total, rem, u, psrc, pri); };

  // Stage the records of the first J picks into LDS before handling any: the
  // merge order is a function of the counts alone while every message is one
  // record, so the picks are known up front and their loads go out together
  // (one global_load_lds per pick, straight to this wave's LDS stage rows)
  // instead of one dependent HBM round trip per message.  A multi-record P1b
  // changes the later picks: staged entries after it are dropped (jv).
  uint32_t jv = 0;
  const uint4* stage = nullptr;
#ifdef PXS_STAMPS
  const unsigned long long g0 = stamp();
  unsigned long long fe = g0;
#endif
  if constexpr (STAGED) {
    const uint32_t sbase = __builtin_amdgcn_readfirstlane(P.off_stage + x.r * P.J * 1024u);
    stage = reinterpret_cast<const uint4*>(x.l_cnt - P.img.off_cnt + sbase) + x.lane;
    auto srem = rem;
    uint32_t su = 0;
    for (uint32_t j = 0; j < P.J; j++) {
      if (!__ballot(j < total)) break;
      if (j < total) {
        uint32_t ssrc, sri;
        pick_from(j, total - j, srem, su, ssrc, sri);
        srem.sub(ssrc, 1u);
        __builtin_amdgcn_global_load_lds(
            (__attribute__((address_space(1))) void*)(x.rec + sri),
            (__attribute__((address_space(3))) void*)((__attribute__((address_space(3))) uint8_t*)(x.l_cnt -
                                                      P.img.off_cnt) + sbase + j * 1024u),
            16, 0, 0);
      }
    }
    jv = total < P.J ? total : P.J;
    // vmcnt(0) (gfx9 encoding: expcnt, lgkmcnt at max) as a builtin, so the
    // compiler's waitcnt pass knows the stage is complete and does not re-wait
    // (behind this step's record stores) before every stage read
    __builtin_amdgcn_s_waitcnt(0x0F70);
  }
#ifdef PXS_STAMPS
  st.stage += stamp() - g0;
#endif
  // PF2 (unstaged loop): records are loaded two messages ahead.  The pick
  // after next assumes the next message is one record; a multi-record P1b
  // invalidates it and it is picked again.  Picks draw statelessly, so a
  // re-pick gives the same answer as the first pick of that index would.
  constexpr bool PF2 = !STAGED && PXS_PREFETCH2;
  auto pick_at = [&](uint32_t idx, uint32_t tot, uint32_t skip, uint32_t& psrc, uint32_t& pri) {
    const uint32_t uu = draw(x.hs, tag(PUR_ORDER, x.r, idx >> 1));
    uint32_t pk = (((idx & 1u) ? (uu >> 16) : (uu & 0xFFFFu)) * tot) >> 16;
    bool found = false;
    psrc = 0;
    uint32_t p0 = 0;
#pragma unroll
    for (uint32_t s = 0; s < NSMAX; s++) {
      const uint32_t rs = rem.get(s) - (s == skip ? 1u : 0u);
      const bool here = !found && pk < rs;
      if (here) { psrc = s; p0 = ((c0w[s >> 2] >> ((s & 3u) * 8u)) & 0xFFu) - rs; found = true; }
      else if (!found) pk -= rs;
    }
    pri = (((box0 + psrc) * P.M + p0) << 6) | x.lane;
  };
  uint32_t nsrc = 0, nri = 0, q2s = 0, q2r = 0;
  uint4 nm = make_uint4(0u, 0u, 0u, 0u), q2 = make_uint4(0u, 0u, 0u, 0u);
  bool nv = false, q2v = false;                       // PF2: next / after-next pick loaded
  if (total) {
    pick(0, src, ri);
    if constexpr (STAGED) {
      if (jv) m = stage[0];
      else m = load_now(x.rec + ri);
    } else {
      PXS_TALLY_AT(P, x.blk, TC_REC_LD, &x.rec[ri], false);
      m = x.rec[ri];
    }
  }
  if constexpr (LINK_LATE) link_step();
  while (total && !x.stop) {
#ifdef PXS_STAMPS
    const unsigned long long w0 = stamp();
#endif
    const uint32_t len = rec_len(m.x);
    rem.sub(src, len);
    total -= len;
    if (len > 1u && jv > i + 1u) jv = i + 1u;          // later picks differ from the staged ones
#ifdef PXS_STAMPS
    const unsigned long long q0 = stamp();
    st.wait += q0 - w0;               // trip head: message decode and FIFO bookkeeping
#endif
    if constexpr (PF2) {
      if (len > 1u) nv = false;                         // picked assuming a one-record message
      if (!nv && total) {
        pick_at(i + 1u, total, NSMAX, nsrc, nri);
        nm = x.rec[nri];
        nv = true;
      }
      q2v = nv && total > 1u;
      if (q2v) {
        pick_at(i + 2u, total - 1u, nsrc, q2s, q2r);
        q2 = x.rec[q2r];
      }
    } else {
      nsrc = 0;
      nri = 0;
      nm = make_uint4(0u, 0u, 0u, 0u);
      if (total) {
        pick(i + 1u, nsrc, nri);
        if constexpr (STAGED) {
          if (i + 1u < jv) nm = stage[(i + 1u) * LANES];  // staged
          else nm = load_now(x.rec + nri);                // past the stage: a blocking load
        } else {
          PXS_TALLY_AT(P, x.blk, TC_REC_LD, &x.rec[nri], false);
          nm = x.rec[nri];                                // no stage: one message ahead from HBM
        }
      }
    }
#ifdef PXS_STAMPS
    const unsigned long long q1 = stamp();
    st.pick += q1 - q0;
#endif
    if (src == N) {
      x.client++;
      Proto::template client_request<NT>(P, x, m.w);
    } else {
      Proto::template dispatch<NT>(P, x, src, m, ri);
    }
#ifdef PXS_STAMPS
    const unsigned long long q2t = stamp();
    st.disp += q2t - q1;
#endif
#if !PXS_FLUSH_LATE
    intent_flush<NT>(P, x);                             // one emit point for all lanes
#endif
    PXS_SUB_T0(pxs_ab0)
    if constexpr ((Proto::kind == PAXISIM_PAXOS && (PXS_ABSORB9 || NT != 9)) ||
                  (Proto::kind == PAXISIM_ABD && PXS_ABSORB_ABD) ||
                  (Proto::kind == PAXISIM_WPAXOS && PXS_WP_ABSORB)) {
      // Next messages whose handling is short and send-free (a P2b that does
      // not complete a quorum: paxos.go:270-297) are handled in this same
      // trip, up to PXS_ABSORB_MAX of them.  Order, counters and state are exactly as
      // with one trip each; the lane needs fewer trips, which shortens the
      // wave's step where it is longest (the leader's bursts of P2bs).
#pragma unroll
      for (int k = 0; k < PXS_ABSORB_MAX; k++) {
        if (!(total && !x.stop && nsrc != N && Proto::template absorb<NT>(P, x, nsrc, nm))) break;
        dv_inc<NT>(x, hdr_type(nm.x));
        rem.sub(nsrc, 1u);
        total -= 1u;
        i++;
        if constexpr (PF2) {                            // the after-next becomes the next
          nm = q2;
          nsrc = q2s;
          nri = q2r;
          nv = q2v;
          q2v = nv && total > 1u;
          if (q2v) {
            pick_at(i + 2u, total - 1u, nsrc, q2s, q2r);
            q2 = x.rec[q2r];
          }
        } else if (total) {
          pick(i + 1u, nsrc, nri);
          if constexpr (STAGED) nm = i + 1u < jv ? stage[(i + 1u) * LANES] : load_now(x.rec + nri);
          else {
            PXS_TALLY_AT(P, x.blk, TC_REC_LD, &x.rec[nri], false);
            nm = x.rec[nri];
          }
        }
      }
    }
    if constexpr (Proto::kind == PAXISIM_PAXOS) { PXS_SUB_T1(pxs_ab0, 12) }
#if PXS_FLUSH_LATE
    // The handler's pending send is emitted after the absorbed messages (they
    // send nothing, so every link still sees its records in handler order):
    // the record loads issued while absorbing then precede this flush's
    // stores, and waiting for them does not wait for the stores (vmcnt
    // retires loads and stores in issue order).
    PXS_SUB_T0(pxs_fl0)
    reply_flush<NT>(P, x);
    intent_flush<NT>(P, x);
    if constexpr (Proto::kind == PAXISIM_PAXOS) { PXS_SUB_T1(pxs_fl0, 13) }
#endif
#ifdef PXS_STAMPS
    fe = stamp();
    st.flush += fe - q2t;
#endif
#ifdef PXS_STAMPS
    st.trips += 1;
#endif
    src = nsrc;
    ri = nri;
    m = nm;
    if constexpr (PF2) {
      nm = q2;
      nsrc = q2s;
      nri = q2r;
      nv = q2v;
    }
    i++;
  }
  reply_flush<NT>(P, x);
#pragma unroll
  for (uint32_t s = 0; s < NSMAX; s++)
    if (s < NS) x.l_cnt[((box0 + s) << 6) | x.lane] = 0;
  if (x.stop) atomicMin(&x.l_poison[x.lane], x.t);
#ifdef PXS_STAMPS
  {
    const unsigned long long e = stamp();
    st.loop += e - s1;
    st.tail += e - fe;
  }
#endif
}

// ---------------------------------------------------------------------------
// Agreement ring (client.go:279-320 Consensus, restated as a running check,
// DESIGN.md §3.9): every CKI executed slots a replica reaches digest
// checkpoint k; the first replica to reach it records its digest in the
// cluster's ring, every later one compares.  Arrivals are applied in a fixed
// order, so the coverage counters do not depend on which wave runs first:
// during a step each replica appends its arrivals to its own list (agree_post),
// and after the step's barrier one wave applies every replica's list in
// replica index order (agree_drain) - the order in which the oracle, which runs
// the replicas of a step one after another, applies them.  Lists alternate by
// step parity, so the next step's arrivals never meet the drain.  A replica
// that reaches more than AGMAX checkpoints in one step counts the extra ones
// as missed (both backends).
// ---------------------------------------------------------------------------
template <int NT>
__device__ __forceinline__ void agree_post(const Params& P, Rep<NT>& x, uint32_t k) {
  const uint32_t par = x.t & 1u;
  uint8_t* cp = &x.l_agn[((par * nrep<NT>(P) + x.r) << 6) | x.lane];
  const uint32_t n = *cp;
  if (n < AGMAX) {
    const uint64_t d = x.digest;
    const uint64_t want = ((uint64_t)k << 40) | ((d ^ (d >> 24)) & 0xFFFFFFFFFFull);
    PXS_TALLY_AT(P, x.blk, TC_AGREE, &P.agq[(((size_t)par * AGMAX + n) * nrep<NT>(P) + x.r) * P.C + x.c], true);
    P.agq[(((size_t)par * AGMAX + n) * nrep<NT>(P) + x.r) * P.C + x.c] =
        make_uint4((uint32_t)want, (uint32_t)(want >> 32), x.key, 0u);
  }
  if (n < 255u) *cp = (uint8_t)(n + 1u);
}
template <int NT, class Proto>
__device__ __forceinline__ void agree_drain(const Params& P, const Rep<NT>& x, uint32_t par) {
  const uint32_t N = nrep<NT>(P);
  for (uint32_t r = 0; r < N; r++) {
    uint8_t* cp = &x.l_agn[((par * N + r) << 6) | x.lane];
    const uint32_t n = *cp;
    if (!n) continue;
    *cp = 0;
    uint32_t cmp = 0, miss = n > AGMAX ? n - AGMAX : 0u, bad = 0;
    for (uint32_t j = 0; j < n && j < AGMAX; j++) {
      PXS_TALLY_AT(P, x.blk, TC_AGREE, &P.agq[(((size_t)par * AGMAX + j) * N + r) * P.C + x.c], false);
      const uint4 e = P.agq[(((size_t)par * AGMAX + j) * N + r) * P.C + x.c];
      const unsigned long long want = (unsigned long long)e.x | ((unsigned long long)e.y << 32);
      const uint32_t k = e.y >> 8;
      // indexed by the cluster, not its slot: compaction does not move the ring
      // (paxisim.hip swap_slots).  Only Multi-Paxos compacts; elsewhere slot ==
      // cluster and the slot index is used as before
      const uint64_t cl = Proto::kind == PAXISIM_PAXOS && !PXS_AGR_SLOT ? x.gid - P.cluster_base : x.c;
      unsigned long long* a = &P.agr[((size_t)(k % P.AR) * P.NK + e.z) * P.C + cl];
      PXS_TALLY_AT(P, x.blk, TC_AGREE, a, false);
      const unsigned long long v = *a;
      const uint32_t tv = (uint32_t)(v >> 40);
      if (v == 0ull || tv < k) {
        *a = want;                                       // first to arrive (or an older checkpoint left): record
      } else if (tv > k) {
        miss++;                                          // the first digest has left the ring
      } else {
        cmp++;
        bad += v != want;
      }
    }
    if (cmp) P.stats[krc(P, ST_AGC, r, x.c)] += cmp;
    if (miss) P.stats[krc(P, ST_AGM, r, x.c)] += miss;
    if (bad) P.stats[krc(P, ST_AGB, r, x.c)] += bad;
  }
}

// ---------------------------------------------------------------------------
// The step kernel: stage the LDS image, run S steps, write everything back.
// ---------------------------------------------------------------------------
// Waves per SIMD the register allocator must allow.  The dispatcher places a
// workgroup of n waves only where every SIMD has ceil(n/4) free wave slots
// (measured: tools/probe/vgpr_probe.hip), so a 5- or 9-wave workgroup of
// cluster groups needs 3 slots per SIMD -> at most 168 VGPRs.
#ifdef PXS_MIN_WAVES
template <int NT> constexpr int min_waves() { return PXS_MIN_WAVES; }
#else
template <int NT> constexpr int min_waves() { return NT == 0 ? 4 : 3; }
#endif

// Instances that carry the LDS-staged merge loop.  Staging only pays where a
// workgroup runs alone on its CU and has LDS to spare (9 replicas, ABD's 3/5);
// elsewhere the second copy of the loop costs registers the packed cluster
// groups need.  StepOps::staged exports it (step_ops.h); paxisim.hip sets J = 0 without it.
#ifndef PXS_STAGE5
#define PXS_STAGE5 0   // 1: the 5-replica Paxos instance carries the staged loop too (A/B)
#endif
template <int NT, class Proto> constexpr bool stage_built() {
  return Proto::kind == PAXISIM_ABD ? NT != 0 : (NT == 9 || (PXS_STAGE5 && NT == 5 && Proto::kind == PAXISIM_PAXOS));
}

// The largest workgroup: as many N-wave cluster groups as min_waves slots per
// SIMD hold.  One workgroup = P.G cluster groups of N waves; group g of
// workgroup b is the 64-cluster tile b*G + g with its own LDS region of
// P.lds_bytes.
template <int NT> constexpr int max_threads() {
  return NT == 0 ? 1024 : ((4 * min_waves<NT>()) / NT > 0 ? (4 * min_waves<NT>()) / NT : 1) * NT * 64;
}
template <int NT, class Proto>
__global__ void __launch_bounds__(max_threads<NT>(), min_waves<NT>()) sim_steps(Params P, uint32_t t0, uint32_t nsteps) {
  extern __shared__ uint4 lds[];
  // slots [bound, C) hold frozen clusters: a workgroup wholly
  // beyond the bound has nothing to do
  const uint32_t bound = __builtin_amdgcn_readfirstlane(*P.bound);
  if ((uint64_t)blockIdx.x * P.G * LANES >= bound) return;
  const uint32_t N = nrep<NT>(P);
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: keeps replica/tile state in SGPRs
  const uint32_t grp = wave / N;
  const uint32_t blk = blockIdx.x * P.G + grp;
  {
    const uint32_t nb = P.img.bytes / 16u;
    const uint4* g = reinterpret_cast<const uint4*>(P.image + (size_t)blockIdx.x * P.G * P.img.bytes);
    for (uint32_t k = threadIdx.x; k < P.G * nb; k += blockDim.x) {
      const uint32_t gg = k / nb;
      lds[gg * (P.lds_bytes / 16u) + (k - gg * nb)] = g[k];
    }
  }
  uint8_t* L = reinterpret_cast<uint8_t*>(lds) + grp * P.lds_bytes;
  Rep<NT> x;
  x.lane = threadIdx.x & 63u;
  // replica played by this wave, rotated per tile: the busiest replica (the
  // leader) then sits on a different wave -> SIMD in neighbouring tiles
  x.r = (wave - grp * N) + blk % N;
  if (x.r >= N) x.r -= N;
  x.blk = blk;
  x.c = (uint64_t)blk * LANES + x.lane;
  x.gid = P.cluster_base + P.cl_of[x.c];
  x.l_a = reinterpret_cast<uint32_t*>(L + P.img.off_a);
  x.l_b = reinterpret_cast<uint32_t*>(L + P.img.off_b);
  x.l_c = reinterpret_cast<uint32_t*>(L + P.img.off_c);
  x.l_wcur = reinterpret_cast<uint32_t*>(L + P.img.off_wcur);
  x.l_wiss = reinterpret_cast<uint32_t*>(L + P.img.off_wiss);
  x.l_poison = reinterpret_cast<uint32_t*>(L + P.img.off_poison);
  x.l_cnt = L + P.img.off_cnt;
  x.l_agn = L + P.off_agn;
  x.rec = P.rec + (size_t)blk * P.rec_per_block;
  if (P.AR)   // this launch's arrival counts (drained every step, so they start empty)
    for (uint32_t k = (wave - grp * N) * LANES + x.lane; k < 2u * N * LANES; k += N * LANES) x.l_agn[k] = 0;
  const bool live = x.c < bound && x.r < N;
  // the log layout is a constant of the instance (paxos_kernel.h: hbm_log)
  x.es = Proto::kind == PAXISIM_WPAXOS ? 4u : LANES;
  x.hw = Proto::kind == PAXISIM_WPAXOS;
  x.ci = ~0u;
  if (live) {
    const size_t i = rc(P, x.r, x.c);
    x.kc = P.kc[x.c];
    x.flags = P.flags[i];
    x.kvver = P.kv ? P.kv_ver[i] : 0u;
    Proto::template load<NT>(P, x);
  }
#pragma unroll
  for (uint32_t k = 0; k < PAXISIM_NMSG / 2; k++) x.dvp[k] = 0;
  x.client = x.sent = x.dropped = x.discarded = x.commits = x.replies = 0;
  __syncthreads();

  uint32_t b0 = t0 % P.D;
#ifdef PXS_STAMPS
  Stamps st = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long t_begin;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_begin)::"memory");
#endif
  for (uint32_t t = t0; t < t0 + nsteps; t++) {
    if (live && x.l_poison[x.lane] >= t) {
      x.t = t;
      x.b0 = b0;
#ifdef PXS_STAMPS
      if (stage_built<NT, Proto>() && P.J) replica_step<NT, Proto, stage_built<NT, Proto>()>(P, x, &st);
      else replica_step<NT, Proto, false>(P, x, &st);
#else
      if (stage_built<NT, Proto>() && P.J)
        replica_step<NT, Proto, stage_built<NT, Proto>()>(P, x);   // records staged into LDS per step
      else
        replica_step<NT, Proto, false>(P, x);                     // one message ahead from HBM
#endif
    }
    if (++b0 == P.D) b0 = 0;
#ifdef PXS_STAMPS
    const unsigned long long sb = stamp();
#endif
    __syncthreads();
#ifdef PXS_STAMPS
    st.barrier += stamp() - sb;
    st.steps++;
#endif
    if (P.AR && live && x.r == N - 1u) agree_drain<NT, Proto>(P, x, t & 1u);   // this step's arrivals, replica order
  }
#ifdef PXS_STAMPS
  if (x.lane == 0 && P.dbg) {
    unsigned long long* d = &P.dbg[((size_t)blk * 16 + x.r) * DBG_PER];
    atomicAdd(&d[0], st.setup); atomicAdd(&d[1], st.loop); atomicAdd(&d[2], st.barrier);
    atomicAdd(&d[3], st.trips); atomicAdd(&d[4], st.msgs); atomicAdd(&d[5], st.steps);
    atomicAdd(&d[6], st.pick); atomicAdd(&d[7], st.disp);
    atomicAdd(&d[8], st.wait); atomicAdd(&d[9], st.flush);
    atomicAdd(&d[10], st.stage); atomicAdd(&d[11], st.tail);
    unsigned long long t_end;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_end)::"memory");
    d[12] = t_begin;                                        // residency: 100 MHz wall clock
    d[13] = t_end;
    d[14] = __builtin_amdgcn_s_getreg((4) | (0 << 6) | ((32 - 1) << 11));   // HW_ID
    d[15] = __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((32 - 1) << 11));  // XCC_ID (gfx940+)
  }
#endif

  // a cluster whose mailboxes are all empty after the launch is at a fixed
  // point: nothing in it changes until a request is injected (compaction)
  if (P.compact && live && x.r == 0) {
    uint32_t any = 0;
    const uint32_t nbox = P.D * N * (N + 1u);
    for (uint32_t b = 0; b < nbox; b++) any |= x.l_cnt[(b << 6) | x.lane];
    P.qf[x.c] = any ? 0u : 1u;
  }
  {
    const uint32_t nb = P.img.bytes / 16u;
    uint4* g = reinterpret_cast<uint4*>(P.image + (size_t)blockIdx.x * P.G * P.img.bytes);
    for (uint32_t k = threadIdx.x; k < P.G * nb; k += blockDim.x) {
      const uint32_t gg = k / nb;
      g[k] = lds[gg * (P.lds_bytes / 16u) + (k - gg * nb)];
    }
  }
  if (live) {
    const uint32_t r = x.r;
    const uint64_t c = x.c;
    P.flags[rc(P, r, c)] = x.flags;
    if (P.kv) P.kv_ver[rc(P, r, c)] = x.kvver;
    Proto::template store<NT>(P, x);
#pragma unroll
    for (uint32_t k = 1; k < PAXISIM_NMSG; k++)
      if (dv_get(x, k)) P.stats[krc(P, ST_DELIV0 + k, r, c)] += dv_get(x, k);
    P.stats[krc(P, ST_CLIENT, r, c)] += x.client;
    P.stats[krc(P, ST_SENT, r, c)] += x.sent;
    P.stats[krc(P, ST_DROPPED, r, c)] += x.dropped;
    P.stats[krc(P, ST_DISCARDED, r, c)] += x.discarded;
    P.stats[krc(P, ST_COMMITS, r, c)] += x.commits;
    P.stats[krc(P, ST_REPLIES, r, c)] += x.replies;
  }
}

// ---------------------------------------------------------------------------
// The serial step kernel: one wave per 64-cluster tile plays
// every replica of its clusters in turn, replica 0 to N-1, each step.  A
// replica's sends land in buckets of later steps only (§3.3), so running the
// replicas of a step one after another is the same step as running them side
// by side - it is how the oracle runs them.  No wave waits at a step barrier
// for the tile's busiest replica, and a wave needs only the mailbox counts and
// client tables in LDS (the log windows and the other image regions stay in
// the HBM image), so many more tiles are resident per CU.  The replica's
// registers are loaded from and stored to HBM around each replica-step.
// ---------------------------------------------------------------------------
// PXS_WB_ACK: with the three planes in HBM (the serial Multi-Paxos kernel) the
// ack word a P2b writes is held back in (ci, ce.z) and stored after the next
// trip's entry loads have issued, so their waits do not include it (vmcnt
// retires loads and stores in issue order).  Every reader of plane c goes
// through ec(), a direct write of index ci drops the pending one, and each
// replica-step ends with wb_flush (paxos_kernel.h set_c / eput).
#ifndef PXS_WB_ACK
#define PXS_WB_ACK 0
#endif
template <int NT>
__device__ __forceinline__ bool wb_on(const Rep<NT>& x) { return PXS_WB_ACK && x.hw && x.es != 4u; }
template <int NT>
__device__ __forceinline__ void wb_flush(Rep<NT>& x) {
  if (wb_on(x) && x.ci != ~0u) {
    x.l_c[x.ci] = x.ce.z;
    x.ci = ~0u;
  }
}
// Replica order per lane (PXS_BUSY_FIRST).  The replica-steps of one step are
// independent - every send lands in a later step's bucket - so each lane may
// run its cluster's replicas in any order.  A wave's replica-step lasts as long
// as its busiest lane's; with every lane taking its replicas busiest first
// (inbox records, ties to the lower index), the k-th replica-step of the wave
// meets the k-th busiest replica of every cluster, and a WPaxos wave no longer
// waits at each of its nine replica-steps for whichever lane holds that
// replica's leader burst (tools/imbalance.py: config 5 cost 3.24 -> 1.84x the
// mean lane; A/B r4h/r4i: config 5 +32%, config 3 +8%).  Returns the order as
// nibbles, first replica lowest.
#ifndef PXS_BUSY_FIRST
#define PXS_BUSY_FIRST 1
#endif
#ifndef PXS_BUSY_FIRST_ALL
#define PXS_BUSY_FIRST_ALL 0   // 1: every protocol (A/B r4i: Paxos -2% on config 2, -4% on config 4); default: WPaxos and ABD
#endif
template <int NT, class Proto> constexpr bool busy_first() {
  return PXS_BUSY_FIRST && (PXS_BUSY_FIRST_ALL || Proto::kind == PAXISIM_WPAXOS || Proto::kind == PAXISIM_ABD);
}
template <int NT>
__device__ __forceinline__ uint64_t replica_order(const Params& P, const Rep<NT>& x, uint32_t b0) {
  constexpr uint32_t NMAX = NT ? (uint32_t)NT : (uint32_t)PAXISIM_MAX_N;
  const uint32_t N = nrep<NT>(P), NS = N + 1u;
  uint32_t key[NMAX];
#pragma unroll
  for (uint32_t r = 0; r < NMAX; r++) {
    uint32_t n = 0;
    if (r < N) {
      const uint32_t box0 = (b0 * N + r) * NS;
      for (uint32_t s = 0; s < NS; s++) n += x.l_cnt[((box0 + s) << 6) | x.lane];
    }
    key[r] = r < N ? (n << 4) | (15u - r) : 0u;   // distinct; more records first, then the lower index
  }
  uint64_t order = 0;
#pragma unroll
  for (uint32_t r = 0; r < NMAX; r++) {
    uint32_t rank = 0;
#pragma unroll
    for (uint32_t q = 0; q < NMAX; q++) rank += key[q] > key[r] ? 1u : 0u;
    if (r < N) order |= (uint64_t)r << (4u * rank);
  }
  return order;
}

#ifndef PXS_PHASE_RECENT
#define PXS_PHASE_RECENT 0   // 1: the residue counts cover the launch's second half only (fresher phase)
#endif
#ifndef PXS_PHASE_HYST
#define PXS_PHASE_HYST 0   // percent a new residue must lead the current one by (phase binning)
#endif
#ifndef PXS_SERIAL_WAVES
#define PXS_SERIAL_WAVES 2   // waves per SIMD the register budget must allow (2: <= 256 VGPRs; A/B r3: 3 waves at 168 VGPRs spill 127 and run 10-24% slower)
#endif
template <int NT>
__device__ __forceinline__ void rep_counters_zero(Rep<NT>& x) {
#pragma unroll
  for (uint32_t k = 0; k < PAXISIM_NMSG / 2; k++) x.dvp[k] = 0;
  x.client = x.sent = x.dropped = x.discarded = x.commits = x.replies = 0;
}
// PXS_COUNTER_ATOMIC: the per-replica-step counts go out as fire-and-forget
// atomic adds (no load to wait for) instead of read-modify-writes
#ifndef PXS_COUNTER_ATOMIC
#define PXS_COUNTER_ATOMIC 1   // (A/B r3, config 2: +4.9%)
#endif
#ifdef PXS_TALLY
#define stat_add(p, v) (PXS_TALLY_AT(P, x.blk, TC_CNT, (p), true), stat_add_((p), (v)))
#endif
__device__ __forceinline__ void stat_add_(uint32_t* p, uint32_t v) {
  if (PXS_COUNTER_ATOMIC) __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p += v;
}
#ifndef PXS_TALLY
#define stat_add stat_add_
#endif
template <int NT>
__device__ __forceinline__ void rep_counters_flush(const Params& P, const Rep<NT>& x) {
  const uint32_t r = x.r;
  const uint64_t c = x.c;
#pragma unroll
  for (uint32_t k = 1; k < PAXISIM_NMSG; k++)
    if (dv_get(x, k)) stat_add(&P.stats[krc(P, ST_DELIV0 + k, r, c)], dv_get(x, k));
  if (x.client) stat_add(&P.stats[krc(P, ST_CLIENT, r, c)], x.client);
  if (x.sent) stat_add(&P.stats[krc(P, ST_SENT, r, c)], x.sent);
  if (x.dropped) stat_add(&P.stats[krc(P, ST_DROPPED, r, c)], x.dropped);
  if (x.discarded) stat_add(&P.stats[krc(P, ST_DISCARDED, r, c)], x.discarded);
  if (x.commits) stat_add(&P.stats[krc(P, ST_COMMITS, r, c)], x.commits);
  if (x.replies) stat_add(&P.stats[krc(P, ST_REPLIES, r, c)], x.replies);
}

// ---------------------------------------------------------------------------
// Lane-asynchronous replica progress (PXS_LANE_ASYNC).  The
// serial kernel's replica-steps of one step are independent (sends land in
// later steps' buckets), so a lane need not wait at each replica-step for the
// wave's busiest lane: here every lane walks its own cluster's replicas
// (busiest first) and starts the next one as soon as its inbox is drained.
// A trip handles one message for every lane that has one; starting a
// replica-step (its registers and inbox counts) and finishing one (write-back,
// counters) run in divergent branches of the same loop, and starts are batched
// - taken when PXS_ASYNC_BATCH lanes wait or no lane has a message left - so
// the wave does not pay a start for every lane that finishes.  Semantics are
// the replica-step's exactly (replica_step's unstaged path, no absorption).
// ---------------------------------------------------------------------------
#ifndef PXS_LANE_ASYNC
#define PXS_LANE_ASYNC 0
#endif
#ifndef PXS_ASYNC_BATCH
#define PXS_ASYNC_BATCH 16
#endif
template <int NT, class Proto>
__device__ __forceinline__ void step_async(const Params& P, Rep<NT>& x, uint64_t order, bool run, uint8_t* img,
                                           uint8_t* scr) {
  constexpr uint32_t NSMAX = NT ? (uint32_t)NT + 1u : (uint32_t)PAXISIM_MAX_N + 1u;
  constexpr uint32_t NCW = (NSMAX + 3u) / 4u;
  const uint32_t N = nrep<NT>(P), NS = N + 1u;
  uint32_t k = run ? 0u : N;            // replica-steps started
  bool act = false;                     // a replica-step in progress
  size_t ri0 = 0;                       // rc() of the current replica
  uint32_t box0 = 0, total = 0, u = 0, i = 0, src = 0, ri = 0;
  uint4 m = make_uint4(0u, 0u, 0u, 0u);
  RemT<NSMAX, NT == 9 && PXS_PACKREM9> rem;
  uint32_t c0w[NCW];
  rem.clear();
#pragma unroll
  for (uint32_t q = 0; q < NCW; q++) c0w[q] = 0;
  auto pick = [&](uint32_t idx, uint32_t& psrc, uint32_t& pri) {
    if (!(idx & 1u)) u = draw(x.hs, tag(PUR_ORDER, x.r, idx >> 1));
    uint32_t pk = (((idx & 1u) ? (u >> 16) : (u & 0xFFFFu)) * total) >> 16;
    bool found = false;
    psrc = 0;
    uint32_t p0 = 0;
#pragma unroll
    for (uint32_t s = 0; s < NSMAX; s++) {
      const uint32_t rs = rem.get(s);
      const bool here = !found && pk < rs;
      if (here) { psrc = s; p0 = ((c0w[s >> 2] >> ((s & 3u) * 8u)) & 0xFFu) - rs; found = true; }
      else if (!found) pk -= rs;
    }
    pri = (((box0 + psrc) * P.M + p0) << 6) | x.lane;
  };
  // Outer loop: finish the lanes whose replica-step is drained, start the next
  // one of every lane that has one left; inner loop: merge trips as in
  // replica_step, until no lane has a message or PXS_ASYNC_BATCH lanes wait.
  for (;;) {
    if (act && (total == 0u || x.stop)) {          // replica_step's tail and the serial kernel's write-back
      act = false;
      reply_flush<NT>(P, x);
#pragma unroll
      for (uint32_t s = 0; s < NSMAX; s++)
        if (s < NS) x.l_cnt[((box0 + s) << 6) | x.lane] = 0;
      if (x.stop) atomicMin(&x.l_poison[x.lane], x.t);
      wb_flush<NT>(x);
      P.flags[ri0] = x.flags;
      if (P.kv) P.kv_ver[ri0] = x.kvver;
      Proto::template store<NT>(P, x);
      if constexpr (Proto::step_scratch) Proto::template step_end<NT>(P, x);
      rep_counters_flush<NT>(P, x);
    }
    if (!act && k < N) {                              // the lane's next replica, busiest first
      const uint32_t r = (uint32_t)(order >> (4u * k)) & 15u;
      k++;
      act = true;
      x.r = r;
      x.ci = ~0u;
      x.l_a = reinterpret_cast<uint32_t*>(img + P.img.off_a);
      x.l_b = reinterpret_cast<uint32_t*>(img + P.img.off_b);
      x.l_c = reinterpret_cast<uint32_t*>(img + P.img.off_c);
      ri0 = rc(P, r, x.c);
      x.flags = P.flags[ri0];
      x.kvver = P.kv ? P.kv_ver[ri0] : 0u;
      Proto::template load<NT>(P, x);
      if constexpr (Proto::step_scratch) Proto::template step_begin<NT>(P, x, scr);
      rep_counters_zero<NT>(x);
      // replica_step's set-up (unstaged path)
      x.send_seq = 0;
      x.stop = false;
      x.im = 0;
      x.rw = 0;
      x.hs = step_key(x.kc, x.t);
      if (P.late_workers) client_start<NT>(P, x);
      const ScriptedStep sc = P.nfaults ? scripted_scan<NT>(P, x) : ScriptedStep{0u, 0u, 0ull, false};
      x.crashed = sc.crash;
      box0 = (x.b0 * N + r) * NS;
      rem.clear();
#pragma unroll
      for (uint32_t q = 0; q < NCW; q++) c0w[q] = 0;
      total = 0;
#pragma unroll
      for (uint32_t s = 0; s < NSMAX; s++) {
        if (s < NS) {
          uint32_t n = x.l_cnt[((box0 + s) << 6) | x.lane];
          if (x.crashed && s < N && n) {                    // socket.Recv discards (socket.go:111-118)
            for (uint32_t q = 0; q < n;) {
              const uint32_t h = ldg(&x.rec[(((box0 + s) * P.M + q) << 6) | x.lane]).x;
              x.discarded++;
              q += rec_len(h);
            }
            n = 0;
          }
          rem.put(s, n);
          c0w[s >> 2] |= n << ((s & 3u) * 8u);
          total += n;
        }
      }
      i = 0;
      if (total) {
        pick(0, src, ri);
        m = x.rec[ri];
      }
      {   // the link state after the first record load (PXS_LINK_LATE)
        const bool random_faults = P.drop_ppm || P.slow_ppm;
        uint32_t du[Rep<NT>::NL], su[Rep<NT>::NL];
#pragma unroll
        for (uint32_t d = 0; d < Rep<NT>::NL; d++) {
          du[d] = d < N && random_faults ? P.link_drop[krc(P, d, x.r, x.c)] : 0u;
          su[d] = d < N && random_faults ? P.link_slow[krc(P, d, x.r, x.c)] : 0u;
        }
        fault_process<NT>(P, x, du, su);
        link_masks<NT>(P, x, du, su, sc);
      }
    }
    if (!__ballot(act)) break;
    // merge trips; a lane whose inbox is drained waits here until the batch ends
    for (;;) {
      const bool busy = act && total != 0u && !x.stop;
      const uint64_t bb = __ballot(busy);
      if (!bb || __popcll(__ballot(!busy && (act || k < N))) >= PXS_ASYNC_BATCH) break;
      if (busy) {
        const uint32_t len = rec_len(m.x);
        rem.sub(src, len);
        total -= len;
        uint32_t nsrc = 0, nri = 0;
        uint4 nm = make_uint4(0u, 0u, 0u, 0u);
        if (total) {
          pick(i + 1u, nsrc, nri);
          nm = x.rec[nri];
        }
        if (src == N) {
          x.client++;
          Proto::template client_request<NT>(P, x, m.w);
        } else {
          Proto::template dispatch<NT>(P, x, src, m, ri);
        }
        reply_flush<NT>(P, x);
        intent_flush<NT>(P, x);
        src = nsrc;
        ri = nri;
        m = nm;
        i++;
      }
    }
  }
}
template <int NT, class Proto> constexpr bool lane_async() {
  // the busiest-first protocols without same-trip absorption (the merge loop above has none)
  return PXS_LANE_ASYNC && Proto::kind == PAXISIM_WPAXOS && !PXS_WP_ABSORB;
}

#ifndef PXS_SERIAL_WAVES_ABD
#define PXS_SERIAL_WAVES_ABD 3   // ABD's kernels fit 168 VGPRs without spilling
#endif
template <class Proto> constexpr int serial_waves() {
  return Proto::kind == PAXISIM_ABD ? PXS_SERIAL_WAVES_ABD : PXS_SERIAL_WAVES;
}
// One tile (64 clusters, one wave) through steps [t0, t0 + nsteps): the body of
// both serial kernels below.
// Idle replica-steps.  A replica whose inbox is empty at a
// step changes nothing - Paxi has no timers (paxos/paxos.go), and with no
// message there is no handler, send or Execute - unless the step itself has
// work: a random fault process advancing its links, or a late worker whose
// first request starts at this replica now (client_start).  Otherwise the
// serial kernel skips such a lane's replica-step whole: no register rows
// loaded or stored, no counters.  PXS_ROW_DIRTY: the per-replica rows (flags,
// database version) are written back only when they changed.  Both are on for
// ABD only: mirrored A/Bs (gpurun_out/r6g2) give ABD (config 3) +4.4%, but
// Multi-Paxos (config 2, where the random fault process leaves no replica-step
// idle) -2% and WPaxos (config 5: 0.4% of replica-steps idle) -8%; the saved
// values and the inbox test cost those kernels registers.  The skip alone is
// on in the 9-replica Multi-Paxos unit (PXS_SKIP_IDLE_PAXOS, __graft_entry__
// TU_FLAGS): config 4 has no random fault process and 41% of its wave-level
// replica-steps are idle (phase-aligned followers), +6.3% (gpurun_out/r6o;
// with the dirty rows too only +2.6%).
#ifndef PXS_SKIP_IDLE
#define PXS_SKIP_IDLE 1
#endif
#ifndef PXS_ROW_DIRTY
#define PXS_ROW_DIRTY 1
#endif
#ifndef PXS_SKIP_IDLE_PAXOS
#define PXS_SKIP_IDLE_PAXOS 0
#endif
#ifndef PXS_ROW_DIRTY_PAXOS
#define PXS_ROW_DIRTY_PAXOS 0
#endif
template <class Proto> constexpr bool skip_idle_on() {
  return PXS_SKIP_IDLE && (Proto::kind == PAXISIM_ABD || (PXS_SKIP_IDLE_PAXOS && Proto::kind == PAXISIM_PAXOS));
}
template <class Proto> constexpr bool row_dirty_on() {
  return PXS_ROW_DIRTY && (Proto::kind == PAXISIM_ABD || (PXS_ROW_DIRTY_PAXOS && Proto::kind == PAXISIM_PAXOS));
}
template <int NT>
__device__ __forceinline__ bool inbox_any(const Rep<NT>& x, uint32_t r, uint32_t b0, uint32_t N) {
  const uint32_t box0 = (b0 * N + r) * (N + 1u);
  uint32_t any = 0;
  for (uint32_t s = 0; s <= N; s++) any |= x.l_cnt[((box0 + s) << 6) | x.lane];
  return any != 0u;
}
template <int NT>
__device__ __forceinline__ bool late_start(const Params& P, uint32_t t, uint32_t r) {
  for (uint32_t m = P.late_workers; m; m &= m - 1u) {
    const uint32_t w = (uint32_t)__builtin_ctz(m);
    if (P.start_step[w] == t && P.target[w] == r) return true;
  }
  return false;
}

template <int NT, class Proto>
__device__ __forceinline__ void serial_tile(const Params& P, uint32_t blk, uint32_t bound, uint32_t t0, uint32_t nsteps,
                                            uint4* lds) {
#ifdef PXS_WAVE_TIMES
  const uint64_t wt0 = __builtin_amdgcn_s_memrealtime();   // 100 MHz, the same clock on every CU
#endif
  const uint32_t N = nrep<NT>(P);
  uint8_t* img = P.image + (size_t)blk * P.img.bytes;
  // LDS holds the image tail [tail, bytes) - from the client tables on, or
  // (P.lds_tail = off_poison) from the poison steps on - then the arrival counts
  const uint32_t tail = P.lds_tail;
  {
    const uint32_t nb = (P.img.bytes - tail) / 16u;
    const uint4* g = reinterpret_cast<const uint4*>(img + tail);
    for (uint32_t k = threadIdx.x; k < nb; k += LANES) lds[k] = g[k];
  }
  uint8_t* L = reinterpret_cast<uint8_t*>(lds);
  Rep<NT> x;
  x.lane = threadIdx.x;
  x.blk = blk;
  x.c = (uint64_t)blk * LANES + x.lane;
  x.gid = P.cluster_base + P.cl_of[x.c];
  if (PXS_CLIENT_LDS) {
    x.l_wcur = reinterpret_cast<uint32_t*>(L + (P.img.off_wcur - tail));
    x.l_wiss = reinterpret_cast<uint32_t*>(L + (P.img.off_wiss - tail));
  } else {                                                   // client tables in the HBM image
    x.l_wcur = reinterpret_cast<uint32_t*>(img + P.img.off_wcur);
    x.l_wiss = reinterpret_cast<uint32_t*>(img + P.img.off_wiss);
  }
  x.l_poison = reinterpret_cast<uint32_t*>(L + (P.img.off_poison - tail));
  x.l_cnt = L + (P.img.off_cnt - tail);
  x.l_agn = L + (P.off_agn - tail);
  x.rec = P.rec + (size_t)blk * P.rec_per_block;
#ifdef PXS_TALLY
  x.tdbg = P.dbg;
#endif
  if (P.AR)
    for (uint32_t k = x.lane; k < 2u * N * LANES; k += LANES) x.l_agn[k] = 0;
  if (P.phase_sort)
    for (uint32_t k = 0; k < P.phase_period; k++) reinterpret_cast<uint32_t*>(x.l_cnt + P.ph_rel)[(k << 6) | x.lane] = 0;
  const bool live = x.c < bound;
  x.es = Proto::kind == PAXISIM_WPAXOS ? 4u : LANES;
  x.hw = true;   // every window is in the HBM image here
  x.kc = live ? P.kc[x.c] : 0u;
  uint32_t b0 = t0 % P.D;
  const bool skip_idle = skip_idle_on<Proto>() && !P.drop_ppm && !P.slow_ppm;
  for (uint32_t t = t0; t < t0 + nsteps; t++) {
    if (PXS_PHASE_RECENT && P.phase_sort && t == t0 + nsteps / 2u)   // the launch's second half only
      for (uint32_t k = 0; k < P.phase_period; k++) reinterpret_cast<uint32_t*>(x.l_cnt + P.ph_rel)[(k << 6) | x.lane] = 0;
#ifndef PXS_STAMPS
    if constexpr (lane_async<NT, Proto>()) {
      const bool run = live && x.l_poison[x.lane] >= t;
      x.t = t;
      x.b0 = b0;
      step_async<NT, Proto>(P, x, run ? replica_order<NT>(P, x, b0) : 0ull, run, img, L + (P.off_wscr - tail));
    } else
#endif
    if (live && x.l_poison[x.lane] >= t) {
      const uint64_t order = busy_first<NT, Proto>() ? replica_order<NT>(P, x, b0) : 0x0FEDCBA987654321ull;
#pragma nounroll
      for (uint32_t k = 0; k < N; k++) {
        const uint32_t r = busy_first<NT, Proto>() ? (uint32_t)(order >> (4u * k)) & 15u : k;
        if constexpr (skip_idle_on<Proto>())
          if (skip_idle && !inbox_any<NT>(x, r, b0, N) && !late_start<NT>(P, t, r)) continue;
        x.r = r;
        x.t = t;
        x.b0 = b0;
        x.ci = ~0u;
        // HBM-resident image regions (a WPaxos bind repoints these at its window)
        x.l_a = reinterpret_cast<uint32_t*>(img + P.img.off_a);
        x.l_b = reinterpret_cast<uint32_t*>(img + P.img.off_b);
        x.l_c = reinterpret_cast<uint32_t*>(img + P.img.off_c);
        const size_t i = rc(P, r, x.c);
        PXS_TALLY_AT(P, x.blk, TC_ROW_LD, &P.flags[i], false);
        x.flags = P.flags[i];
        x.kvver = P.kv ? P.kv_ver[i] : 0u;
#ifdef PXS_TALLY
        if (P.kv) PXS_TALLY_AT(P, x.blk, TC_ROW_LD, &P.kv_ver[i], false);
#endif
        const uint32_t flags0 = row_dirty_on<Proto>() ? x.flags : 0u, kvver0 = row_dirty_on<Proto>() ? x.kvver : 0u;
        Proto::template load<NT>(P, x);
        if constexpr (Proto::step_scratch) Proto::template step_begin<NT>(P, x, L + (P.off_wscr - tail));
        rep_counters_zero<NT>(x);
#ifdef PXS_STAMPS
        Stamps st = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        const unsigned long long sr0 = stamp();
        replica_step<NT, Proto, false>(P, x, &st);
        st.steps = 1;
        st.barrier = stamp() - sr0;   // serial kernel: the whole replica-step (no barrier)
        if (x.lane == 0 && P.dbg) {
          unsigned long long* d = &P.dbg[((size_t)blk * 16 + r) * DBG_PER];
          atomicAdd(&d[0], st.setup); atomicAdd(&d[1], st.loop); atomicAdd(&d[2], st.barrier);
          atomicAdd(&d[3], st.trips); atomicAdd(&d[4], st.msgs); atomicAdd(&d[5], st.steps);
          atomicAdd(&d[6], st.pick); atomicAdd(&d[7], st.disp);
          atomicAdd(&d[8], st.wait); atomicAdd(&d[9], st.flush);
          atomicAdd(&d[10], st.stage); atomicAdd(&d[11], st.tail);
        }
#else
        replica_step<NT, Proto, false>(P, x);
#endif
        wb_flush<NT>(x);
        if (!row_dirty_on<Proto>() || x.flags != flags0) {
          PXS_TALLY_AT(P, x.blk, TC_ROW_ST, &P.flags[i], true);
          P.flags[i] = x.flags;
        }
        if (P.kv && (!row_dirty_on<Proto>() || x.kvver != kvver0)) {
          PXS_TALLY_AT(P, x.blk, TC_ROW_ST, &P.kv_ver[i], true);
          P.kv_ver[i] = x.kvver;
        }
        Proto::template store<NT>(P, x);
        if constexpr (Proto::step_scratch) Proto::template step_end<NT>(P, x);
        rep_counters_flush<NT>(P, x);
      }
    }
    if (P.AR && live) agree_drain<NT, Proto>(P, x, t & 1u);   // this step's arrivals, replica order
    if (++b0 == P.D) b0 = 0;
  }
  if (P.compact && live) {
    uint32_t any = 0;
    const uint32_t nbox = P.D * N * (N + 1u);
    for (uint32_t b = 0; b < nbox; b++) any |= x.l_cnt[(b << 6) | x.lane];
    P.qf[x.c] = any ? 0u : 1u;
    if (P.phase_sort) {   // the residue with the most records (the first on ties)
      const uint32_t* ph = reinterpret_cast<const uint32_t*>(x.l_cnt + P.ph_rel);
      uint32_t best = 0, most = ph[x.lane];
      for (uint32_t k = 1; k < P.phase_period; k++) {
        const uint32_t v = ph[(k << 6) | x.lane];
        if (v > most) { most = v; best = k; }
      }
      // hysteresis: a cluster keeps its residue unless the new one leads it by
      // more than PXS_PHASE_HYST percent, so near-ties do not move it back and forth
      const uint32_t prev = P.phase[x.c];
      if (PXS_PHASE_HYST && prev < P.phase_period && prev != best &&
          most * 100u <= ph[(prev << 6) | x.lane] * (100u + PXS_PHASE_HYST))
        best = prev;
      P.phase[x.c] = best;
    }
  }
  {
    const uint32_t nb = (P.img.bytes - tail) / 16u;
    uint4* g = reinterpret_cast<uint4*>(img + tail);
    for (uint32_t k = threadIdx.x; k < nb; k += LANES) g[k] = lds[k];
  }
#ifdef PXS_WAVE_TIMES
  if (threadIdx.x == 0 && P.dbg) {
    const uint64_t wt1 = __builtin_amdgcn_s_memrealtime();
    P.dbg[2 * (size_t)blk] = wt0;
    P.dbg[2 * (size_t)blk + 1] = wt1;
  }
#endif
}

template <int NT, class Proto>
__global__ void __launch_bounds__(LANES, serial_waves<Proto>()) sim_serial(Params P, uint32_t t0, uint32_t nsteps) {
  extern __shared__ uint4 lds[];
  const uint32_t bound = __builtin_amdgcn_readfirstlane(*P.bound);
  const uint32_t blk = blockIdx.x;
  if ((uint64_t)blk * LANES >= bound) return;
  serial_tile<NT, Proto>(P, blk, bound, t0, nsteps, lds);
}

// The pipelined serial kernel: K chunks of nsteps steps of
// every live tile in one launch, so a slot freed by a tile that finishes its
// chunk takes the next ready (tile, chunk) instead of idling until the last
// wave of the launch ends (config 2 at 2.5 waves per slot: up to 19% idle).
// Clusters are independent, so the only ordering is a tile's own chunks.
// Each workgroup (one wave) takes one ticket from its XCD's queue - tile i
// belongs to XCD i mod 8, tickets chunk-major - so a tile's chunks all run
// under one L2 and the hand-over needs no L2 write-back: the finishing wave
// waits for its stores (vmcnt 0) and raises the tile's chunk count; the next
// chunk's wave polls it and invalidates its L1.
//
// Liveness: a ticket is taken only by a wave that is running, and the wave
// holding ticket j waits only for ticket j - tx (the same tile's previous
// chunk), which was taken earlier, so by a wave that is running or done; by
// induction on j every wait ends, whatever the dispatcher makes resident.
// A poll that outlives the spin limit (q[9], PAXISIM_PIPE_SPIN) sets q[8],
// records the first stuck wait in q[10..15] and leaves, and an XCD given
// fewer workgroups than tickets leaves chunks unrun, which pipe_verify
// (paxisim.hip) reports - either way the host fails loudly at its next call.
// The grid is 8 * ceil(tiles / 8) * K workgroups (the dispatcher deals
// workgroups to the 8 XCDs in turn).
//
// PXS_PIPE_PERSIST (off): the persistent form, a grid of the
// resident slots whose waves loop over tickets.  Round 5's first version of it
// hung on the GPU (gpurun_out/r5t) and its source was not kept; this is the
// form rebuilt to find out why (tools/pipe_persist.sh).
// q: [0, 8) tickets per XCD, [8] error (sticky), [9] spin limit,
//    [10, 16) the first give-up: xcd, ticket, tile, chunk, done[tile], q[xcd];
//    [16, 16 + tiles) chunks done.
#ifndef PXS_PIPE_PERSIST
#define PXS_PIPE_PERSIST 0
#endif
#define PXS_PIPE_SPIN_DEFAULT (1u << 22)   // polls of ~2 us: seconds, against chunks of at most ~0.1 s
template <int NT, class Proto>
__device__ __forceinline__ bool pipe_item(const Params& P, uint32_t t0, uint32_t nsteps, uint32_t K, uint32_t* q,
                                          uint32_t bound, uint32_t xcd, uint32_t tx, uint32_t spin_max, uint4* lds) {
  uint32_t it = 0;
  if (threadIdx.x == 0) it = atomicAdd(&q[xcd], 1u);
  it = __builtin_amdgcn_readfirstlane(it);
  if (it >= tx * K) return false;
  // uniform by construction; said so, so the tile's addressing stays in scalar registers
  const uint32_t c = __builtin_amdgcn_readfirstlane(it / tx);
  const uint32_t blk = __builtin_amdgcn_readfirstlane(xcd + 8u * (it - c * tx));
  uint32_t* done = q + 16;
  if (c) {
    uint32_t spins = 0;
    uint32_t seen;
    while ((seen = __hip_atomic_load(&done[blk], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) < c) {
      __builtin_amdgcn_s_sleep(8);
      if (++spins > spin_max) {
        if (threadIdx.x == 0 && atomicOr(&q[8], 1u) == 0u) {   // the first give-up names its wait
          q[10] = xcd;
          q[11] = it;
          q[12] = blk;
          q[13] = c;
          q[14] = seen;
          q[15] = __hip_atomic_load(&q[xcd], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return false;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // L1 invalidate: the chunk before ran on another CU
  }
  serial_tile<NT, Proto>(P, blk, bound, t0 + c * nsteps, nsteps, lds);
  // the tile's stores must be issued before the wait and the wait before the
  // flag: the fence keeps the compiler from moving a store past the waitcnt
  // (the intrinsic is not a memory barrier to LLVM)
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  __builtin_amdgcn_s_waitcnt(0x0F70);                     // vmcnt(0): the tile's stores are in this XCD's L2
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  if (threadIdx.x == 0) __hip_atomic_store(&done[blk], c + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

template <int NT, class Proto>
__global__ void __launch_bounds__(LANES, serial_waves<Proto>()) sim_serial_pipe(Params P, uint32_t t0, uint32_t nsteps,
                                                                               uint32_t K, uint32_t* q) {
  extern __shared__ uint4 lds[];
  const uint32_t bound = __builtin_amdgcn_readfirstlane(*P.bound);
  const uint32_t tiles = (bound + LANES - 1u) / LANES;
  const uint32_t xcd = __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((32 - 1) << 11)) & 7u;   // HW_REG_XCC_ID
  const uint32_t tx = tiles > xcd ? (tiles - xcd + 7u) / 8u : 0u;
  const uint32_t spin_max = __builtin_amdgcn_readfirstlane(q[9]);
  if constexpr (PXS_PIPE_PERSIST) {
    // every iteration takes a new ticket, so a wave runs at most tx * K items (a bound, not a guess)
    for (uint32_t n = 0; n <= tx * K; n++)
      if (!pipe_item<NT, Proto>(P, t0, nsteps, K, q, bound, xcd, tx, spin_max, lds)) break;
  } else {
    pipe_item<NT, Proto>(P, t0, nsteps, K, q, bound, xcd, tx, spin_max, lds);
  }
}

}  // namespace pxs
