// epaxos_kernel.h — EPaxos handlers on gfx950 (a protocol policy of sim_core.h).
//
// Follows epaxos/replica.go:58-384 and epaxos/instance.go (cited per
// function); oracle/oracle.c restates the same code (ep_*).  Leaderless: every
// replica leads the instances of its own log; instance (o, s) of owner o lives
// in a ring of W over slots (executed[o], executed[o] + W] of each replica.
// Slots at or below executed[o] are COMMITTED for good (execute() advances only
// over committed instances, and no handler changes one afterwards); a message
// for a slot beyond the ring cannot be held: WOVF | UNFAITHFUL.  An entry
// keeps its data after execute() passes it, as Go keeps the instance, until a
// later slot takes the entry (slot tag).
//
// State in HBM (per lane, 64 B per instance, so one instance is one line):
//   ep_inst [blk][r][o][W][64] x 4 uint4: {cmd, req, acks | nrep << 16, seq},
//            {slot, exists | ballot << 8 | status << 16 | changed << 24, dep0, dep1}, {dep2..5}, {dep6..9}
//   ep_sce  [3][o][r][C]       slot, committed, executed of owner o's log
//   ep_cf   [2][o][K][r][C]    conflicts[o][key] {slot or -1, seq}
//   ep_max  [K][r][C]          maxSeqPerKey, -1 = absent
// Ballots are NewBallot(0, owner) only (replica.go:114): stored as 1 + owner.
#pragma once
#include "paxos_kernel.h"

namespace pxs {

constexpr uint32_t EP_NMAX = 10;   // dep words in an instance record
enum { EP_NONE = 0, EP_PREACCEPTED = 1, EP_ACCEPTED = 2, EP_COMMITTED = 3 };

struct EpI {
  uint32_t cmd, req, acks, nrep;
  int32_t seq, slot;
  uint32_t exists, ballot, status, changed;
  int32_t dep[EP_NMAX];
};

template <int NT>
__device__ __forceinline__ size_t ep_at(const Params& P, const Rep<NT>& x, uint32_t o, int32_t s) {
  const uint32_t N = nrep<NT>(P);
  return (((((size_t)x.blk * N + x.r) * N + o) * P.W + ((uint32_t)s & (P.W - 1u))) * LANES + x.lane) * 4u;
}
template <int NT>
__device__ __forceinline__ size_t ep_sce(const Params& P, const Rep<NT>& x, uint32_t k, uint32_t o) {
  const uint32_t N = nrep<NT>(P);
  return (((size_t)k * N + o) * N + x.r) * P.C + x.c;
}
template <int NT>
__device__ __forceinline__ size_t ep_cfi(const Params& P, const Rep<NT>& x, uint32_t k, uint32_t o, uint32_t key) {
  const uint32_t N = nrep<NT>(P);
  return ((((size_t)k * N + o) * P.keys + key) * N + x.r) * P.C + x.c;
}
template <int NT>
__device__ __forceinline__ size_t ep_maxi(const Params& P, const Rep<NT>& x, uint32_t key) {
  return ((size_t)key * nrep<NT>(P) + x.r) * P.C + x.c;
}
template <int NT>
__device__ __forceinline__ int32_t ep_get(const Params& P, const Rep<NT>& x, uint32_t k, uint32_t o) {
  return (int32_t)ldg(&P.ep_sce[ep_sce<NT>(P, x, k, o)]);
}
template <int NT>
__device__ __forceinline__ void ep_set(const Params& P, const Rep<NT>& x, uint32_t k, uint32_t o, int32_t v) {
  P.ep_sce[ep_sce<NT>(P, x, k, o)] = (uint32_t)v;
}

template <int NT>
__device__ __forceinline__ void ep_load(const Params& P, const Rep<NT>& x, size_t i, EpI& e) {
  const uint4 a = ldg(&P.ep_inst[i]), b = ldg(&P.ep_inst[i + 1]), c = ldg(&P.ep_inst[i + 2]), d = ldg(&P.ep_inst[i + 3]);
  e.cmd = a.x; e.req = a.y; e.acks = a.z & 0xFFFFu; e.nrep = a.z >> 16; e.seq = (int32_t)a.w;
  e.slot = (int32_t)b.x;
  e.exists = b.y & 0xFFu; e.ballot = (b.y >> 8) & 0xFFu; e.status = (b.y >> 16) & 0xFFu; e.changed = b.y >> 24;
  const uint32_t w[EP_NMAX] = {b.z, b.w, c.x, c.y, c.z, c.w, d.x, d.y, d.z, d.w};
#pragma unroll
  for (uint32_t k = 0; k < EP_NMAX; k++) e.dep[k] = (int32_t)w[k];
}
template <int NT>
__device__ __forceinline__ void ep_store(const Params& P, size_t i, const EpI& e) {
  P.ep_inst[i] = make_uint4(e.cmd, e.req, e.acks | (e.nrep << 16), (uint32_t)e.seq);
  P.ep_inst[i + 1] = make_uint4((uint32_t)e.slot, e.exists | (e.ballot << 8) | (e.status << 16) | (e.changed << 24),
                                (uint32_t)e.dep[0], (uint32_t)e.dep[1]);
  P.ep_inst[i + 2] = make_uint4((uint32_t)e.dep[2], (uint32_t)e.dep[3], (uint32_t)e.dep[4], (uint32_t)e.dep[5]);
  P.ep_inst[i + 3] = make_uint4((uint32_t)e.dep[6], (uint32_t)e.dep[7], (uint32_t)e.dep[8], (uint32_t)e.dep[9]);
}
__device__ __forceinline__ void ep_new(EpI& e, int32_t s) {
  e.cmd = e.req = e.acks = e.nrep = 0;
  e.seq = 0;
  e.slot = s;
  e.exists = 1;
  e.ballot = e.status = e.changed = 0;
#pragma unroll
  for (uint32_t k = 0; k < EP_NMAX; k++) e.dep[k] = 0;
}
__device__ __forceinline__ bool ep_live(const EpI& e, int32_t s) { return e.exists && e.slot == s; }

// 0: at or below executed (COMMITTED for good), 1: in the ring, 2: beyond it
template <int NT>
__device__ __forceinline__ int ep_where(const Params& P, const Rep<NT>& x, uint32_t o, int32_t s) {
  const int32_t ex = ep_get<NT>(P, x, 2, o);
  if (s <= ex) return 0;
  return s > ex + (int32_t)P.W ? 2 : 1;
}

template <int NT>
__device__ __forceinline__ uint32_t ep_key(const Params& P, Rep<NT>& x, uint32_t cmd) {
  return key_fit<NT>(P, x, wl_key(P, x.kc, cmd));
}

// attributes (replica.go:58-80): seq = 1 + the largest seq among the latest
// conflicting instance of every log (dep), and above maxSeqPerKey
template <int NT>
__device__ __forceinline__ int32_t ep_attributes(const Params& P, Rep<NT>& x, uint32_t key, int32_t (&dep)[EP_NMAX]) {
  const uint32_t N = nrep<NT>(P);
  int32_t seq = 0;
#pragma unroll
  for (uint32_t k = 0; k < EP_NMAX; k++) dep[k] = 0;
  for (uint32_t id = 0; id < N; id++) {
    const int32_t d = (int32_t)ldg(&P.ep_cf[ep_cfi<NT>(P, x, 0, id, key)]);
    if (d < 0 || d <= 0) continue;                       // absent, or not above dep[id] == 0
    int32_t sd = (int32_t)ldg(&P.ep_cf[ep_cfi<NT>(P, x, 1, id, key)]);
    if (ep_where<NT>(P, x, id, d) == 1) {                // in the ring: its current seq
      const uint4 a = ldg(&P.ep_inst[ep_at<NT>(P, x, id, d)]), b = ldg(&P.ep_inst[ep_at<NT>(P, x, id, d) + 1]);
      if ((b.y & 0xFFu) && (int32_t)b.x == d) sd = (int32_t)a.w;
    }
#pragma unroll
    for (uint32_t k = 0; k < EP_NMAX; k++)
      if (k == id) dep[k] = d;
    if (seq <= sd) seq = sd + 1;
  }
  const int32_t ms = (int32_t)ldg(&P.ep_max[ep_maxi<NT>(P, x, key)]);
  if (ms >= 0 && seq <= ms) seq = ms + 1;
  return seq;
}

// update (replica.go:83-101)
template <int NT>
__device__ __forceinline__ void ep_update(const Params& P, Rep<NT>& x, uint32_t cmd, uint32_t id, int32_t slot,
                                          int32_t seq) {
  const uint32_t k = ep_key<NT>(P, x, cmd);
  const size_t ci = ep_cfi<NT>(P, x, 0, id, k);
  const int32_t d = (int32_t)ldg(&P.ep_cf[ci]);
  if (d < 0 || d < slot) {
    P.ep_cf[ci] = (uint32_t)slot;
    P.ep_cf[ep_cfi<NT>(P, x, 1, id, k)] = (uint32_t)seq;
  }
  const size_t mi = ep_maxi<NT>(P, x, k);
  if ((int32_t)ldg(&P.ep_max[mi]) < seq) P.ep_max[mi] = (uint32_t)seq;
}

// a message with payload words: header record {type | n << 8, w1, w2, w3} + n records
template <int NT>
__device__ __forceinline__ void ep_send(const Params& P, Rep<NT>& x, uint32_t to, uint32_t type, uint32_t w1,
                                        uint32_t w2, uint32_t w3, const uint32_t* pay, uint32_t npay) {
  const uint32_t n = (npay + 3u) / 4u;
  uint32_t ri;
  if (!send_begin<NT>(P, x, to, 1u + n, ri)) return;
  x.rec[ri] = make_uint4(type | (n << 8), w1, w2, w3);
  for (uint32_t k = 0; k < n; k++) {
    uint32_t w[4];
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) w[j] = 4u * k + j < npay ? pay[4u * k + j] : 0u;
    x.rec[ri + (k + 1u) * LANES] = make_uint4(w[0], w[1], w[2], w[3]);
  }
}
template <int NT>
__device__ __forceinline__ void ep_broadcast(const Params& P, Rep<NT>& x, uint32_t type, uint32_t w1, uint32_t w2,
                                             uint32_t w3, const uint32_t* pay, uint32_t npay) {
  intent_flush<NT>(P, x);                                // keep every link's record order
  for (uint32_t d = 0; d < nrep<NT>(P); d++)
    if (d != x.r) ep_send<NT>(P, x, d, type, w1, w2, w3, pay, npay);
}

// i.request.Reply (message.go:32-34): req.c is buffered 1 (http.go:97), so the
// HTTP handler takes the first reply, the second waits, a third would block
template <int NT>
__device__ __forceinline__ void ep_reply(const Params& P, Rep<NT>& x, EpI& e, uint32_t value) {
  if (++e.nrep >= 3u) x.flags |= PAXISIM_F_UNFAITHFUL;
  request_reply<NT>(P, x, e.req, e.cmd, value);
}

// execute (replica.go:355-384): owners in index order where Go ranges over a map
template <int NT>
__device__ void ep_execute(const Params& P, Rep<NT>& x) {
  const uint32_t N = nrep<NT>(P);
  for (uint32_t id = 0; id < N; id++) {
    const int32_t top = ep_get<NT>(P, x, 0, id);
    for (int32_t sl = ep_get<NT>(P, x, 2, id) + 1; sl <= top; sl++) {
      const int w = ep_where<NT>(P, x, id, sl);
      if (w == 2) { x.flags |= PAXISIM_F_WOVF | PAXISIM_F_UNFAITHFUL; continue; }
      const size_t ii = ep_at<NT>(P, x, id, sl);
      EpI e;
      ep_load<NT>(P, x, ii, e);
      if (!ep_live(e, sl)) continue;                     // nil: skipped, not executed
      if (e.status != EP_COMMITTED) break;
      x.digest = mix64(x.digest ^ (((uint64_t)((id << 24) | (uint32_t)sl) << 32) | e.cmd));
      x.execute++;                                       // Execute calls, re-executions included
      const uint32_t h = P.kv ? wl_hash(x.kc, e.cmd) : 0u;
      const uint32_t key = P.kv ? kv_key<NT>(P, x, h, e.cmd) : 0u;
      const uint32_t v = P.kv && e.req ? kv_get<NT>(P, x, key) : 0u;   // v := r.Execute(i.cmd)
      if (P.kv) kv_exec<NT>(P, x, h, key, e.cmd);
      if (e.req) {
        ep_reply<NT>(P, x, e, v);
        P.ep_inst[ii] = make_uint4(e.cmd, e.req, e.acks | (e.nrep << 16), (uint32_t)e.seq);
      }
      if (sl == ep_get<NT>(P, x, 2, id) + 1) {
        const uint32_t k = ep_key<NT>(P, x, e.cmd);
        if ((int32_t)ldg(&P.ep_cf[ep_cfi<NT>(P, x, 0, id, k)]) == sl) P.ep_cf[ep_cfi<NT>(P, x, 1, id, k)] = (uint32_t)e.seq;
        ep_set<NT>(P, x, 2, id, sl);
      }
    }
  }
}

// updateCommit (replica.go:103-111)
template <int NT>
__device__ void ep_update_commit(const Params& P, Rep<NT>& x, uint32_t id) {
  for (;;) {
    const int32_t nx = ep_get<NT>(P, x, 1, id) + 1;
    const int w = ep_where<NT>(P, x, id, nx);
    if (w == 2) {
      if (nx <= ep_get<NT>(P, x, 0, id)) x.flags |= PAXISIM_F_WOVF | PAXISIM_F_UNFAITHFUL;
      break;
    }
    if (w == 1) {
      const uint4 b = ldg(&P.ep_inst[ep_at<NT>(P, x, id, nx) + 1]);
      if (!((b.y & 0xFFu) && (int32_t)b.x == nx && ((b.y >> 16) & 0xFFu) == EP_COMMITTED)) break;
    }
    ep_set<NT>(P, x, 1, id, nx);
  }
  ep_execute<NT>(P, x);
}

template <int NT>
__device__ void ep_handle_request(const Params& P, Rep<NT>& x, uint32_t req) {   // replica.go:113-145
  const uint32_t N = nrep<NT>(P), self = x.r, cmd = req_cid(req), key = ep_key<NT>(P, x, cmd);
  const int32_t s = ep_get<NT>(P, x, 0, self) + 1;
  ep_set<NT>(P, x, 0, self, s);
  int32_t dep[EP_NMAX];
  const int32_t seq = ep_attributes<NT>(P, x, key, dep);
  if (ep_where<NT>(P, x, self, s) != 1) { x.flags |= PAXISIM_F_WOVF | PAXISIM_F_UNFAITHFUL; return; }
  EpI e;
  ep_new(e, s);
  e.cmd = cmd;
  e.ballot = 1u + self;
  e.status = EP_PREACCEPTED;
  e.seq = seq;
#pragma unroll
  for (uint32_t k = 0; k < EP_NMAX; k++) e.dep[k] = dep[k];
  e.req = req;
  e.acks = 1u << self;                                   // self ack
  ep_store<NT>(P, ep_at<NT>(P, x, self, s), e);
  ep_update<NT>(P, x, cmd, self, s, seq);
  uint32_t pay[1 + EP_NMAX];
  pay[0] = (uint32_t)seq;
#pragma unroll
  for (uint32_t k = 0; k < EP_NMAX; k++) pay[1 + k] = (uint32_t)dep[k];
  ep_broadcast<NT>(P, x, PAXISIM_MSG_PREACCEPT, e.ballot, (uint32_t)s, cmd, pay, 1u + N);
}

template <int NT>
__device__ void ep_handle_preaccept(const Params& P, Rep<NT>& x, uint32_t o, const uint4& m, uint32_t ri) {  // 147-191
  const uint32_t N = nrep<NT>(P);
  const int32_t s = (int32_t)m.z;
  const uint32_t mb = m.y, mcmd = m.w;
  const int w = ep_where<NT>(P, x, o, s);
  if (w == 0) return;                                    // COMMITTED, command set: no reply
  if (w == 2) { x.flags |= PAXISIM_F_WOVF | PAXISIM_F_UNFAITHFUL; return; }
  const uint4 p0 = ldg(&x.rec[ri + LANES]);              // seq, dep0..2
  const size_t ii = ep_at<NT>(P, x, o, s);
  EpI e;
  ep_load<NT>(P, x, ii, e);
  if (!ep_live(e, s)) ep_new(e, s);                      // &instance{}
  if (e.status == EP_COMMITTED || e.status == EP_ACCEPTED) {
    if (!e.cmd) {
      e.cmd = mcmd;
      ep_store<NT>(P, ii, e);
      ep_update<NT>(P, x, mcmd, o, s, (int32_t)p0.x);
    } else {
      ep_store<NT>(P, ii, e);                            // a fresh &instance{} is stored either way
    }
    return;
  }
  if (s > ep_get<NT>(P, x, 0, o)) ep_set<NT>(P, x, 0, o, s);
  int32_t dep[EP_NMAX];
  const int32_t seq = ep_attributes<NT>(P, x, ep_key<NT>(P, x, mcmd), dep);
  if (mb >= e.ballot) {
    e.ballot = mb;
    e.cmd = mcmd;
    e.status = EP_PREACCEPTED;
    e.seq = seq;
#pragma unroll
    for (uint32_t k = 0; k < EP_NMAX; k++) e.dep[k] = dep[k];
  }
  ep_store<NT>(P, ii, e);
  ep_update<NT>(P, x, mcmd, o, s, seq);
  uint32_t pay[2 * EP_NMAX];
  for (uint32_t k = 0; k < N; k++) {
    pay[k] = (uint32_t)e.dep[k < EP_NMAX ? k : 0];
    pay[N + k] = (uint32_t)ep_get<NT>(P, x, 1, k);
  }
  intent_flush<NT>(P, x);
  ep_send<NT>(P, x, o, PAXISIM_MSG_PREACCEPTREPLY, e.ballot, (uint32_t)s, (uint32_t)seq, pay, 2u * N);
}

template <int NT>
__device__ __forceinline__ void ep_commit_broadcast(const Params& P, Rep<NT>& x, const EpI& e, int32_t s) {
  uint32_t pay[1 + EP_NMAX];
  pay[0] = (uint32_t)e.seq;
#pragma unroll
  for (uint32_t k = 0; k < EP_NMAX; k++) pay[1 + k] = (uint32_t)e.dep[k];
  ep_broadcast<NT>(P, x, PAXISIM_MSG_COMMIT, e.ballot, (uint32_t)s, e.cmd, pay, 1u + nrep<NT>(P));
}

template <int NT>
__device__ void ep_handle_preaccept_reply(const Params& P, Rep<NT>& x, uint32_t src, const uint4& m, uint32_t ri) {  // 193-260
  const uint32_t N = nrep<NT>(P);
  const int32_t sl = (int32_t)m.z;
  if (ep_where<NT>(P, x, x.r, sl) != 1) return;          // executed: COMMITTED
  const size_t ii = ep_at<NT>(P, x, x.r, sl);
  EpI e;
  ep_load<NT>(P, x, ii, e);
  if (!ep_live(e, sl) || e.status != EP_PREACCEPTED) return;
  if (m.y > e.ballot) return;
  e.acks |= 1u << src;
  if ((int32_t)m.w > e.seq) { e.seq = (int32_t)m.w; e.changed = 1; }          // merge (instance.go:30-41)
  bool committed = true;
  for (uint32_t k = 0; k < 2u * N; k++) {                // payload: Dep[N], Committed[N]
    const uint4 r4 = ldg(&x.rec[ri + (k / 4u + 1u) * LANES]);
    const uint32_t j = k & 3u;
    const int32_t v = (int32_t)(j == 0 ? r4.x : j == 1 ? r4.y : j == 2 ? r4.z : r4.w);
    if (k < N) {
#pragma unroll
      for (uint32_t q = 0; q < EP_NMAX; q++)
        if (q == k && v > e.dep[q]) { e.dep[q] = v; e.changed = 1; }
    } else {
      const uint32_t id = k - N;
      int32_t c = ep_get<NT>(P, x, 1, id);
      if (v > c) { c = v; ep_set<NT>(P, x, 1, id, c); }
      int32_t di = 0;
#pragma unroll
      for (uint32_t q = 0; q < EP_NMAX; q++)
        if (q == id) di = e.dep[q];
      if (c >= 0 && c < di) committed = false;
    }
  }
  if (__popc(e.acks) >= (int)(N * 3u / 4u)) {            // FastQuorum (quorum.go:65-67)
    if (!e.changed && committed) {                       // fast path
      e.status = EP_COMMITTED;
      x.commits++;
      ep_store<NT>(P, ii, e);
      ep_update_commit<NT>(P, x, x.r);
      ep_load<NT>(P, x, ii, e);                          // execute() may have replied
      ep_commit_broadcast<NT>(P, x, e, sl);
      if (P.rwc && e.req) {
        ep_reply<NT>(P, x, e, 0u);
        ep_store<NT>(P, ii, e);
      }
      return;
    }
    e.status = EP_ACCEPTED;                              // slow path
    e.acks = 1u << x.r;
    ep_store<NT>(P, ii, e);
    uint32_t pay[EP_NMAX];
#pragma unroll
    for (uint32_t k = 0; k < EP_NMAX; k++) pay[k] = (uint32_t)e.dep[k];
    ep_broadcast<NT>(P, x, PAXISIM_MSG_ACCEPT, e.ballot, (uint32_t)sl, (uint32_t)e.seq, pay, N);
    return;
  }
  ep_store<NT>(P, ii, e);
}

template <int NT>
__device__ void ep_handle_accept(const Params& P, Rep<NT>& x, uint32_t o, const uint4& m, uint32_t ri) {  // 262-290
  const uint32_t N = nrep<NT>(P);
  const int32_t s = (int32_t)m.z;
  const int w = ep_where<NT>(P, x, o, s);
  if (w == 0) return;
  if (w == 2) { x.flags |= PAXISIM_F_WOVF | PAXISIM_F_UNFAITHFUL; return; }
  const size_t ii = ep_at<NT>(P, x, o, s);
  EpI e;
  ep_load<NT>(P, x, ii, e);
  if (!ep_live(e, s)) ep_new(e, s);
  if (e.status == EP_COMMITTED) {
    ep_store<NT>(P, ii, e);
    return;
  }
  if (s > ep_get<NT>(P, x, 0, o)) ep_set<NT>(P, x, 0, o, s);
  if (m.y >= e.ballot) {
    e.status = EP_ACCEPTED;
    e.ballot = m.y;
    e.seq = (int32_t)m.w;
    for (uint32_t k = 0; k < N; k++) {
      const uint4 r4 = ldg(&x.rec[ri + (k / 4u + 1u) * LANES]);
      const uint32_t j = k & 3u;
      const int32_t v = (int32_t)(j == 0 ? r4.x : j == 1 ? r4.y : j == 2 ? r4.z : r4.w);
#pragma unroll
      for (uint32_t q = 0; q < EP_NMAX; q++)
        if (q == k) e.dep[q] = v;
    }
  }
  ep_store<NT>(P, ii, e);
  post_unicast<NT>(P, x, o, PAXISIM_MSG_ACCEPTREPLY, e.ballot, (uint32_t)s, 0u);
}

template <int NT>
__device__ void ep_handle_accept_reply(const Params& P, Rep<NT>& x, uint32_t src, const uint4& m) {  // 292-321
  const int32_t sl = (int32_t)m.z;
  if (ep_where<NT>(P, x, x.r, sl) != 1) return;
  const size_t ii = ep_at<NT>(P, x, x.r, sl);
  EpI e;
  ep_load<NT>(P, x, ii, e);
  if (!ep_live(e, sl) || e.status != EP_ACCEPTED) return;
  if (e.ballot < m.y) {
    e.ballot = m.y;
    ep_store<NT>(P, ii, e);
    return;
  }
  e.acks |= 1u << src;
  if (__popc(e.acks) > (int)(nrep<NT>(P) / 2u)) {        // Majority
    e.status = EP_COMMITTED;
    x.commits++;
    ep_store<NT>(P, ii, e);
    ep_update_commit<NT>(P, x, x.r);
    ep_load<NT>(P, x, ii, e);
    if (P.rwc && e.req) {
      ep_reply<NT>(P, x, e, 0u);
      ep_store<NT>(P, ii, e);
    }
    ep_commit_broadcast<NT>(P, x, e, sl);
    return;
  }
  ep_store<NT>(P, ii, e);
}

// the request's worker is re-queued at this replica for the next step
template <int NT>
__device__ __forceinline__ void ep_retry(const Params& P, Rep<NT>& x, uint32_t cid) {
  uint32_t b = x.b0 + 1u;
  if (b >= P.D) b -= P.D;
  const uint32_t box = (b * nrep<NT>(P) + x.r) * P.NS + nrep<NT>(P);
  uint8_t* cp = &x.l_cnt[(box << 6) | x.lane];
  const uint32_t k = *cp;
  if (k >= P.M) {
    x.flags |= PAXISIM_F_MBOX_OVF | PAXISIM_F_UNFAITHFUL;
    return;
  }
  x.rec[((box * P.M + k) << 6) | x.lane] = make_uint4(PAXISIM_MSG_REQUEST, 0u, 0u, cid);
  *cp = (uint8_t)(k + 1u);
}

template <int NT>
__device__ void ep_handle_commit(const Params& P, Rep<NT>& x, uint32_t o, const uint4& m, uint32_t ri) {  // 323-353
  const uint32_t N = nrep<NT>(P);
  const int32_t s = (int32_t)m.z;
  const int w = ep_where<NT>(P, x, o, s);
  if (s > ep_get<NT>(P, x, 0, o)) ep_set<NT>(P, x, 0, o, s);
  if (w == 2) { x.flags |= PAXISIM_F_WOVF | PAXISIM_F_UNFAITHFUL; return; }
  const int32_t mseq = (int32_t)ldg(&x.rec[ri + LANES]).x;
  if (w == 0) {                                          // committed for good: re-commit in place
    const uint32_t k = ep_key<NT>(P, x, m.w);
    const bool mine = (int32_t)ldg(&P.ep_cf[ep_cfi<NT>(P, x, 0, o, k)]) == s;
    ep_update<NT>(P, x, m.w, o, s, mseq);
    if (mine) P.ep_cf[ep_cfi<NT>(P, x, 1, o, k)] = (uint32_t)mseq;
    ep_update_commit<NT>(P, x, o);
    return;
  }
  const size_t ii = ep_at<NT>(P, x, o, s);
  EpI e;
  ep_load<NT>(P, x, ii, e);
  if (!ep_live(e, s)) ep_new(e, s);
  if (m.y >= e.ballot) {
    e.ballot = m.y;
    e.cmd = m.w;
    e.status = EP_COMMITTED;
    e.seq = mseq;
    for (uint32_t k = 0; k < N; k++) {
      const uint4 r4 = ldg(&x.rec[ri + ((k + 1u) / 4u + 1u) * LANES]);
      const uint32_t j = (k + 1u) & 3u;
      const int32_t v = (int32_t)(j == 0 ? r4.x : j == 1 ? r4.y : j == 2 ? r4.z : r4.w);
#pragma unroll
      for (uint32_t q = 0; q < EP_NMAX; q++)
        if (q == k) e.dep[q] = v;
    }
    ep_store<NT>(P, ii, e);
    ep_update<NT>(P, x, m.w, o, s, mseq);
  }
  if (e.req) {                                           // r.Retry: back into MessageChan
    ep_retry<NT>(P, x, req_cid(e.req));
    e.req = 0;
  }
  ep_store<NT>(P, ii, e);
  ep_update_commit<NT>(P, x, o);
}

struct EPaxosProto {
  static constexpr uint32_t kind = PAXISIM_EPAXOS;
  static constexpr bool step_scratch = false;   // (no per-replica-step LDS scratch: sim_core.h sim_serial)
  template <int NT>
  __device__ static __forceinline__ void load(const Params& P, Rep<NT>& x) {
    const size_t i = rc(P, x.r, x.c);
    x.digest = P.digest[i];
    x.execute = (int32_t)P.execute[i];   // Execute calls
    x.nfwd = P.nfwd[i];
    x.key = 0;
    x.ktag = 0;
    x.inst = x.r;
  }
  template <int NT>
  __device__ static __forceinline__ void store(const Params& P, const Rep<NT>& x) {
    const size_t i = rc(P, x.r, x.c);
    P.digest[i] = x.digest;
    P.execute[i] = (uint32_t)x.execute;
    P.nfwd[i] = x.nfwd;
  }
  template <int NT>
  __device__ static __forceinline__ void client_request(const Params& P, Rep<NT>& x, uint32_t cid) {
    ep_handle_request<NT>(P, x, mkreq(cid, PAXISIM_CLIENT_SRC));
  }
  // registrations replica.go:49-54
  template <int NT>
  __device__ static __forceinline__ void dispatch(const Params& P, Rep<NT>& x, uint32_t src, const uint4& m,
                                                  uint32_t ri) {
    switch (hdr_type(m.x)) {
      case PAXISIM_MSG_REQUEST: dv_inc<NT>(x, PAXISIM_MSG_REQUEST); ep_handle_request<NT>(P, x, mkreq(m.w, src)); break;
      case PAXISIM_MSG_REPLY: dv_inc<NT>(x, PAXISIM_MSG_REPLY); handle_reply<NT>(P, x, m.w, m.y); break;
      case PAXISIM_MSG_PREACCEPT: dv_inc<NT>(x, PAXISIM_MSG_PREACCEPT); ep_handle_preaccept<NT>(P, x, src, m, ri); break;
      case PAXISIM_MSG_PREACCEPTREPLY:
        dv_inc<NT>(x, PAXISIM_MSG_PREACCEPTREPLY);
        ep_handle_preaccept_reply<NT>(P, x, src, m, ri);
        break;
      case PAXISIM_MSG_ACCEPT: dv_inc<NT>(x, PAXISIM_MSG_ACCEPT); ep_handle_accept<NT>(P, x, src, m, ri); break;
      case PAXISIM_MSG_ACCEPTREPLY: dv_inc<NT>(x, PAXISIM_MSG_ACCEPTREPLY); ep_handle_accept_reply<NT>(P, x, src, m); break;
      case PAXISIM_MSG_COMMIT: dv_inc<NT>(x, PAXISIM_MSG_COMMIT); ep_handle_commit<NT>(P, x, src, m, ri); break;
      default: break;
    }
  }
};

}  // namespace pxs
