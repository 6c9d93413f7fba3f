// abd_kernel.h — ABD atomic storage handlers on gfx950 (a protocol policy of sim_core.h).
//
// Follows abd/replica.go:50-157 (cited per function).  A replica coordinates
// the client requests it receives in two majority rounds: Get (collect the
// highest version) then Set (write back, or write version+1).  Versions have
// no writer-id tie-break (abd/replica.go:123), so concurrent writers can
// commit different values under one version; that behaviour is reproduced.
//
// ABD state during a launch:
//   registers: op counter (cid, abd/replica.go:30), history length
//   LDS:       KV value [r][K][lane] (region a), KV version (region b),
//              op table [r][OW][6][lane] (region c): tag, request, state|get<<2|set<<17,
//              value, version, start step
//   HBM:       completed-op history [r][C][H] for the linearizability scan
// Records: hdr = type | key << 8, y = op id (CID), z = version, w = value
// (a write's value is its command id; 0 is nil).
#pragma once
#include "sim_core.h"

namespace pxs {

template <int NT>
__device__ __forceinline__ uint32_t kv_i(const Params& P, const Rep<NT>& x, uint32_t key) {
  return ((x.r * P.keys + key) << 6) | x.lane;
}
template <int NT>
__device__ __forceinline__ uint32_t op_i(const Params& P, const Rep<NT>& x, uint32_t opid, uint32_t f) {
  return (((x.r * P.OW + (opid & (P.OW - 1u))) * ABD_OPF + f) << 6) | x.lane;
}

// database.Put (db.go:123-134): only a non-nil value is written
template <int NT>
__device__ __forceinline__ void abd_put(const Params& P, Rep<NT>& x, uint32_t key, uint32_t val) {
  if (val) x.l_a[kv_i<NT>(P, x, key)] = val;
}

template <int NT>
__device__ __forceinline__ bool abd_majority(const Params& P, uint32_t mask) {   // quorum.go:60-62
  return __popc(mask) > (int)(nrep<NT>(P) / 2);
}

template <int NT>
__device__ __forceinline__ void abd_handle_request(const Params& P, Rep<NT>& x, uint32_t cid) {  // replica.go:50-71
  const uint32_t k = key_fit<NT>(P, x, wl_key(P, x.kc, cid));
  const uint32_t opid = (uint32_t)x.slot + 1u;
  x.slot = (int32_t)opid;
  const uint32_t st = x.l_c[op_i<NT>(P, x, opid, 2)] & 3u;
  if (st == ABD_GET || st == ABD_SET) x.flags |= PAXISIM_F_PEND_OVF | PAXISIM_F_UNFAITHFUL;  // evicting a live op
  const uint32_t ki = kv_i<NT>(P, x, k);
  x.l_c[op_i<NT>(P, x, opid, 0)] = opid;
  x.l_c[op_i<NT>(P, x, opid, 1)] = cid;
  x.l_c[op_i<NT>(P, x, opid, 2)] = ABD_GET | ((1u << x.r) << 2);
  x.l_c[op_i<NT>(P, x, opid, 3)] = x.l_a[ki];
  x.l_c[op_i<NT>(P, x, opid, 4)] = x.l_b[ki];
  x.l_c[op_i<NT>(P, x, opid, 5)] = x.t;
  post_broadcast<NT>(P, x, PAXISIM_MSG_GET | (k << 8), opid, 0u, 0u);
}

template <int NT>
__device__ __forceinline__ void abd_handle_get(const Params& P, Rep<NT>& x, uint32_t src, uint32_t key,
                                               uint32_t opid) {                     // replica.go:73-82
  const uint32_t ki = kv_i<NT>(P, x, key);
  post_unicast<NT>(P, x, src, PAXISIM_MSG_GETREPLY | (key << 8), opid, x.l_b[ki], x.l_a[ki]);
}

template <int NT>
__device__ __forceinline__ void abd_handle_set(const Params& P, Rep<NT>& x, uint32_t src, uint32_t key, uint32_t opid,
                                               uint32_t ver, uint32_t val) {        // replica.go:84-95
  const uint32_t ki = kv_i<NT>(P, x, key);
  if (ver > x.l_b[ki]) {
    abd_put<NT>(P, x, key, val);
    x.l_b[ki] = ver;
  }
  post_unicast<NT>(P, x, src, PAXISIM_MSG_SETREPLY | (key << 8), opid, 0u, 0u);
}

template <int NT>
__device__ __forceinline__ void abd_handle_getreply(const Params& P, Rep<NT>& x, uint32_t src, uint32_t key,
                                                    uint32_t opid, uint32_t ver, uint32_t val) {  // replica.go:97-136
  if (x.l_c[op_i<NT>(P, x, opid, 0)] != opid) return;    // retired: Done in Go, or flagged when evicted
  const uint32_t si = op_i<NT>(P, x, opid, 2);
  uint32_t sm = x.l_c[si];
  if ((sm & 3u) != ABD_GET) return;
  const uint32_t vi = op_i<NT>(P, x, opid, 3), ni = op_i<NT>(P, x, opid, 4);
  uint32_t ev = x.l_c[vi], en = x.l_c[ni];
  const uint32_t ki = kv_i<NT>(P, x, key);
  if (ver > en) {
    ev = val;
    en = ver;
    abd_put<NT>(P, x, key, val);
    x.l_b[ki] = ver;
  }
  sm |= (1u << src) << 2;
  if (abd_majority<NT>(P, (sm >> 2) & 0x7FFFu)) {
    sm = (sm & ~3u) | ABD_SET | ((1u << x.r) << 17);
    const uint32_t req = x.l_c[op_i<NT>(P, x, opid, 1)];
    if (wl_write(P, x.kc, req)) {
      ev = req;                                         // the write's value
      en++;
      abd_put<NT>(P, x, key, ev);
      x.l_b[ki] = en;
    }
    post_broadcast<NT>(P, x, PAXISIM_MSG_SET | (key << 8), opid, en, ev);
  }
  x.l_c[si] = sm;
  x.l_c[vi] = ev;
  x.l_c[ni] = en;
}

template <int NT>
__device__ __forceinline__ void abd_handle_setreply(const Params& P, Rep<NT>& x, uint32_t src, uint32_t key,
                                                    uint32_t opid) {                // replica.go:138-157
  if (x.l_c[op_i<NT>(P, x, opid, 0)] != opid) return;
  const uint32_t si = op_i<NT>(P, x, opid, 2);
  uint32_t sm = x.l_c[si];
  if ((sm & 3u) != ABD_SET) return;
  sm |= (1u << src) << 17;
  if (abd_majority<NT>(P, sm >> 17)) {
    sm = (sm & ~3u) | ABD_DONE;
    x.commits++;
    const uint32_t req = x.l_c[op_i<NT>(P, x, opid, 1)];
    const uint32_t w = wl_write(P, x.kc, req) ? 1u : 0u;
    if ((uint32_t)x.execute < P.H) {                   // History.AddOperation (history.go:44-52)
      P.hist[((size_t)x.r * P.C + x.c) * P.H + (uint32_t)x.execute] =
          make_uint4(key | (w << 31), x.l_c[op_i<NT>(P, x, opid, 3)], x.l_c[op_i<NT>(P, x, opid, 5)], x.t);
      x.execute++;
    } else if (P.H) {
      x.flags |= PAXISIM_F_HIST_OVF;
    }
    x.l_c[si] = sm;
    client_reply<NT>(P, x, req, w ? 0u : x.l_c[op_i<NT>(P, x, opid, 3)]);   // Reply{Value: e.value} for a read
    return;
  }
  x.l_c[si] = sm;
}

struct AbdProto {
  static constexpr uint32_t kind = PAXISIM_ABD;
  static constexpr bool step_scratch = false;   // (no per-replica-step LDS scratch: sim_core.h sim_serial)
  template <int NT>
  __device__ static __forceinline__ void load(const Params& P, Rep<NT>& x) {
    const size_t i = rc(P, x.r, x.c);
    x.slot = (int32_t)P.slot[i];        // op counter
    x.execute = (int32_t)P.execute[i];  // history length
  }
  template <int NT>
  __device__ static __forceinline__ void store(const Params& P, const Rep<NT>& x) {
    const size_t i = rc(P, x.r, x.c);
    P.slot[i] = (uint32_t)x.slot;
    P.execute[i] = (uint32_t)x.execute;
  }
  template <int NT>
  __device__ static __forceinline__ void client_request(const Params& P, Rep<NT>& x, uint32_t cid) {
    abd_handle_request<NT>(P, x, cid);
  }
  // A GetReply or SetReply that does not complete its majority sends nothing
  // (replica.go:97-157): apply it as the full handler would and return true
  // (a late reply to a retired op or a finished phase is ignored).  Returns
  // false, with no effect, for every other message.
  template <int NT>
  __device__ static __forceinline__ bool absorb(const Params& P, Rep<NT>& x, uint32_t src, const uint4& m) {
    const uint32_t type = hdr_type(m.x), opid = m.y;
    if (type != PAXISIM_MSG_GETREPLY && type != PAXISIM_MSG_SETREPLY) return false;
    if (x.l_c[op_i<NT>(P, x, opid, 0)] != opid) return true;
    const uint32_t si = op_i<NT>(P, x, opid, 2);
    const uint32_t sm = x.l_c[si];
    if (type == PAXISIM_MSG_SETREPLY) {
      if ((sm & 3u) != ABD_SET) return true;
      const uint32_t s2 = sm | ((1u << src) << 17);
      if (abd_majority<NT>(P, s2 >> 17)) return false;            // Done: the full handler
      x.l_c[si] = s2;
      return true;
    }
    if ((sm & 3u) != ABD_GET) return true;
    if (abd_majority<NT>(P, ((sm | ((1u << src) << 2)) >> 2) & 0x7FFFu)) return false;   // Set phase
    abd_handle_getreply<NT>(P, x, src, hdr_n(m.x), opid, m.z, m.w);
    return true;
  }
  // registrations abd/replica.go:42-46
  template <int NT>
  __device__ static __forceinline__ void dispatch(const Params& P, Rep<NT>& x, uint32_t src, const uint4& m,
                                                  uint32_t) {
    const uint32_t key = hdr_n(m.x);
    switch (hdr_type(m.x)) {
      case PAXISIM_MSG_REQUEST: dv_inc<NT>(x, PAXISIM_MSG_REQUEST); abd_handle_request<NT>(P, x, m.w); break;
      case PAXISIM_MSG_GET: dv_inc<NT>(x, PAXISIM_MSG_GET); abd_handle_get<NT>(P, x, src, key, m.y); break;
      case PAXISIM_MSG_GETREPLY:
        dv_inc<NT>(x, PAXISIM_MSG_GETREPLY);
        abd_handle_getreply<NT>(P, x, src, key, m.y, m.z, m.w);
        break;
      case PAXISIM_MSG_SET: dv_inc<NT>(x, PAXISIM_MSG_SET); abd_handle_set<NT>(P, x, src, key, m.y, m.z, m.w); break;
      case PAXISIM_MSG_SETREPLY: dv_inc<NT>(x, PAXISIM_MSG_SETREPLY); abd_handle_setreply<NT>(P, x, src, key, m.y); break;
      default: break;
    }
  }
};

}  // namespace pxs
