// paxisim.hip — C-ABI (include/paxisim.h) over the gfx950 simulation kernels.
//
// Product path: everything here runs on the GPU.  There is no CPU fallback;
// a handle whose device cannot be initialised fails paxisim_create with
// PAXISIM_EDEVICE.
#include <hip/hip_runtime.h>

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstdarg>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <new>
#include <utility>
#include <algorithm>
#include <vector>

#include "epaxos_kernel.h"
#include "lin_kernel.h"
#include "paxisim_dev.h"
#include "sim_core.h"
#include "step_ops.h"

using namespace pxs;

static thread_local char g_err[512];
static int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
  return code;
}
#define HIPCHK(expr)                                                                  \
  do {                                                                                \
    hipError_t e_ = (expr);                                                           \
    if (e_ != hipSuccess)                                                             \
      return fail(PAXISIM_EDEVICE, "%s failed: %s", #expr, hipGetErrorString(e_));    \
  } while (0)

struct paxisim {
  paxisim_config cfg;
  paxisim_workload wl;
  paxisim_fault_process fp;
  Params P;
  uint32_t zone_of[PAXISIM_MAX_N], node_of[PAXISIM_MAX_N];
  std::vector<DevFault> faults;
  DevFault* d_faults = nullptr;
  uint32_t* d_move = nullptr;      // moving-Mu key CDF tables (paxisim_workload.move_cdf)
  uint32_t* d_ph = nullptr;        // phase binning: class counts, region, per-block sums
  void* arena = nullptr;
  size_t arena_bytes = 0;
  uint64_t* d_scratch = nullptr;   // reductions
  hipStream_t stream = nullptr;
  StepOps ops{};
  int lds_set = -1;                // dynamic-LDS ceiling set for ops on this handle's device
  uint32_t t = 0;
  uint32_t S = 32;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> evs;
  double kernel_ms = 0;
  uint64_t launches = 0;
  // live-cluster compaction
  uint32_t* d_cmp = nullptr;       // [0] bound, [1] lnew, [2] npairs, [3] live, [4] live before lnew, then block sums
  uint32_t* d_pairs = nullptr;     // [2][C/2+64]: dead slots below lnew, live slots above it
  uint32_t cmp_every = 50;         // steps between compactions
  // pipelined serial launches (sim_core.h sim_serial_pipe): up to pipe_max chunks of S steps per launch
  uint32_t pipe_max = 4;
  uint32_t* d_pipe = nullptr;      // [0,8) tickets, [8] error, [16, 16 + max(C/64, 64)) chunks done per tile
  uint32_t last_cmp = 0;
  uint32_t late_until = 0;         // no compaction before every late worker has started
  uint32_t bound_host = 0;         // last bound read back (diagnostics)
  uint64_t lin_big = 0, lin_nmax = 0;   // last linearizability scan: partitions above LIN_SMAX, largest
};

static inline size_t rc_host(const Params& P, uint32_t r, uint64_t c) { return (size_t)r * P.C + c; }

// compressed (n << 4) | r  ->  the 64-bit Ballot of ballot.go:15-17
static uint64_t expand_ballot(const paxisim* h, uint32_t b) {
  if (!b) return 0;
  const uint32_t id = b & 15u;
  return ((uint64_t)(b >> 4) << 32) | ((uint64_t)h->zone_of[id] << 16) | h->node_of[id];
}

extern "C" int paxisim_abi_version(void) { return PAXISIM_ABI_VERSION; }
extern "C" const char* paxisim_last_error(void) { return g_err; }

// ---------------------------------------------------------------------------
// kernels: init, stats reduction, state gather, agreement scan
// ---------------------------------------------------------------------------
__global__ void init_kernel(Params P) {
  const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= P.C) return;
  const uint32_t blk = (uint32_t)(c / LANES), lane = (uint32_t)(c % LANES);
  uint8_t* img = P.image + (size_t)blk * P.img.bytes;
  P.kc[c] = cluster_key(P.seed, P.cluster_base + c);
  P.slot_of[c] = (uint32_t)c;
  P.cl_of[c] = (uint32_t)c;
  reinterpret_cast<uint32_t*>(img + P.img.off_poison)[lane] = 0xFFFFFFFFu;
  if (P.protocol == PAXISIM_PAXOS)
    for (uint32_t r = 0; r < P.N; r++) P.slot[rc(P, r, c)] = 0xFFFFFFFFu;   // slot: -1 (paxos.go:45)
  if (P.protocol == PAXISIM_WPAXOS)                                         // fresh kpaxos instances
    for (uint32_t k = 0; k < P.keys; k++)
      for (uint32_t r = 0; r < P.N; r++)
        wp_write(P, blk, k, r, lane, make_uint4(0u, 0xFFFFFFFFu, 0u, 0u), make_uint4(0u, 0u, 0u, POL_NONE));
  if (P.protocol == PAXISIM_EPAXOS) {                                      // replica.go:37-47: -1 everywhere
    for (uint32_t k = 0; k < 3 * P.N * P.N; k++) P.ep_sce[(size_t)k * P.C + c] = 0xFFFFFFFFu;
    for (uint32_t k = 0; k < P.N * P.keys * P.N; k++) P.ep_cf[(size_t)k * P.C + c] = 0xFFFFFFFFu;
    for (uint32_t k = 0; k < P.keys * P.N; k++) P.ep_max[(size_t)k * P.C + c] = 0xFFFFFFFFu;
  }
  if (c >= P.clusters) return;
  uint8_t* cnt = img + P.img.off_cnt;
  uint32_t* wcur = reinterpret_cast<uint32_t*>(img + P.img.off_wcur);
  uint32_t* wiss = reinterpret_cast<uint32_t*>(img + P.img.off_wiss);
  uint4* rec = P.rec + (size_t)blk * P.rec_per_block;
  for (uint32_t w = 0; w < P.WK; w++) {         // each worker's first request waits at step 0
    if (P.start_step[w]) continue;              // joins later (client_start, sim_core.h)
    const uint32_t box = (0u * P.N + P.target[w]) * P.NS + P.N;
    const uint32_t k = cnt[(box << 6) | lane];
    rec[((box * P.M + k) << 6) | lane] = make_uint4(PAXISIM_MSG_REQUEST, 0u, 0u, 1u + w);
    cnt[(box << 6) | lane] = (uint8_t)(k + 1u);
    wcur[(w << 6) | lane] = 1u + w;
    wiss[(w << 6) | lane] = 1u;
  }
}

constexpr int NRED = NSTAT + 8;   // counters + flagged bits

__device__ __forceinline__ uint64_t wave_sum(uint64_t v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  return v;
}

__global__ void stats_kernel(Params P, uint64_t* out) {
  const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = c < P.clusters;
  uint32_t cf = 0;
  for (int k = 0; k < NSTAT; k++) {
    uint64_t v = 0;
    if (live)
      for (uint32_t r = 0; r < P.N; r++) v += P.stats[krc(P, k, r, c)];
    v = wave_sum(v);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd((unsigned long long*)&out[k], (unsigned long long)v);
  }
  if (live)
    for (uint32_t r = 0; r < P.N; r++) cf |= P.flags[rc(P, r, c)];
  for (int b = 0; b < 8; b++) {
    uint64_t v = wave_sum((cf >> b) & 1u);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd((unsigned long long*)&out[NSTAT + b], (unsigned long long)v);
  }
}

__global__ void gather_kernel(Params P, uint64_t lo, uint64_t n, paxisim_replica_state* out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * P.N) return;
  const uint64_t c = slot_of(P, lo + i / P.N);
  const uint32_t r = (uint32_t)(i % P.N);
  const size_t j = rc(P, r, c);
  paxisim_replica_state s;
  memset(&s, 0, sizeof s);
  s.ballot = P.ballot[j];             // compressed; expanded on the host
  s.slot = (int32_t)P.slot[j];
  s.execute = (int32_t)P.execute[j];
  s.active = P.meta[j] & 1u;
  s.p1_acks = P.meta[j] >> 16;
  s.flags = P.flags[j];
  s.digest = P.digest[j];
  s.npending = P.npend[j];
  for (int k = 0; k < PAXISIM_NMSG; k++) s.delivered[k] = P.stats[krc(P, ST_DELIV0 + k, r, c)];
  s.client_requests = P.stats[krc(P, ST_CLIENT, r, c)];
  s.sent = P.stats[krc(P, ST_SENT, r, c)];
  s.dropped = P.stats[krc(P, ST_DROPPED, r, c)];
  s.discarded = P.stats[krc(P, ST_DISCARDED, r, c)];
  s.commits = P.stats[krc(P, ST_COMMITS, r, c)];
  s.replies = P.stats[krc(P, ST_REPLIES, r, c)];
  if (P.protocol == PAXISIM_ABD) {   // op counter, Done ops recorded, KV digest, live ops
    const uint8_t* img = P.image + (c / LANES) * (size_t)P.img.bytes;
    const uint32_t lane = (uint32_t)(c % LANES);
    const uint32_t* kv_val = reinterpret_cast<const uint32_t*>(img + P.img.off_a);
    const uint32_t* kv_ver = reinterpret_cast<const uint32_t*>(img + P.img.off_b);
    const uint32_t* ops = reinterpret_cast<const uint32_t*>(img + P.img.off_c);
    uint64_t d = 0;
    for (uint32_t k = 0; k < P.keys; k++) {
      const uint32_t ki = ((r * P.keys + k) << 6) | lane;
      d = mix64(d ^ (((uint64_t)kv_ver[ki] << 32) | kv_val[ki]));
    }
    uint32_t live = 0;
    for (uint32_t k = 0; k < P.OW; k++) {
      const uint32_t st = ops[(((r * P.OW + k) * ABD_OPF + 2) << 6) | lane] & 3u;
      live += st == ABD_GET || st == ABD_SET;
    }
    s.ballot = 0;
    s.active = 0;
    s.p1_acks = 0;
    s.digest = d;
    s.npending = live;
  }
  if (P.protocol == PAXISIM_EPAXOS) {   // own log head, executed prefix over all logs (paxisim.h)
    int32_t ex = 0;
    for (uint32_t o = 0; o < P.N; o++) ex += (int32_t)P.ep_sce[(((size_t)2 * P.N + o) * P.N + r) * P.C + c] + 1;
    s.ballot = 0;
    s.slot = (int32_t)P.ep_sce[(((size_t)0 * P.N + r) * P.N + r) * P.C + c];
    s.execute = ex;
    s.active = 0;
    s.p1_acks = 0;
    s.npending = 0;
  }
  if (P.protocol == PAXISIM_WPAXOS) {   // aggregate over the key instances (paxisim.h read_state)
    uint32_t hi = 0, led = 0, act = 0, ex = 0, np = 0, em = 0;
    uint64_t d = 0;
    for (uint32_t k = 0; k < P.keys; k++) {
      uint4 a, b;
      wp_read(P, c / LANES, k, r, (uint32_t)(c % LANES), a, b);
      const uint32_t exists = (a.w >> 1) & 1u;
      hi = a.x > hi ? a.x : hi;
      led += exists && ((a.w & 1u) || bal_id(a.x) == r);    // Replica.keys() replica.go:110-118
      act += a.w & 1u;
      ex += a.z;
      np += b.x;
      em |= exists << k;
      d = mix64(d ^ ((uint64_t)b.y | ((uint64_t)b.z << 32)));
    }
    s.ballot = hi;
    s.slot = (int32_t)led;
    s.execute = (int32_t)ex;
    s.active = act;
    s.p1_acks = em;
    s.npending = np;
    s.digest = d;
  }
  s.executions = P.protocol == PAXISIM_EPAXOS ? P.execute[j] : P.protocol == PAXISIM_ABD ? 0u : (uint32_t)s.execute;
  s.executed_writes = P.kv ? P.kv_ver[j] : 0u;
  out[i] = s;
}

// read_instances: one record per (cluster, replica, instance)
__global__ void gather_inst_kernel(Params P, uint64_t lo, uint64_t n, paxisim_instance_state* out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (P.protocol == PAXISIM_EPAXOS) {   // (replica, owner log): slot, executed + 1, committed + 1
    if (i >= n * P.N * P.N) return;
    const uint64_t c = slot_of(P, lo + i / (P.N * P.N));
    const uint32_t r = (uint32_t)((i / P.N) % P.N), o = (uint32_t)(i % P.N);
    paxisim_instance_state s;
    memset(&s, 0, sizeof s);
    auto sce = [&](uint32_t k) { return (int32_t)P.ep_sce[(((size_t)k * P.N + o) * P.N + r) * P.C + c]; };
    s.slot = sce(0);
    s.execute = sce(2) + 1;
    s.p1_acks = (uint32_t)(sce(1) + 1);
    s.exists = 1;
    s.policy_last = POL_NONE;
    out[i] = s;
    return;
  }
  if (i >= n * P.NI) return;
  const uint64_t c = slot_of(P, lo + i / P.NI);
  const uint32_t r = (uint32_t)((i / P.NK) % P.N), k = (uint32_t)(i % P.NK);
  paxisim_instance_state s;
  memset(&s, 0, sizeof s);
  if (P.protocol == PAXISIM_WPAXOS) {
    const size_t si = wp_si(P, c / LANES, k, r, (uint32_t)(c % LANES));
    uint4 a, b;
    wp_read(P, c / LANES, k, r, (uint32_t)(c % LANES), a, b);
    s.ballot = a.x;
    s.slot = (int32_t)a.y;
    s.execute = (int32_t)a.z;
    s.active = a.w & 1u;
    s.exists = (a.w >> 1) & 1u;
    s.p1_acks = a.w >> 16;
    s.npending = b.x;
    s.digest = (uint64_t)b.y | ((uint64_t)b.z << 32);
    s.policy_last = b.w & 0xFFu;
    s.policy_hits = (b.w >> 8) & 0xFFu;
    if (P.policy == PAXISIM_POLICY_MAJORITY) {
      const uint4 h0 = P.wpx[3 * si], h1 = P.wpx[3 * si + 1], m = P.wpx[3 * si + 2];
      const uint32_t w[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
      uint32_t h = 0x811C9DC5u;
      for (uint32_t j = 0; j < P.N; j++) h = fmix32(h ^ (((w[j >> 1] >> ((j & 1u) * 16u)) & 0xFFFFu) | j << 16));
      s.policy_state[0] = m.x;
      s.policy_state[1] = m.y;
      s.policy_state[2] = h;
    } else if (P.policy == PAXISIM_POLICY_EMA) {
      const uint4 m = P.wpx[3 * si + 2];
      s.policy_state[0] = m.x;
      s.policy_state[1] = m.y;
      s.policy_state[2] = m.z;
    }
  } else {
    const size_t j = rc(P, r, c);
    s.ballot = P.ballot[j];
    s.slot = (int32_t)P.slot[j];
    s.execute = (int32_t)P.execute[j];
    s.active = P.meta[j] & 1u;
    s.exists = 1;
    s.p1_acks = P.meta[j] >> 16;
    s.npending = P.npend[j];
    s.digest = P.digest[j];
    s.policy_last = POL_NONE;
  }
  out[i] = s;
}

// Agreement scan (client.go:279-320; tla/wpaxos.tla Safety): replicas that
// executed the same number of slots must hold the same digest, and digest
// checkpoints taken at the same executed count must agree.
__global__ void check_kernel(Params P, uint64_t* out) {
  const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t bad = 0;
  if (c < P.clusters && P.protocol != PAXISIM_EPAXOS) {   // EPaxos: no single log (paxisim.h)
    for (uint32_t r = 0; r < P.N; r++) bad |= P.stats[krc(P, ST_AGB, r, c)] != 0;   // running check (paxos_exec)
    auto exec_digest = [&](uint32_t key, uint32_t r, uint32_t& e, uint64_t& d) {
      if (P.protocol == PAXISIM_WPAXOS) {
        uint4 a, b;
        wp_read(P, c / LANES, key, r, (uint32_t)(c % LANES), a, b);
        e = a.z;
        d = (uint64_t)b.y | ((uint64_t)b.z << 32);
      } else {
        e = P.execute[rc(P, r, c)];
        d = P.digest[rc(P, r, c)];
      }
    };
    auto ck = [&](uint32_t k, uint32_t inst) { return ((size_t)k * P.NI + inst) * P.C + c; };
    for (uint32_t key = 0; key < P.NK && !bad; key++)       // per Paxos instance (WPaxos: per key)
      for (uint32_t a = 0; a < P.N && !bad; a++)
        for (uint32_t b = a + 1; b < P.N && !bad; b++) {
          uint32_t ea, eb;
          uint64_t da, db;
          exec_digest(key, a, ea, da);
          exec_digest(key, b, eb, db);
          if (ea == eb && da != db) bad = 1;
          const uint32_t ia = key * P.N + a, ib = key * P.N + b;
          for (uint32_t k = 0; k < CKR && !bad; k++) {
            const uint32_t e = P.ck_e[ck(k, ia)];
            if (!e) continue;
            for (uint32_t j = 0; j < CKR && !bad; j++)
              if (P.ck_e[ck(j, ib)] == e && P.ck_d[ck(k, ia)] != P.ck_d[ck(j, ib)]) bad = 1;
          }
        }
  }
  bad = wave_sum(bad);
  if ((threadIdx.x & 63) == 0 && bad) atomicAdd((unsigned long long*)out, (unsigned long long)bad);
}

// Pipelined launches (sim_core.h sim_serial_pipe) need the dispatcher to deal a
// launch's workgroups to 8 XCDs in turn (any rotation): each XCD's ticket queue
// then has exactly one workgroup per ticket.  This records the XCD of 64
// workgroups; create turns pipelining off when they are not dealt that way
// (another compute partition mode), rather than let chunks go unrun.
__global__ void xcc_probe(uint32_t* out) {
  if (threadIdx.x == 0) out[blockIdx.x] = __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((32 - 1) << 11));   // HW_REG_XCC_ID
}

// paxisim_inject: one client request record into (bucket b, dst r, src client)
__global__ void inject_kernel(Params P, uint64_t cl, uint32_t r, uint32_t b, uint32_t cid, uint32_t* status) {
  if (threadIdx.x != 0) return;
  const uint64_t c = slot_of(P, cl);
  const uint32_t blk = (uint32_t)(c / LANES), lane = (uint32_t)(c % LANES);
  uint8_t* cnt = P.image + (size_t)blk * P.img.bytes + P.img.off_cnt;
  const uint32_t box = (b * P.N + r) * P.NS + P.N;
  const uint32_t k = cnt[(box << 6) | lane];
  if (k >= P.M) {
    *status = 1;
    return;
  }
  P.rec[(size_t)blk * P.rec_per_block + (((box * P.M + k) << 6) | lane)] = make_uint4(PAXISIM_MSG_REQUEST, 0u, 0u, cid);
  cnt[(box << 6) | lane] = (uint8_t)(k + 1u);
  *status = 0;
}

// paxisim_read_inbox: replica r's bucket b, source by source, FIFO order
__global__ void read_inbox_kernel(Params P, uint64_t cl, uint32_t r, uint32_t b, paxisim_inbox_record* out,
                                  uint32_t cap, uint32_t* n_out) {
  if (threadIdx.x != 0) return;
  const uint64_t c = slot_of(P, cl);
  const uint32_t blk = (uint32_t)(c / LANES), lane = (uint32_t)(c % LANES);
  const uint8_t* cnt = P.image + (size_t)blk * P.img.bytes + P.img.off_cnt;
  const uint4* rec = P.rec + (size_t)blk * P.rec_per_block;
  uint32_t n = 0;
  for (uint32_t src = 0; src < P.NS; src++) {
    const uint32_t box = (b * P.N + r) * P.NS + src;
    const uint32_t k_n = cnt[(box << 6) | lane];
    for (uint32_t k = 0; k < k_n; k++, n++) {
      if (n >= cap) continue;
      const uint4 m = rec[((box * P.M + k) << 6) | lane];
      out[n] = paxisim_inbox_record{src, m.x, m.y, m.z, m.w};
    }
  }
  *n_out = n;
}

// paxisim_deliver: n records appended to (bucket b, dst r, src)
__global__ void deliver_kernel(Params P, uint64_t cl, uint32_t r, uint32_t src, uint32_t b,
                               const paxisim_inbox_record* in, uint32_t n, uint32_t* status) {
  if (threadIdx.x != 0) return;
  const uint64_t c = slot_of(P, cl);
  const uint32_t blk = (uint32_t)(c / LANES), lane = (uint32_t)(c % LANES);
  uint8_t* cnt = P.image + (size_t)blk * P.img.bytes + P.img.off_cnt;
  const uint32_t box = (b * P.N + r) * P.NS + src;
  const uint32_t k = cnt[(box << 6) | lane];
  if (k + n > P.M) {
    *status = 1;
    return;
  }
  uint4* rec = P.rec + (size_t)blk * P.rec_per_block;
  for (uint32_t i = 0; i < n; i++)
    rec[(((box * P.M + k + i) << 6) | lane)] = make_uint4(in[i].hdr, in[i].ballot, in[i].slot, in[i].cid);
  cnt[(box << 6) | lane] = (uint8_t)(k + n);
  *status = 0;
}

// paxisim_commands: the workload's key and kind of each command id
__global__ void command_kernel(Params P, uint64_t cl, const uint32_t* cids, uint32_t n, uint32_t* keys,
                               uint32_t* writes) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t kc = P.kc[slot_of(P, cl)];
  keys[i] = wl_key(P, kc, cids[i]);
  writes[i] = wl_write(P, kc, cids[i]) ? 1u : 0u;
}

// paxisim_read_log: one thread per slot of one instance's window
__global__ void read_log_kernel(Params P, uint64_t cl, uint32_t r, uint32_t key, int32_t lo, uint32_t n,
                                paxisim_log_entry* out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t c = slot_of(P, cl);
  const uint32_t blk = (uint32_t)(c / LANES), lane = (uint32_t)(c % LANES);
  const int32_t s = lo + (int32_t)i;
  paxisim_log_entry o;
  memset(&o, 0, sizeof o);
  o.slot = s;
  int32_t execute;
  uint32_t eb, ec, ea, ex;
  const uint32_t w = (uint32_t)s & (P.W - 1u);
  if (P.protocol == PAXISIM_WPAXOS) {
    const size_t si = wp_si(P, blk, key, r, lane);
    uint4 a, b;
    wp_read(P, blk, key, r, lane, a, b);
    execute = (int32_t)a.z;
    const uint32_t* e = P.wlog + si * P.wlog_str + w * 4u;
    eb = e[0]; ec = e[1]; ea = e[2]; ex = e[3];
  } else {
    execute = (int32_t)P.execute[rc(P, r, c)];
    const uint8_t* img = P.image + (size_t)blk * P.img.bytes;
    const uint32_t li = ((r * P.W + w) << 6) | lane;
    eb = reinterpret_cast<const uint32_t*>(img + P.img.off_a)[li];
    ec = reinterpret_cast<const uint32_t*>(img + P.img.off_b)[li];
    ea = reinterpret_cast<const uint32_t*>(img + P.img.off_c)[li];
    ex = P.reqx[(size_t)blk * (P.N * P.W * LANES) + li];
  }
  if (s >= execute && s < execute + (int32_t)P.W) {
    o.flags = PAXISIM_LOG_HELD;
    if (ec & EF_EXISTS) {
      o.flags |= PAXISIM_LOG_EXISTS | ((ec & EF_COMMIT) ? PAXISIM_LOG_COMMIT : 0u) |
                 ((ec & EF_QUORUM) ? PAXISIM_LOG_QUORUM : 0u) |
                 ((ec & (EF_REQSELF | EF_REQEXT)) ? PAXISIM_LOG_REQUEST : 0u);
      o.ballot = eb;                                          // compressed; expanded on the host
      o.cmd = ec & CMD_MASK;
      o.acks = ea;
      o.request = (ec & EF_REQSELF) ? ((ec & CMD_MASK) | (PAXISIM_CLIENT_SRC << 27)) : (ec & EF_REQEXT) ? ex : 0u;
    }
  }
  out[i] = o;
}


// ---------------------------------------------------------------------------
// Live-cluster compaction.  A Paxos cluster whose mailboxes
// are empty at the end of a launch is at a fixed point: Paxi has no timers or
// retries, so nothing in it changes again unless a request is injected.  Its
// only evolving state is the random fault process of its links, which no
// handler can observe while no message moves.  Every cmp_every steps the
// slots [0, bound) are partitioned so that live clusters fill whole 64-cluster
// tiles at the front: the k-th quiescent slot below lnew swaps all its state
// with the k-th live slot above it, and slots [lnew, bound) freeze (frz =
// the step they stopped at).  Workgroups past the bound exit at once, so
// launches stop paying for lanes whose clusters have died.  A request
// injected into a frozen cluster wakes its tile: the link fault process is
// replayed over the frozen steps, so the trajectory is exactly the one the
// oracle computes without any of this.
// ---------------------------------------------------------------------------
constexpr uint32_t CB = 1024;                    // slots per counting block
enum { CM_BOUND = 0, CM_LNEW, CM_NPAIRS, CM_LIVE, CM_LBL, CM_SUMS = 8 };

template <typename T>
__device__ __forceinline__ void swap_rows(T* a, size_t rows, size_t C, uint64_t p, uint64_t q, uint32_t j) {
  for (size_t k = j; k < rows; k += LANES) {
    const T v = a[k * C + p];
    a[k * C + p] = a[k * C + q];
    a[k * C + q] = v;
  }
}
// lane-fastest per-block regions: element (row, lane) of block b at base + b*bstride + row*64 + lane
template <typename T>
__device__ __forceinline__ void swap_lanes(T* base, size_t bstride, size_t rows, uint64_t p, uint64_t q, uint32_t j) {
  T* bp = base + (p / LANES) * bstride + (p % LANES);
  T* bq = base + (q / LANES) * bstride + (q % LANES);
  for (size_t k = j; k < rows; k += LANES) {
    const T v = bp[k * LANES];
    bp[k * LANES] = bq[k * LANES];
    bq[k * LANES] = v;
  }
}

// Swap every per-slot datum of the Paxos step kernel between slots p and q
// (one wave per pair, lane j takes every 64th element).  Only live data moves
// (round 5): pending / forward entries past their counts and the ghost table
// of a replica that never raised GHOST are never read before they are written
// (paxos_kernel.h), so a pair moves max(count_p, count_q) of them; the
// agreement ring is indexed by cluster id, not slot (sim_core.h agree_drain),
// and does not move at all.
static_assert(PMAX + FMAX == LANES, "swap_slots: one lane per pending / forwards entry");
__device__ void swap_slots(const Params& P, uint64_t p, uint64_t q, uint32_t j) {
  const size_t C = P.C, N = P.N;
  // live extents, read before any row moves (uniform across the wave)
  for (uint32_t r = 0; r < N; r++) {
    const size_t ip = (size_t)r * C + p, iq = (size_t)r * C + q;
    const uint32_t np0 = P.npend[ip], np1 = P.npend[iq];
    const uint32_t nf0 = P.nfwd[ip], nf1 = P.nfwd[iq];
    const bool gh = ((P.flags[ip] | P.flags[iq]) & PAXISIM_F_GHOST) != 0u;
    const uint32_t np = np0 > np1 ? np0 : np1, nf = nf0 > nf1 ? nf0 : nf1;
    // lane j < 32: pending entry j, 32 <= j < 64: forwards entry j - 32 (PMAX = FMAX = 32)
    uint32_t* a = nullptr;
    if (j < PMAX && j < np) a = P.pend + ((size_t)j * P.NI + r) * C;
    else if (j >= PMAX && j - PMAX < nf) a = P.fwd + ((size_t)(j - PMAX) * N + r) * C;
    uint32_t vp = 0, vq = 0;
    uint4 gp = make_uint4(0u, 0u, 0u, 0u), gq = gp;
    uint4* g = nullptr;
    if (gh && j < GMAX) g = P.gst + ((size_t)j * P.NI + r) * C;
    if (a) { vp = a[p]; vq = a[q]; }
    if (g) { gp = g[p]; gq = g[q]; }
    if (a) { a[p] = vq; a[q] = vp; }
    if (g) { g[p] = gq; g[q] = gp; }
  }
  swap_rows(P.ballot, 7 * N, C, p, q, j);        // ballot slot execute meta flags npend nfwd
  swap_rows(P.digest, N, C, p, q, j);
  swap_rows(P.kc, 1, C, p, q, j);
  swap_rows(P.link_drop, 2 * N * N, C, p, q, j);   // link_drop then link_slow
  swap_rows(P.ck_e, (size_t)CKR * P.NI, C, p, q, j);
  swap_rows(P.ck_d, (size_t)CKR * P.NI, C, p, q, j);
  swap_rows(P.stats, (size_t)NSTAT * N, C, p, q, j);
  swap_rows(P.kv_val, P.kv ? (size_t)P.keys * N : 0, C, p, q, j);
  swap_rows(P.kv_ver, P.kv ? N : 0, C, p, q, j);
  swap_rows(P.wrep, P.WK, C, p, q, j);
  swap_rows(P.frz, 1, C, p, q, j);
  swap_rows(P.qf, 1, C, p, q, j);
  if (P.phase_sort) swap_rows(P.phase, 1, C, p, q, j);
  swap_lanes(P.reqx, (size_t)N * P.W * LANES, (size_t)N * P.W, p, q, j);
  // LDS image: u32 rows (log window a/b/c, worker tables, poison), then u8 mailbox counts
  swap_lanes(reinterpret_cast<uint32_t*>(P.image), P.img.bytes / 4u, P.img.off_cnt / (LANES * 4u), p, q, j);
  {
    uint8_t* cp = P.image + (p / LANES) * (size_t)P.img.bytes + P.img.off_cnt + (p % LANES);
    uint8_t* cq = P.image + (q / LANES) * (size_t)P.img.bytes + P.img.off_cnt + (q % LANES);
    uint4* rp = P.rec + (p / LANES) * (size_t)P.rec_per_block + (p % LANES);
    uint4* rq = P.rec + (q / LANES) * (size_t)P.rec_per_block + (q % LANES);
    const uint32_t nbox = P.D * P.N * P.NS;
    for (uint32_t b = j; b < nbox; b += LANES) {           // records in flight, then their counts
      const uint32_t kp = cp[b * LANES], kq = cq[b * LANES];
      const uint32_t kn = kp > kq ? kp : kq;
      for (uint32_t k = 0; k < kn; k++) {
        const size_t o = (size_t)(b * P.M + k) * LANES;
        const uint4 v = rp[o];
        rp[o] = rq[o];
        rq[o] = v;
      }
      cp[b * LANES] = (uint8_t)kq;
      cq[b * LANES] = (uint8_t)kp;
    }
  }
  if (j == 0) {
    const uint32_t a = P.cl_of[p], b = P.cl_of[q];
    P.cl_of[p] = b;
    P.cl_of[q] = a;
    P.slot_of[b] = (uint32_t)p;
    P.slot_of[a] = (uint32_t)q;
  }
}

__global__ void cmp_count(Params P, uint32_t* cm) {
  const uint64_t s = (uint64_t)blockIdx.x * CB + threadIdx.x;
  const int live = s < cm[CM_BOUND] && !P.qf[s];
  const int n = __syncthreads_count(live);
  if (threadIdx.x == 0) cm[CM_SUMS + blockIdx.x] = (uint32_t)n;
}

// one workgroup of CB threads: exclusive scan of the block counts, then the
// new bound and the number of pairs to swap
__global__ void cmp_scan(Params P, uint32_t* cm, uint32_t nb) {
  __shared__ uint32_t sh[CB];
  __shared__ uint32_t carry;
  const uint32_t tid = threadIdx.x;
  if (tid == 0) carry = 0;
  __syncthreads();
  for (uint32_t base = 0; base < nb; base += CB) {
    const uint32_t v = base + tid < nb ? cm[CM_SUMS + base + tid] : 0u;
    sh[tid] = v;
    __syncthreads();
    for (uint32_t off = 1; off < CB; off <<= 1) {
      const uint32_t t = tid >= off ? sh[tid - off] : 0u;
      __syncthreads();
      sh[tid] += t;
      __syncthreads();
    }
    if (base + tid < nb) cm[CM_SUMS + base + tid] = carry + sh[tid] - v;
    __syncthreads();
    if (tid == 0) carry += sh[CB - 1];
    __syncthreads();
  }
  const uint32_t live = carry, bound = cm[CM_BOUND];
  uint32_t lnew = (live + LANES - 1u) / LANES * LANES;
  if (lnew > bound) lnew = bound;
  const uint32_t b = lnew / CB;
  const uint64_t s = (uint64_t)b * CB + tid;
  const int cnt = __syncthreads_count(s < lnew && !P.qf[s]);
  const uint32_t lbl = (b < nb ? cm[CM_SUMS + b] : live) + (uint32_t)cnt;   // live slots below lnew
  if (tid == 0) {
    cm[CM_LNEW] = lnew;
    cm[CM_LIVE] = live;
    cm[CM_LBL] = lbl;
    cm[CM_NPAIRS] = live - lbl;
  }
}

__global__ void cmp_index(Params P, uint32_t* cm, uint32_t* lo, uint32_t* hi) {
  __shared__ uint32_t wsum[CB / LANES];
  const uint64_t s = (uint64_t)blockIdx.x * CB + threadIdx.x;
  const uint32_t bound = cm[CM_BOUND], lnew = cm[CM_LNEW], lbl = cm[CM_LBL], np = cm[CM_NPAIRS];
  const bool live = s < bound && !P.qf[s];
  const uint64_t m = __ballot(live);
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  const uint32_t inw = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
  if (lane == 0) wsum[w] = (uint32_t)__popcll(m);
  __syncthreads();
  uint32_t off = 0;
  for (uint32_t k = 0; k < w; k++) off += wsum[k];
  const uint32_t before = cm[CM_SUMS + blockIdx.x] + off + inw;     // live slots in [0, s)
  if (s >= bound) return;
  if (!live && s < lnew) {
    const uint32_t k = (uint32_t)s - before;                       // dead slots in [0, s)
    if (k < np) lo[k] = (uint32_t)s;
  } else if (live && s >= lnew) {
    hi[before - lbl] = (uint32_t)s;
  }
}

__global__ void cmp_swap(Params P, const uint32_t* cm, const uint32_t* lo, const uint32_t* hi) {
  const uint32_t np = cm[CM_NPAIRS];
  for (uint32_t k = blockIdx.x; k < np; k += gridDim.x) swap_slots(P, lo[k], hi[k], threadIdx.x);
}

__global__ void cmp_freeze(Params P, uint32_t* cm, uint32_t t) {
  const uint64_t s = (uint64_t)blockIdx.x * CB + threadIdx.x;
  if (s >= cm[CM_LNEW] && s < cm[CM_BOUND]) P.frz[s] = t;
}
__global__ void cmp_setbound(uint32_t* cm) { cm[CM_BOUND] = cm[CM_LNEW]; }

__global__ void swap_one(Params P, uint64_t p, uint64_t q) { swap_slots(P, p, q, threadIdx.x); }

// ---------------------------------------------------------------------------
// Phase binning.  After the live/dead partition, the stepped
// slots [0, bound) are grouped by class - the phase residue each live cluster
// was busiest at in the last launch, then the quiescent slots - with the same
// pair swaps: pass p moves every class-p slot into the region [base_p, end_p)
// by swapping the k-th misplaced slot inside it with the k-th class-p slot
// beyond it.  Slots that kept their phase stay where they are, so a pass costs
// the clusters whose phase drifted.
// ---------------------------------------------------------------------------
enum { PH_N = 0, PH_BASE = 8, PH_END = 9, PH_SUMS = 16 };   // PH_N + class: classes 0..period (quiescent last)
__device__ __forceinline__ uint32_t ph_class(const Params& P, uint64_t s) {
  return P.qf[s] ? P.phase_period : P.phase[s];
}
__global__ void ph_classes(Params P, const uint32_t* cm, uint32_t* ph) {
  const uint64_t s = (uint64_t)blockIdx.x * CB + threadIdx.x;
  const uint32_t bound = cm[CM_BOUND];
  const uint32_t c = s < bound ? ph_class(P, s) : 0xFFu;
  for (uint32_t k = 0; k <= P.phase_period; k++) {
    const int n = __syncthreads_count(c == k);
    if (threadIdx.x == 0 && n) atomicAdd(&ph[PH_N + k], (uint32_t)n);
  }
}
// region of class p: [sum of classes < p, + count of p)
__global__ void ph_region(uint32_t* ph, uint32_t p) {
  uint32_t b = 0;
  for (uint32_t k = 0; k < p; k++) b += ph[PH_N + k];
  ph[PH_BASE] = b;
  ph[PH_END] = b + ph[PH_N + p];
}
// per block: misplaced slots inside the region (class != p) and class-p slots beyond it
__global__ void ph_count(Params P, const uint32_t* cm, uint32_t* ph, uint32_t p, uint32_t nb) {
  const uint64_t s = (uint64_t)blockIdx.x * CB + threadIdx.x;
  const uint32_t bound = cm[CM_BOUND], base = ph[PH_BASE], end = ph[PH_END];
  const uint32_t c = s < bound ? ph_class(P, s) : 0xFFu;
  const int in = __syncthreads_count(s >= base && s < end && c != p);
  const int out = __syncthreads_count(s >= end && s < bound && c == p);
  if (threadIdx.x == 0) {
    ph[PH_SUMS + blockIdx.x] = (uint32_t)in;
    ph[PH_SUMS + nb + blockIdx.x] = (uint32_t)out;
  }
}
// exclusive scans of both count arrays (one workgroup); the pair count to cm
__global__ void ph_scan(uint32_t* cm, uint32_t* ph, uint32_t nb) {
  __shared__ uint32_t sh[CB];
  __shared__ uint32_t carry;
  const uint32_t tid = threadIdx.x;
  for (uint32_t a = 0; a < 2; a++) {
    uint32_t* arr = ph + PH_SUMS + a * nb;
    if (tid == 0) carry = 0;
    __syncthreads();
    for (uint32_t base = 0; base < nb; base += CB) {
      const uint32_t v = base + tid < nb ? arr[base + tid] : 0u;
      sh[tid] = v;
      __syncthreads();
      for (uint32_t off = 1; off < CB; off <<= 1) {
        const uint32_t t = tid >= off ? sh[tid - off] : 0u;
        __syncthreads();
        sh[tid] += t;
        __syncthreads();
      }
      if (base + tid < nb) arr[base + tid] = carry + sh[tid] - v;
      __syncthreads();
      if (tid == 0) carry += sh[CB - 1];
      __syncthreads();
    }
    if (a == 0 && tid == 0) cm[CM_NPAIRS] = carry;   // misplaced inside = class-p outside
  }
}
__global__ void ph_index(Params P, const uint32_t* cm, const uint32_t* ph, uint32_t p, uint32_t nb, uint32_t* lo,
                         uint32_t* hi) {
  __shared__ uint32_t wa[CB / LANES], wb[CB / LANES];
  const uint64_t s = (uint64_t)blockIdx.x * CB + threadIdx.x;
  const uint32_t bound = cm[CM_BOUND], base = ph[PH_BASE], end = ph[PH_END];
  const uint32_t c = s < bound ? ph_class(P, s) : 0xFFu;
  const bool in = s >= base && s < end && c != p, out = s >= end && s < bound && c == p;
  const uint64_t ma = __ballot(in), mb = __ballot(out);
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  if (lane == 0) { wa[w] = (uint32_t)__popcll(ma); wb[w] = (uint32_t)__popcll(mb); }
  __syncthreads();
  uint32_t oa = 0, ob = 0;
  for (uint32_t k = 0; k < w; k++) { oa += wa[k]; ob += wb[k]; }
  const uint64_t below = (1ull << lane) - 1ull;
  if (in) lo[ph[PH_SUMS + blockIdx.x] + oa + (uint32_t)__popcll(ma & below)] = (uint32_t)s;
  if (out) hi[ph[PH_SUMS + nb + blockIdx.x] + ob + (uint32_t)__popcll(mb & below)] = (uint32_t)s;
}

// Wake: the link fault process of slots [s0, s1) over the steps they were frozen
__global__ void replay_kernel(Params P, uint64_t s0, uint64_t s1, uint32_t tnow) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t c = s0 + i / P.N;
  if (c >= s1) return;
  Rep<0> x;
  x.r = (uint32_t)(i % P.N);
  x.c = c;
  x.kc = P.kc[c];
  const uint32_t poison =
      reinterpret_cast<const uint32_t*>(P.image + (c / LANES) * (size_t)P.img.bytes + P.img.off_poison)[c % LANES];
  uint32_t du[Rep<0>::NL], su[Rep<0>::NL];
  for (uint32_t d = 0; d < Rep<0>::NL; d++) {
    du[d] = d < P.N ? P.link_drop[krc(P, d, x.r, c)] : 0u;
    su[d] = d < P.N ? P.link_slow[krc(P, d, x.r, c)] : 0u;
  }
  for (uint32_t t = P.frz[c]; t < tnow && t <= poison; t++) {   // the step kernel's gate: poison >= t
    x.t = t;
    x.hs = step_key(x.kc, t);
    fault_process<0>(P, x, du, su);
  }
}

// ---------------------------------------------------------------------------
// C-ABI
// ---------------------------------------------------------------------------
static Image proto_image(uint32_t protocol, uint32_t N, uint32_t W, uint32_t K, uint32_t WK, uint32_t D,
                         uint32_t wlds) {
  if (protocol == PAXISIM_ABD) {
    const uint32_t kv = N * K * LANES * 4u;
    return image_layout(kv, kv, N * abd_ow(WK) * ABD_OPF * LANES * 4u, N, WK, D);
  }
  if (protocol == PAXISIM_WPAXOS)   // instance scalars in the image (wlds), or all in HBM
    return image_layout(wlds ? K * N * WP_WORDS * LANES * 4u : 0u, 0, 0, N, WK, D);
  if (protocol == PAXISIM_EPAXOS) return image_layout(0, 0, 0, N, WK, D);   // state in HBM
  const uint32_t logb = N * W * LANES * 4u;
  return image_layout(logb, logb, logb, N, WK, D);
}

// The serial kernel (one wave per tile plays every replica, sim_core.h
// sim_serial) for the protocols that have it; PAXISIM_SERIAL=0/1 overrides
// (A/B).  Any other value is refused (serial_env_ok), so an A/B arm cannot
// silently measure the default kernel.
static bool serial_env_ok() {
  const char* e = getenv("PAXISIM_SERIAL");
  return !e || !strcmp(e, "0") || !strcmp(e, "1");
}
static bool serial_for(uint32_t protocol) {
  const char* e = getenv("PAXISIM_SERIAL");
  (void)protocol;
  return !e || strcmp(e, "0") != 0;
}

// The workload's key space (paxisim.h): ORDER / UNIFORM / CONFLICT range over
// key_space indices; CONFLICT's literal key 0 is its own index when key_min != 0.
static uint32_t key_space_of(const paxisim_config* cfg, const paxisim_workload* wl) {
  const uint32_t keys = cfg->keys ? cfg->keys : 1u;
  return wl->key_space ? wl->key_space : keys;
}
static int check_keys(const paxisim_config* cfg, const paxisim_workload* wl) {
  const uint32_t keys = cfg->keys ? cfg->keys : 1u;
  const uint32_t ks = key_space_of(cfg, wl);
  if (ks > keys) return fail(PAXISIM_EINVAL, "key_space %u exceeds keys %u", ks, keys);
  if (wl->distribution == PAXISIM_DIST_CONFLICT && wl->key_min && ks >= keys)
    return fail(PAXISIM_EINVAL, "conflict with key_min != 0 needs key_space < keys (literal key 0 has its own index)");
  if (wl->distribution == PAXISIM_DIST_TABLE) {
    for (uint32_t k = 1; k + 1u < keys; k++)
      if (wl->key_cdf[k] < wl->key_cdf[k - 1]) return fail(PAXISIM_EINVAL, "key_cdf must be non-decreasing");
    if (wl->key_tail && keys >= 2 && wl->key_tail < wl->key_cdf[keys - 2])
      return fail(PAXISIM_EINVAL, "key_tail below the last key_cdf threshold");
  } else if (wl->key_tail) {
    return fail(PAXISIM_EINVAL, "key_tail needs a table distribution");
  }
  if (wl->move_every) {
    if (wl->distribution != PAXISIM_DIST_TABLE) return fail(PAXISIM_EINVAL, "move_every needs a table distribution");
    if (!wl->move_cdf || wl->move_tables < 1 || wl->move_loop >= wl->move_tables)
      return fail(PAXISIM_EINVAL, "move_cdf / move_tables / move_loop");
    for (uint32_t e = 0; e < wl->move_tables; e++)
      for (uint32_t k = 1; k + 1u < keys; k++)
        if (wl->move_cdf[e * PAXISIM_MAX_KEYS + k] < wl->move_cdf[e * PAXISIM_MAX_KEYS + k - 1])
          return fail(PAXISIM_EINVAL, "move_cdf table %u must be non-decreasing", e);
  }
  return 0;
}

static int check_config(const paxisim_config* cfg, const paxisim_workload* wl, const paxisim_fault_process* fp,
                        uint32_t* N_out) {
  uint32_t N = 0;
  if (cfg->protocol > PAXISIM_EPAXOS || cfg->protocol == PAXISIM_M2PAXOS || cfg->protocol == PAXISIM_KPAXOS)
    return fail(PAXISIM_EUNSUPP, "protocol %u not built", cfg->protocol);
  if (cfg->protocol == PAXISIM_EPAXOS && (cfg->keys < 1 || cfg->keys > 32))
    return fail(PAXISIM_EINVAL, "EPaxos keys must be in [1,32]");
  if (cfg->protocol == PAXISIM_ABD && (cfg->keys < 1 || cfg->keys > 64)) return fail(PAXISIM_EINVAL, "keys");
  if (cfg->protocol == PAXISIM_WPAXOS && (cfg->keys < 1 || cfg->keys > 32))
    return fail(PAXISIM_EINVAL, "WPaxos keys must be in [1,32]");
  if (cfg->policy_threshold > 255) return fail(PAXISIM_EINVAL, "policy_threshold");
  if (cfg->policy > PAXISIM_POLICY_EMA) return fail(PAXISIM_EINVAL, "policy %u", cfg->policy);
  if (cfg->policy == PAXISIM_POLICY_MAJORITY && cfg->policy_interval < 1) return fail(PAXISIM_EINVAL, "policy_interval");
  if (cfg->policy == PAXISIM_POLICY_EMA && !(cfg->policy_alpha > 0.0 && cfg->policy_alpha <= 1.0))
    return fail(PAXISIM_EINVAL, "policy_alpha must be in (0, 1]");
  if (cfg->n_zones < 1 || cfg->n_zones > PAXISIM_MAX_ZONES) return fail(PAXISIM_EINVAL, "n_zones");
  for (uint32_t z = 0; z < cfg->n_zones; z++) {
    if (cfg->npz[z] < 1) return fail(PAXISIM_EINVAL, "npz[%u] must be >= 1", z);
    N += cfg->npz[z];
  }
  if (N < 1 || N > PAXISIM_MAX_N) return fail(PAXISIM_EINVAL, "N=%u out of range", N);
  if (cfg->protocol == PAXISIM_ABD && N > 15) return fail(PAXISIM_EINVAL, "ABD supports N <= 15");
  if (cfg->protocol == PAXISIM_EPAXOS && N > EP_NMAX) return fail(PAXISIM_EINVAL, "EPaxos supports N <= %u", EP_NMAX);
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
  if (int rc = check_keys(cfg, wl)) return rc;
  if (!serial_env_ok()) return fail(PAXISIM_EINVAL, "PAXISIM_SERIAL must be 0 or 1");
  for (uint32_t w = 0; w < wl->outstanding; w++)
    if (wl->target[w] >= N) return fail(PAXISIM_EINVAL, "target[%u]", w);
  if (fp->slow_ppm && (fp->slow_min > fp->slow_max || fp->slow_max > cfg->max_delay))
    return fail(PAXISIM_EINVAL, "slow delay range exceeds max_delay");
  const Image img = proto_image(cfg->protocol, N, cfg->window, cfg->keys, wl->outstanding, cfg->max_delay + 2u, 0);
  // the serial kernel keeps only the image's tail (client tables on) in LDS;
  // either kernel adds the agreement-ring arrival counts after the image
  const bool ring = cfg->protocol != PAXISIM_ABD && cfg->protocol != PAXISIM_EPAXOS;
  const uint32_t agn = ring ? (2u * N * LANES + 15u) & ~15u : 0u;
  if ((serial_for(cfg->protocol) ? img.bytes - img.off_wcur : img.bytes) + agn > LDS_MAX)
    return fail(PAXISIM_EUNSUPP, "workgroup image %u B exceeds LDS (%u B): reduce window/max_delay/replicas",
                img.bytes, LDS_MAX);
  *N_out = N;
  return 0;
}

template <typename T>
static T* carve(char*& p, size_t count) {
  T* out = reinterpret_cast<T*>(p);
  p += (count * sizeof(T) + 255) & ~size_t(255);
  return out;
}

static int pipe_check(paxisim* h);
static int flush_events(paxisim* h) {
  const bool any = !h->evs.empty();
  for (auto& e : h->evs) {
    float ms = 0;
    HIPCHK(hipEventSynchronize(e.second));
    HIPCHK(hipEventElapsedTime(&ms, e.first, e.second));
    h->kernel_ms += ms;
    (void)hipEventDestroy(e.first);
    (void)hipEventDestroy(e.second);
  }
  h->evs.clear();
  // after the waits: the error word is read once every timed launch has ended
  return any ? pipe_check(h) : 0;
}

extern "C" int paxisim_destroy(paxisim* h) {
  if (!h) return 0;
  (void)hipSetDevice(h->cfg.device);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  flush_events(h);
  if (h->arena) (void)hipFree(h->arena);
  if (h->d_faults) (void)hipFree(h->d_faults);
  if (h->d_move) (void)hipFree(h->d_move);
  if (h->d_ph) (void)hipFree(h->d_ph);
  if (h->d_scratch) (void)hipFree(h->d_scratch);
  if (h->d_cmp) (void)hipFree(h->d_cmp);
  if (h->d_pairs) (void)hipFree(h->d_pairs);
  if (h->d_pipe) (void)hipFree(h->d_pipe);
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
  return 0;
}

static StepOps step_ops_for(uint32_t protocol, uint32_t N, bool wlds, bool serial) {
  if (serial) {
    if (protocol == PAXISIM_WPAXOS) return wpaxos_serial_step_ops(N, wlds);
    if (protocol == PAXISIM_ABD) return abd_serial_step_ops(N);
    if (protocol == PAXISIM_EPAXOS) return epaxos_serial_step_ops(N);
    return paxos_serial_step_ops(N);
  }
  if (protocol == PAXISIM_WPAXOS) return wpaxos_step_ops(N, wlds);
  if (protocol == PAXISIM_ABD) return abd_step_ops(N);
  if (protocol == PAXISIM_EPAXOS) return epaxos_step_ops(N);
  return paxos_step_ops(N);
}

extern "C" int paxisim_create(const paxisim_config* cfg, const paxisim_workload* wl, const paxisim_fault_process* fp,
                              paxisim** out) {
  if (!cfg || !wl || !out) return fail(PAXISIM_EINVAL, "null argument");
  // M2Paxos and KPaxos are per-key Paxos like WPaxos: same kernel and state, a
  // different request path and quorums (P.variant)
  paxisim_config ncfg = *cfg;
  const uint32_t variant = cfg->protocol;
  if (variant == PAXISIM_M2PAXOS || variant == PAXISIM_KPAXOS) ncfg.protocol = PAXISIM_WPAXOS;
  cfg = &ncfg;
  paxisim_fault_process nofp;
  memset(&nofp, 0, sizeof nofp);
  if (!fp) fp = &nofp;
  uint32_t N = 0;
  int rc0 = check_config(cfg, wl, fp, &N);
  if (rc0) return rc0;
  int ndev = 0;
  HIPCHK(hipGetDeviceCount(&ndev));
  if (cfg->device < 0 || cfg->device >= ndev) return fail(PAXISIM_EDEVICE, "device %d not present (%d visible)", cfg->device, ndev);
  HIPCHK(hipSetDevice(cfg->device));

  paxisim* h = new (std::nothrow) paxisim();
  if (!h) return fail(PAXISIM_ENOMEM, "oom");
  h->cfg = *cfg;
  h->wl = *wl;
  h->fp = *fp;
  h->S = cfg->steps_per_launch ? cfg->steps_per_launch : 32;
  {   // per-type delivered counts are 16-bit in the kernel: at most NS*M messages per replica-step
    const uint32_t smax = 65535u / ((N + 1u) * cfg->mbox_cap);
    if (h->S > smax) h->S = smax;
  }
  Params& P = h->P;
  memset(&P, 0, sizeof P);
  P.protocol = cfg->protocol;
  P.N = N;
  P.Z = cfg->n_zones;
  P.keys = cfg->keys ? cfg->keys : 1;
  P.write_ppm = wl->write_ppm;
  P.locality_ppm = wl->locality_ppm;
  P.dist = wl->distribution;
  P.conflicts = wl->conflicts;
  memcpy(P.key_cdf, wl->key_cdf, sizeof P.key_cdf);
  P.NK = cfg->protocol == PAXISIM_WPAXOS ? P.keys : 1u;
  P.NI = P.NK * N;
  P.adaptive = cfg->adaptive;
  P.policy_thr = cfg->policy_threshold;
  P.policy = cfg->policy;
  P.policy_interval = cfg->policy_interval;
  P.policy_alpha = cfg->policy_alpha;
  P.H = cfg->protocol == PAXISIM_ABD ? cfg->history : 0;
  P.AR = (cfg->protocol == PAXISIM_ABD || cfg->protocol == PAXISIM_EPAXOS) ? 0u
         : cfg->agree_ring ? cfg->agree_ring : (cfg->protocol == PAXISIM_WPAXOS ? 128u : 1024u);
  P.OW = abd_ow(wl->outstanding);
  P.W = cfg->window;
  P.M = cfg->mbox_cap;
  P.D = cfg->max_delay + 2u;
  P.NS = N + 1u;
  P.WK = wl->outstanding;
  P.wk_magic = 0xFFFFFFFFu / P.WK;
  P.max_requests = wl->max_requests;
  P.clusters = cfg->clusters;
  P.cluster_base = cfg->cluster_base;
  P.seed = cfg->seed;
  P.q1 = cfg->q1;
  P.q2 = cfg->q2;
  P.fz = cfg->fz;
  P.thrifty = cfg->thrifty;
  P.ephemeral = cfg->ephemeral_leader;
  P.rwc = cfg->reply_when_commit;
  if (cfg->protocol == PAXISIM_WPAXOS) {
    // kpaxos: Q1/Q2 from fz (wpaxos/kpaxos.go:15-27); no ReplyWhenCommit option
    // (kpaxos.go:35-39); the Paxos replica's -ephemeral_leader is not consulted
    P.q1 = cfg->fz ? PAXISIM_Q_FGRID_Q1 : PAXISIM_Q_GRID_ROW;
    P.q2 = cfg->fz ? PAXISIM_Q_FGRID_Q2 : PAXISIM_Q_GRID_COLUMN;
    P.rwc = 0;
    P.ephemeral = 0;
  }
  P.variant = cfg->protocol == PAXISIM_WPAXOS ? variant : cfg->protocol;
  if (P.variant == PAXISIM_M2PAXOS || P.variant == PAXISIM_KPAXOS) {   // m2paxos/kpaxos.go:15-21; paxos.NewPaxos default
    P.q1 = PAXISIM_Q_MAJORITY;
    P.q2 = PAXISIM_Q_MAJORITY;
  }
  if (P.variant == PAXISIM_M2PAXOS) P.adaptive = 1;
  P.key_min = wl->key_min;
  P.kspace = key_space_of(cfg, wl);
  P.kspace_magic = 0xFFFFFFFFu / P.kspace;
  P.conflict_key = wl->key_min ? P.kspace : 0u;
  P.key_tail = wl->distribution == PAXISIM_DIST_TABLE ? wl->key_tail : 0u;
  P.move_every = wl->move_every;
  P.move_tables = wl->move_every ? wl->move_tables : 0u;
  P.move_loop = wl->move_every ? wl->move_loop : 0u;
  P.kv = cfg->protocol != PAXISIM_ABD && cfg->kv ? 1u : 0u;   // m2paxos/replica.go:34-52 has no -adaptive switch
  P.max_delay = cfg->max_delay;
  P.drop_ppm = fp->drop_ppm;
  P.drop_len = fp->drop_len;
  P.slow_ppm = fp->slow_ppm;
  P.slow_len = fp->slow_len;
  P.slow_min = fp->slow_min;
  P.slow_max = fp->slow_max;
  uint32_t r = 0;
  for (uint32_t z = 0; z < P.Z; z++) {
    P.npz[z] = cfg->npz[z];
    P.zmask[z] = ((1u << cfg->npz[z]) - 1u) << r;
    for (uint32_t k = 0; k < cfg->npz[z]; k++, r++) {
      P.zone_of[r] = z;
      h->zone_of[r] = z + 1;
      h->node_of[r] = k + 1;
    }
    P.zfirst[z] = r - cfg->npz[z];
  }
  for (uint32_t w = 0; w < PAXISIM_MAX_WORKERS; w++) {
    P.target[w] = wl->target[w];
    P.start_step[w] = w < wl->outstanding ? wl->start_step[w] : 0u;
    if (P.start_step[w]) P.late_workers |= 1u << w;
  }

  P.keys_magic = 0xFFFFFFFFu / P.keys;
  for (uint32_t w = 0; w < PAXISIM_MAX_WORKERS; w++) {
    const uint32_t z = w < P.WK ? P.zone_of[P.target[w] < N ? P.target[w] : 0u] : 0u;
    P.wzone[w] = z;
    P.wnk[w] = z < P.keys ? (P.keys - z + P.Z - 1u) / P.Z : 0u;
    P.wnk_magic[w] = P.wnk[w] ? 0xFFFFFFFFu / P.wnk[w] : 0u;
  }
  // WPaxos: the instance scalars move into the tile image when one tile's
  // image (and the agreement counts) fits the LDS; PAXISIM_WLDS=0 keeps them in HBM (A/B)
  if (P.protocol == PAXISIM_WPAXOS) {
    // The serial kernel keeps the image in HBM, where the packed 32-B table
    // (wst, one line per bind) moves 0.67x the bytes of the image's word
    // planes at the same speed (A/B r4, config 5: 267 vs 400 GB per launch,
    // profiles/r4/config5_layout.json); PAXISIM_WLDS=0/1 overrides (A/B).
    const char* ev = getenv("PAXISIM_WLDS");
    const uint32_t agn = P.AR ? (2u * N * LANES + 15u) & ~15u : 0u;
    const bool ser = serial_for(P.protocol);
    P.wlds = (ev ? atoi(ev) != 0 : !ser) &&
             (ser || proto_image(P.protocol, N, P.W, P.keys, P.WK, P.D, 1).bytes + agn <= LDS_MAX);
    // Each instance's 32-B scalars and its window in one block of whole lines: a
    // layout only, the kernels address both through wst_str / wlog_str.  On by default at W = 8, where
    // six of the eight entries share the line the bind loads (mirrored A/B r6g2, config 5: +4.2% over
    // the packed table at W = 8); at W = 16 it is 6% slower (r6g1).  PAXISIM_WCOLOC=0/1 overrides.
    const char* cv = getenv("PAXISIM_WCOLOC");
    P.wcoloc = !P.wlds && (cv ? atoi(cv) != 0 : P.W == 8u);
  }
  P.img = proto_image(P.protocol, N, P.W, P.keys, P.WK, P.D, P.wlds);
  {
    // Cluster groups per workgroup (sim_core.h): as many 64-cluster tiles as
    // the step kernel's registers leave wave slots for on every SIMD
    // (ceil(G*N/4) <= waves per SIMD) and the LDS holds, at most 4.
    int vgprs = 0, maxthr = 0;
    const bool serial = serial_for(P.protocol);
    h->ops = step_ops_for(P.protocol, N, P.wlds != 0, serial);
    if (h->ops.attrs(&vgprs, &maxthr) != hipSuccess || vgprs <= 0) vgprs = 512;
    if (maxthr <= 0) maxthr = (int)(N * LANES);
    const uint32_t alloc = ((uint32_t)vgprs + 7u) / 8u * 8u;
    const uint32_t wps = alloc >= 512u ? 1u : (512u / alloc < 8u ? 512u / alloc : 8u);
    // per tile: the image, the agreement-ring arrival counts (not persisted:
    // drained every step), then the stage
    const uint32_t agn = P.AR ? (2u * N * LANES + 15u) & ~15u : 0u;
    const uint32_t base = P.img.bytes + agn;
    uint32_t G = 1, gmax = 4;
    if (const char* e = getenv("PAXISIM_GROUPS")) gmax = (uint32_t)atoi(e) ? (uint32_t)atoi(e) : 1u;   // tuning
    for (uint32_t g = 2; g <= gmax; g++)
      if ((g * N + 3u) / 4u <= wps && g * N * LANES <= (uint32_t)maxthr && g * base <= LDS_MAX) G = g;
    P.G = G;
    // LDS stage for the first J picks of every replica's step, from what the groups leave
    uint32_t jmax = 16;
    if (const char* e = getenv("PAXISIM_STAGE")) jmax = (uint32_t)atoi(e);   // tuning override
    const uint32_t room = LDS_MAX / G > base ? (LDS_MAX / G - base) / (N * LANES * 16u) : 0u;
    P.J = room < jmax ? room : jmax;
    if (!h->ops.staged) P.J = 0;   // that instance has no staged loop
    P.off_agn = P.img.bytes;
    P.off_stage = base;
    P.lds_bytes = base + P.J * N * LANES * 16u;
    if (serial) {   // one tile per workgroup; LDS: the image tail and the arrival counts
      P.G = 1;
      P.J = 0;
      P.lds_tail = PXS_CLIENT_LDS ? P.img.off_wcur : P.img.off_poison;
      P.lds_bytes = base - P.lds_tail;
      if (PXS_WP_SCRATCH && P.protocol == PAXISIM_WPAXOS && P.wlds) {   // the replica-step instance scratch (wpaxos_kernel.h)
        P.off_wscr = base;
        P.lds_bytes += P.keys * WP_WORDS * LANES * 4u;
      }
      // phase binning (Paxos, with compaction): per-residue record counts after the rest
      const char* pe = getenv("PAXISIM_PHASE_SORT");
      const char* pp = getenv("PAXISIM_PHASE_PERIOD");
      const char* ce = getenv("PAXISIM_COMPACT");
      if (P.protocol == PAXISIM_PAXOS && !(ce && atoi(ce) == 0) && (pe ? atoi(pe) != 0 : PXS_PHASE_SORT)) {
        P.phase_period = pp ? (uint32_t)atoi(pp) : 3u;
        if (P.phase_period < 2u || P.phase_period > 7u) { delete h; return fail(PAXISIM_EINVAL, "PAXISIM_PHASE_PERIOD in [2,7]"); }
        P.ph_rel = P.lds_tail + P.lds_bytes - P.img.off_cnt;
        P.lds_bytes += P.phase_period * LANES * 4u;
        P.phase_sort = 1;
      }
      // check_config bounds the image tail and the arrival counts; the phase
      // counts come on top of them: refuse here, not at the first launch
      if (P.lds_bytes > LDS_MAX) {
        const uint32_t b = P.lds_bytes;
        delete h;
        return fail(PAXISIM_EUNSUPP, "serial LDS %u B (image tail, arrival and phase counts) exceeds LDS (%u B): "
                    "reduce window/max_delay/replicas or set PAXISIM_PHASE_SORT=0", b, LDS_MAX);
      }
    }
  }
  P.C = (cfg->clusters + LANES * P.G - 1) / (LANES * P.G) * (LANES * P.G);
  const size_t C = P.C, NC = (size_t)N * C, NIC = (size_t)P.NI * C, blocks = C / LANES;
  const bool wp = P.protocol == PAXISIM_WPAXOS;
  P.rec_per_block = P.D * N * P.NS * P.M * LANES;
  // size the arena (rec last: it is the only region not zeroed)
  size_t zero_bytes = 0, total = 0;
  auto layout = [&](char* p, bool assign) {
    uint32_t* s7 = carve<uint32_t>(p, NC * 7);
    uint64_t* dg = carve<uint64_t>(p, NC);
    uint32_t* kc = carve<uint32_t>(p, C);
    uint32_t* pend = carve<uint32_t>(p, wp ? 0 : NC * PMAX);
    uint32_t* fwd = carve<uint32_t>(p, NC * FMAX);
    uint32_t* links = carve<uint32_t>(p, NC * N * 2);
    uint32_t* cke = carve<uint32_t>(p, NIC * CKR);
    uint64_t* ckd = carve<uint64_t>(p, NIC * CKR);
    uint4* gst = carve<uint4>(p, NIC * GMAX);
    uint32_t* st = carve<uint32_t>(p, NC * NSTAT);
    uint32_t* reqx = carve<uint32_t>(p, wp ? 0 : NC * P.W);
    // WPaxos instances: the scalars table and the windows apart, or (wcoloc) one block per instance
    // holding both - 32 B of scalars, then the window - padded to whole 128-B lines, so the entries
    // at the window's head share the line the bind loads
    const bool coloc = wp && !P.wlds && P.wcoloc;
    const size_t wblk_b = ((32u + 16u * P.W) + 127u) & ~size_t(127);
    uint4* wblk = carve<uint4>(p, coloc ? NIC * (wblk_b / 16u) : 0);
    uint4* wst = carve<uint4>(p, wp && !P.wlds && !coloc ? NIC * 2 : 0);
    uint64_t* wdig = carve<uint64_t>(p, wp && P.wlds ? NIC : 0);
    uint32_t* wlog = carve<uint32_t>(p, wp && !coloc ? NIC * P.W * 4 : 0);
    if (coloc) {
      wst = wblk;
      wlog = reinterpret_cast<uint32_t*>(wblk) + 8;
    }
    uint32_t* wpend = carve<uint32_t>(p, wp ? NIC * PMAX : 0);
    uint4* wpx = carve<uint4>(p, wp && cfg->policy != PAXISIM_POLICY_CONSECUTIVE ? NIC * 3 : 0);
    uint4* hist = carve<uint4>(p, NC * P.H);
    uint32_t* maps = carve<uint32_t>(p, C * 4);
    uint32_t* phs = carve<uint32_t>(p, C);
    unsigned long long* agr = carve<unsigned long long>(p, (size_t)P.AR * P.NK * C);
    uint4* agq = carve<uint4>(p, P.AR ? (size_t)2 * AGMAX * N * C : 0);
    const bool ep = P.protocol == PAXISIM_EPAXOS;
    uint4* ep_inst = carve<uint4>(p, ep ? (size_t)N * N * P.W * C * 4 : 0);
    uint32_t* ep_sce = carve<uint32_t>(p, ep ? (size_t)3 * N * N * C : 0);
    uint32_t* ep_cf = carve<uint32_t>(p, ep ? (size_t)2 * N * P.keys * N * C : 0);
    uint32_t* ep_max = carve<uint32_t>(p, ep ? (size_t)P.keys * N * C : 0);
    uint32_t* kv_val = carve<uint32_t>(p, P.kv ? (size_t)P.keys * N * C : 0);
    uint32_t* kv_ver = carve<uint32_t>(p, P.kv ? (size_t)N * C : 0);
    uint32_t* wrep = carve<uint32_t>(p, (size_t)P.WK * C);
    uint8_t* image = carve<uint8_t>(p, blocks * P.img.bytes);
    char* zend = p;
    uint4* rec = carve<uint4>(p, blocks * P.rec_per_block);
    if (assign) {
      P.ballot = s7; P.slot = s7 + NC; P.execute = s7 + 2 * NC; P.meta = s7 + 3 * NC;
      P.flags = s7 + 4 * NC; P.npend = s7 + 5 * NC; P.nfwd = s7 + 6 * NC;
      P.digest = dg; P.kc = kc; P.pend = pend; P.fwd = fwd;
      P.link_drop = links; P.link_slow = links + NC * N;
      P.ck_e = cke; P.ck_d = ckd; P.stats = st; P.reqx = reqx; P.hist = hist; P.image = image; P.rec = rec;
      P.wst = wst; P.wdig = wdig; P.wlog = wlog; P.wpend = wpend; P.gst = gst; P.wpx = wpx;
      P.wst_str = coloc ? (uint32_t)(wblk_b / 16u) : 2u;
      P.wlog_str = coloc ? (uint32_t)(wblk_b / 4u) : P.W * 4u;
      P.slot_of = maps; P.cl_of = maps + C; P.frz = maps + 2 * C; P.qf = maps + 3 * C;
      P.phase = phs;
      P.agr = agr;
      P.agq = agq;
      P.ep_inst = ep_inst; P.ep_sce = ep_sce; P.ep_cf = ep_cf; P.ep_max = ep_max;
      P.kv_val = kv_val; P.kv_ver = kv_ver; P.wrep = wrep;
    }
    return std::make_pair((size_t)zend, (size_t)p);
  };
  {
    auto sz = layout(nullptr, false);
    zero_bytes = sz.first;
    total = sz.second;
  }
  // Arena placement experiments (the two run modes): PAXISIM_ARENA_PAD_MB
  // reserves that much device memory first and frees it once the arena is placed;
  // PAXISIM_ARENA_CONTIG=1 asks for physically contiguous memory.  Placement only.
  void* pad = nullptr;
  if (const char* ev = getenv("PAXISIM_ARENA_PAD_MB"))
    if (atoll(ev) > 0) (void)hipMalloc(&pad, (size_t)atoll(ev) << 20);
  const char* cev = getenv("PAXISIM_ARENA_CONTIG");
  hipError_t e = cev && atoi(cev) ? hipExtMallocWithFlags(&h->arena, total, hipDeviceMallocContiguous)
                                  : hipMalloc(&h->arena, total);
  if (pad) (void)hipFree(pad);
  if (e != hipSuccess) {
    delete h;
    return fail(PAXISIM_ENOMEM, "hipMalloc(%zu bytes) failed: %s", total, hipGetErrorString(e));
  }
  h->arena_bytes = total;
  layout((char*)h->arena, true);
  int rc1 = 0;
  const size_t ncmp = CM_SUMS + (cfg->clusters + CB - 1) / CB;
  if ((e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking)) != hipSuccess ||
      (e = hipMalloc(&h->d_scratch, sizeof(uint64_t) * 64)) != hipSuccess ||
      (e = hipMalloc(&h->d_cmp, sizeof(uint32_t) * ncmp)) != hipSuccess ||
      (e = hipMalloc(&h->d_pairs, sizeof(uint32_t) * 2 * (C / 2 + LANES))) != hipSuccess ||
      (e = hipMalloc(&h->d_ph, sizeof(uint32_t) * (PH_SUMS + 2 * ((cfg->clusters + CB - 1) / CB)))) != hipSuccess ||
      (e = hipMalloc(&h->d_faults, sizeof(DevFault) * PAXISIM_MAX_FAULTS)) != hipSuccess ||
      (e = hipMemsetAsync(h->arena, 0, zero_bytes, h->stream)) != hipSuccess)
    rc1 = fail(PAXISIM_EDEVICE, "device setup failed: %s", hipGetErrorString(e));
  if (!rc1 && P.move_every) {   // the moving-Mu tables (the caller's buffer is not kept)
    const size_t mb = (size_t)P.move_tables * PAXISIM_MAX_KEYS * sizeof(uint32_t);
    if ((e = hipMalloc(&h->d_move, mb)) != hipSuccess ||
        (e = hipMemcpy(h->d_move, wl->move_cdf, mb, hipMemcpyHostToDevice)) != hipSuccess)
      rc1 = fail(PAXISIM_EDEVICE, "move_cdf upload failed: %s", hipGetErrorString(e));
    P.move_cdf = h->d_move;
  }
  h->wl.move_cdf = nullptr;
  if (!rc1) {
    P.faults = h->d_faults;
    P.bound = h->d_cmp;
    // compaction: Paxos (the swap covers its arrays); PAXISIM_COMPACT=0 turns it off (A/B)
    const char* ce = getenv("PAXISIM_COMPACT");
    P.compact = cfg->protocol == PAXISIM_PAXOS && !(ce && atoi(ce) == 0);
    for (uint32_t w = 0; w < wl->outstanding; w++)
      if (P.start_step[w] + 1u > h->late_until) h->late_until = P.start_step[w] + 1u;
    // pipelined launches (serial kernels): PAXISIM_PIPE = chunks per launch at most (1: off; default 4)
    if (const char* pe = getenv("PAXISIM_PIPE")) h->pipe_max = (uint32_t)atoi(pe) ? (uint32_t)atoi(pe) : 1u;
    if (h->pipe_max > 1 && h->ops.serial && h->ops.launch_pipe) {
      uint32_t xcc[64] = {0};
      const size_t nq = 16 + (C / LANES > 64 ? C / LANES : 64);   // the probe writes 64 words after the header
      if ((e = hipMalloc(&h->d_pipe, sizeof(uint32_t) * nq)) != hipSuccess ||
          (e = hipMemsetAsync(h->d_pipe, 0, sizeof(uint32_t) * 16, h->stream)) != hipSuccess)
        rc1 = fail(PAXISIM_EDEVICE, "pipelined launch setup failed: %s", hipGetErrorString(e));
      if (!rc1) {
        // the poll limit of a chunk wait (sim_core.h pipe_item); PAXISIM_PIPE_SPIN sets it for tests
        uint32_t spin = PXS_PIPE_SPIN_DEFAULT;
        if (const char* se = getenv("PAXISIM_PIPE_SPIN")) spin = (uint32_t)strtoul(se, nullptr, 0);
        if ((e = hipMemcpyAsync(h->d_pipe + 9, &spin, sizeof spin, hipMemcpyHostToDevice, h->stream)) != hipSuccess)
          rc1 = fail(PAXISIM_EDEVICE, "pipelined launch setup failed: %s", hipGetErrorString(e));
      }
      if (!rc1) {
        xcc_probe<<<64, 64, 0, h->stream>>>(h->d_pipe + 16);
        if ((e = hipGetLastError()) != hipSuccess ||
            (e = hipMemcpyAsync(xcc, h->d_pipe + 16, sizeof xcc, hipMemcpyDeviceToHost, h->stream)) != hipSuccess ||
            (e = hipStreamSynchronize(h->stream)) != hipSuccess)
          rc1 = fail(PAXISIM_EDEVICE, "XCD probe failed: %s", hipGetErrorString(e));
        for (uint32_t b = 0; b < 64 && !rc1; b++)     // round robin over 8 XCDs, any rotation
          if ((xcc[b] & 7u) != ((xcc[0] + b) & 7u) || xcc[b] > 7u) h->pipe_max = 1;
      }
    } else {
      h->pipe_max = 1;
    }
    // pipelined (PAXISIM_PIPE > 1, the default): compaction every three chunks (at most pipe_max), so
    // they fuse (A/B r5v / r5x, config 2: 50-step chunks with compaction every 100 +2.0% against every
    // 50 unpipelined, every 200 with four chunks +0.0%; 25-step chunks every 75 another +0.9 / +2.2%
    // in the two run modes, every 50 +0.5 / +1.1%)
    if (h->pipe_max > 1 && h->ops.serial && h->ops.launch_pipe) h->cmp_every = (h->pipe_max < 3u ? h->pipe_max : 3u) * h->S;
    if (const char* ev = getenv("PAXISIM_COMPACT_EVERY")) h->cmp_every = (uint32_t)atoi(ev) ? (uint32_t)atoi(ev) : 1u;
    const uint32_t b0 = (uint32_t)cfg->clusters;
    h->bound_host = b0;
    e = hipMemcpyAsync(h->d_cmp, &b0, sizeof b0, hipMemcpyHostToDevice, h->stream);
    if (e == hipSuccess) init_kernel<<<(unsigned)((C + 255) / 256), 256, 0, h->stream>>>(P);
    if (e != hipSuccess || (e = hipGetLastError()) != hipSuccess || (e = hipStreamSynchronize(h->stream)) != hipSuccess)
      rc1 = fail(PAXISIM_EDEVICE, "init kernel failed: %s", hipGetErrorString(e));
  }
  if (rc1) {
    paxisim_destroy(h);
    return rc1;
  }
  *out = h;
  return 0;
}

extern "C" int paxisim_fault_add(paxisim* h, const paxisim_fault* f) {
  if (!h || !f) return fail(PAXISIM_EINVAL, "null argument");
  if (h->faults.size() == PAXISIM_MAX_FAULTS) return fail(PAXISIM_EINVAL, "fault table full");
  if (f->kind > PAXISIM_FAULT_CRASH || f->src >= h->P.N || (f->dst != PAXISIM_ALL_DST && f->dst >= h->P.N))
    return fail(PAXISIM_EINVAL, "bad fault");
  if (f->kind == PAXISIM_FAULT_SLOW && f->param > h->cfg.max_delay)
    return fail(PAXISIM_EINVAL, "slow delay exceeds max_delay");
  HIPCHK(hipSetDevice(h->cfg.device));
  h->faults.push_back(dev_fault(*f));
  HIPCHK(hipMemcpyAsync(h->d_faults, h->faults.data(), h->faults.size() * sizeof(DevFault),
                        hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  h->P.nfaults = (uint32_t)h->faults.size();
  return 0;
}

static hipError_t ensure_lds(paxisim* h) {
  const int lds = (int)(h->P.G * h->P.lds_bytes);
  if (h->lds_set != lds) {            // per handle, so per device
    hipError_t e = h->ops.set_lds(lds);
    if (e != hipSuccess) return e;
    h->lds_set = lds;
  }
  return hipSuccess;
}

static hipError_t launch_any(paxisim* h, uint32_t t0, uint32_t n) {
  const hipError_t e = ensure_lds(h);
  return e != hipSuccess ? e : h->ops.launch(h->P, h->stream, t0, n);
}

// After a pipelined launch every live tile must have run all K chunks; a tile
// that did not (a wait that gave up, or waves missing from an XCD's queue)
// sets the error word, which the host reads at the next sync (pipe_check).
__global__ void pipe_verify(const uint32_t* bound, uint32_t* q, uint32_t K) {
  const uint32_t tiles = (*bound + LANES - 1u) / LANES;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < tiles; i += gridDim.x * blockDim.x)
    if (q[16 + i] != K) atomicOr(&q[8], 2u);
}

// K chunks of n steps in one pipelined launch (sim_core.h sim_serial_pipe)
static hipError_t launch_pipe(paxisim* h, uint32_t t0, uint32_t n, uint32_t K) {
  hipError_t e = ensure_lds(h);          // the serial instances set both kernels' ceilings
  if (e != hipSuccess) return e;
  // tickets and chunk counts restart; the error word q[8] is sticky (cleared at create only)
  if ((e = hipMemsetAsync(h->d_pipe, 0, sizeof(uint32_t) * 8, h->stream)) != hipSuccess ||
      (e = hipMemsetAsync(h->d_pipe + 16, 0, sizeof(uint32_t) * (h->P.C / LANES), h->stream)) != hipSuccess)
    return e;
  if ((e = h->ops.launch_pipe(h->P, h->stream, t0, n, K, h->d_pipe)) != hipSuccess) return e;
  pipe_verify<<<64, 256, 0, h->stream>>>(h->P.bound, h->d_pipe, K);
  return hipGetLastError();
}

// a pipelined launch whose wait gave up (q[9], PAXISIM_PIPE_SPIN) left its tiles unstepped: fail loudly
// The copy is ordered on h->stream (a non-blocking stream: a null-stream
// hipMemcpy would not wait for the launches in flight), so the word read is
// the one every earlier launch left.  Every readout entry point calls this
// first, so no caller gets stats or state of a step that did not fully run.
static int pipe_check(paxisim* h) {
  if (!h->d_pipe) return 0;
  uint32_t w[8] = {0};   // q[8..16): error word, spin limit, the first give-up
  HIPCHK(hipMemcpyAsync(w, h->d_pipe + 8, sizeof w, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  if (!w[0]) return 0;
  if (w[0] & 1u)
    return fail(PAXISIM_EDEVICE, "pipelined step launch: a chunk wait timed out (xcd %u ticket %u tile %u chunk %u: "
                "done[tile] = %u, xcd tickets taken %u)", w[2], w[3], w[4], w[5], w[6], w[7]);
  return fail(PAXISIM_EDEVICE, "pipelined step launch: a tile missed chunks");
}

static int compact(paxisim* h) {
  const Params& P = h->P;
  const unsigned nb = (unsigned)((h->cfg.clusters + CB - 1) / CB);
  uint32_t* lo = h->d_pairs;
  uint32_t* hi = h->d_pairs + (P.C / 2 + LANES);
  cmp_count<<<nb, CB, 0, h->stream>>>(P, h->d_cmp);
  cmp_scan<<<1, CB, 0, h->stream>>>(P, h->d_cmp, nb);
  cmp_index<<<nb, CB, 0, h->stream>>>(P, h->d_cmp, lo, hi);
  cmp_swap<<<4096, LANES, 0, h->stream>>>(P, h->d_cmp, lo, hi);
  cmp_freeze<<<nb, CB, 0, h->stream>>>(P, h->d_cmp, h->t);
  cmp_setbound<<<1, 1, 0, h->stream>>>(h->d_cmp);
  if (P.phase_sort) {   // group the stepped slots by phase class
    uint32_t* ph = h->d_ph;
    HIPCHK(hipMemsetAsync(ph, 0, PH_SUMS * sizeof(uint32_t), h->stream));
    ph_classes<<<nb, CB, 0, h->stream>>>(P, h->d_cmp, ph);
    for (uint32_t p = 0; p < P.phase_period; p++) {   // classes 0..period-1; the quiescent ones end up last
      ph_region<<<1, 1, 0, h->stream>>>(ph, p);
      ph_count<<<nb, CB, 0, h->stream>>>(P, h->d_cmp, ph, p, nb);
      ph_scan<<<1, CB, 0, h->stream>>>(h->d_cmp, ph, nb);
      ph_index<<<nb, CB, 0, h->stream>>>(P, h->d_cmp, ph, p, nb, lo, hi);
      cmp_swap<<<4096, LANES, 0, h->stream>>>(P, h->d_cmp, lo, hi);
    }
  }
  HIPCHK(hipGetLastError());
  h->last_cmp = h->t;
  return 0;
}

// A request for a frozen cluster: move it to the first frozen slot, replay the
// fault process of that slot's tile up to now and step the tile again.
static int wake(paxisim* h, uint64_t cluster) {
  const Params& P = h->P;
  uint32_t bound = 0, slot = 0;
  HIPCHK(hipMemcpyAsync(&bound, h->d_cmp + CM_BOUND, 4, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipMemcpyAsync(&slot, P.slot_of + cluster, 4, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  h->bound_host = bound;
  if (slot < bound) return 0;
  if (slot != bound) swap_one<<<1, LANES, 0, h->stream>>>(P, bound, slot);
  uint64_t end = (uint64_t)bound + LANES;
  if (end > h->cfg.clusters) end = h->cfg.clusters;
  const uint64_t n = (end - bound) * P.N;
  replay_kernel<<<(unsigned)((n + 63) / 64), 64, 0, h->stream>>>(P, bound, end, h->t);
  const uint32_t nb32 = (uint32_t)end;
  HIPCHK(hipMemcpyAsync(h->d_cmp + CM_BOUND, &nb32, 4, hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(h->stream));
  h->bound_host = nb32;
  return 0;
}

__global__ void read_client_kernel(Params P, uint64_t cl, paxisim_worker_state* out) {
  const uint32_t w = threadIdx.x;
  if (w >= P.WK) return;
  const uint64_t c = slot_of(P, cl);
  const uint8_t* img = P.image + (c / LANES) * (size_t)P.img.bytes;
  const uint32_t wi = (w << 6) | (uint32_t)(c % LANES);
  paxisim_worker_state s;
  s.cid = reinterpret_cast<const uint32_t*>(img + P.img.off_wcur)[wi];
  s.issued = reinterpret_cast<const uint32_t*>(img + P.img.off_wiss)[wi];
  s.reply_value = P.wrep[(size_t)w * P.C + c];
  s.pad = 0;
  out[w] = s;
}

extern "C" int paxisim_read_client(paxisim* h, uint64_t cluster, paxisim_worker_state* out, uint32_t cap,
                                   uint32_t* n_out) {
  if (!h || !n_out || (cap && !out)) return fail(PAXISIM_EINVAL, "null argument");
  if (cluster >= h->cfg.clusters) return fail(PAXISIM_ERANGE, "bad cluster");
  HIPCHK(hipSetDevice(h->cfg.device));
  if (const int rc = pipe_check(h)) return rc;   // results only of launches that fully ran
  const uint32_t n = h->P.WK;
  *n_out = n;
  if (!cap || !n) return 0;
  paxisim_worker_state* d = nullptr;
  HIPCHK(hipMalloc(&d, n * sizeof(paxisim_worker_state)));
  read_client_kernel<<<1, 64, 0, h->stream>>>(h->P, cluster, d);
  hipError_t e = hipGetLastError();
  std::vector<paxisim_worker_state> tmp(n);
  if (e == hipSuccess) e = hipMemcpyAsync(tmp.data(), d, n * sizeof(paxisim_worker_state), hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  (void)hipFree(d);
  if (e != hipSuccess) return fail(PAXISIM_EDEVICE, "read_client: %s", hipGetErrorString(e));
  for (uint32_t w = 0; w < n && w < cap; w++) out[w] = tmp[w];
  return 0;
}

__global__ void read_kv_kernel(Params P, uint64_t cl, uint32_t r, uint32_t n, uint32_t* out) {
  const uint32_t k = threadIdx.x + blockIdx.x * blockDim.x;
  if (k >= n) return;
  const uint64_t c = slot_of(P, cl);
  if (P.protocol == PAXISIM_ABD)
    out[k] = reinterpret_cast<const uint32_t*>(P.image + (c / LANES) * (size_t)P.img.bytes +
                                               P.img.off_a)[((r * P.keys + k) << 6) | (c % LANES)];
  else
    out[k] = P.kv_val[((size_t)k * P.N + r) * P.C + c];
}

// Database.Get (db.go:116-121) of keys [0, n) of one replica
extern "C" int paxisim_read_kv(paxisim* h, uint64_t cluster, uint32_t replica, uint32_t* values, uint32_t n) {
  if (!h || (n && !values)) return fail(PAXISIM_EINVAL, "null argument");
  if (cluster >= h->cfg.clusters || replica >= h->P.N || n > h->P.keys) return fail(PAXISIM_ERANGE, "bad key range");
  if (h->P.protocol != PAXISIM_ABD && !h->P.kv) return fail(PAXISIM_EUNSUPP, "replicas keep no Database (config.kv = 0)");
  if (n == 0) return 0;
  HIPCHK(hipSetDevice(h->cfg.device));
  if (const int rc = pipe_check(h)) return rc;   // results only of launches that fully ran
  uint32_t* d = nullptr;
  HIPCHK(hipMalloc(&d, n * sizeof(uint32_t)));
  read_kv_kernel<<<(n + 63) / 64, 64, 0, h->stream>>>(h->P, cluster, replica, n, d);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipMemcpyAsync(values, d, n * sizeof(uint32_t), hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  (void)hipFree(d);
  if (e != hipSuccess) return fail(PAXISIM_EDEVICE, "read_kv: %s", hipGetErrorString(e));
  return 0;
}

extern "C" int paxisim_active_clusters(paxisim* h, uint64_t* active) {
  if (!h || !active) return fail(PAXISIM_EINVAL, "null argument");
  HIPCHK(hipSetDevice(h->cfg.device));
  if (const int rc = pipe_check(h)) return rc;   // results only of launches that fully ran
  uint32_t bound = 0;
  HIPCHK(hipMemcpyAsync(&bound, h->d_cmp + CM_BOUND, 4, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  h->bound_host = bound;
  *active = bound;
  return 0;
}

__global__ void activity_kernel(Params P, uint64_t lo, uint64_t n, uint32_t* out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t s = slot_of(P, lo + i);
  out[i] = s < *P.bound ? 0xFFFFFFFFu : P.frz[s];
}

extern "C" int paxisim_quorum(const paxisim_config* cfg, uint32_t kind, uint32_t ack_mask, int* satisfied) {
  if (!cfg || !satisfied) return fail(PAXISIM_EINVAL, "null argument");
  if (cfg->n_zones == 0 || cfg->n_zones > PAXISIM_MAX_ZONES || kind > PAXISIM_Q_FGRID_Q2)
    return fail(PAXISIM_EINVAL, "bad zones or quorum kind");
  uint32_t npz[PAXISIM_MAX_ZONES], zmask[PAXISIM_MAX_ZONES], N = 0;
  for (uint32_t z = 0; z < cfg->n_zones; z++) {
    if (cfg->npz[z] == 0 || N + cfg->npz[z] > PAXISIM_MAX_N) return fail(PAXISIM_EINVAL, "bad nodes per zone");
    npz[z] = cfg->npz[z];
    zmask[z] = ((1u << npz[z]) - 1u) << N;
    N += npz[z];
  }
  *satisfied = quorum_check(kind, N, cfg->n_zones, npz, zmask, cfg->fz, ack_mask & ((1u << N) - 1u)) ? 1 : 0;
  return 0;
}

extern "C" int paxisim_read_activity(paxisim* h, uint64_t lo, uint64_t n, uint32_t* frozen_at) {
  if (!h || !frozen_at) return fail(PAXISIM_EINVAL, "null argument");
  if (lo + n > h->cfg.clusters || lo + n < lo) return fail(PAXISIM_ERANGE, "cluster range");
  if (n == 0) return 0;
  HIPCHK(hipSetDevice(h->cfg.device));
  if (const int rc = pipe_check(h)) return rc;   // results only of launches that fully ran
  uint32_t* d = nullptr;
  HIPCHK(hipMalloc(&d, n * sizeof(uint32_t)));
  activity_kernel<<<(unsigned)((n + 255) / 256), 256, 0, h->stream>>>(h->P, lo, n, d);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipMemcpyAsync(frozen_at, d, n * sizeof(uint32_t), hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  (void)hipFree(d);
  if (e != hipSuccess) return fail(PAXISIM_EDEVICE, "read_activity: %s", hipGetErrorString(e));
  return 0;
}

extern "C" int paxisim_step(paxisim* h, uint32_t nsteps) {
  if (!h) return fail(PAXISIM_EINVAL, "null handle");
  if ((uint64_t)h->t + nsteps >= T_MAX) return fail(PAXISIM_EINVAL, "step counter would exceed 2^28");
  HIPCHK(hipSetDevice(h->cfg.device));
  while (nsteps > 0) {
    const uint32_t n = nsteps < h->S ? nsteps : h->S;
    // chunks fused into this launch: up to pipe_max whole chunks, none past a due compaction
    uint32_t K = 1;
    if (h->pipe_max > 1 && n == h->S) {
      auto due = [&](uint32_t t) { return h->P.compact && t >= h->late_until && t - h->last_cmp >= h->cmp_every; };
      while (K < h->pipe_max && (K + 1u) * n <= nsteps && !due(h->t + K * n)) K++;
    }
    hipEvent_t a, b;
    HIPCHK(hipEventCreate(&a));
    hipError_t e = hipEventCreate(&b);
    if (e != hipSuccess) {
      (void)hipEventDestroy(a);
      return fail(PAXISIM_EDEVICE, "hipEventCreate: %s", hipGetErrorString(e));
    }
    if ((e = hipEventRecord(a, h->stream)) == hipSuccess &&
        (e = K > 1 ? launch_pipe(h, h->t, n, K) : launch_any(h, h->t, n)) == hipSuccess)
      e = hipEventRecord(b, h->stream);
    if (e != hipSuccess) {              // no leaked events on the error path
      (void)hipEventDestroy(a);
      (void)hipEventDestroy(b);
      return fail(PAXISIM_EDEVICE, "step launch: %s", hipGetErrorString(e));
    }
    h->evs.emplace_back(a, b);
    h->launches++;
    h->t += K * n;
    nsteps -= K * n;
    if (h->P.compact && h->t >= h->late_until && h->t - h->last_cmp >= h->cmp_every) {
      const int rc = compact(h);
      if (rc) return rc;
    }
    if (h->evs.size() >= 256) {
      int rc = flush_events(h);
      if (rc) return rc;
    }
  }
  return 0;
}

extern "C" int paxisim_sync(paxisim* h) {
  if (!h) return fail(PAXISIM_EINVAL, "null handle");
  HIPCHK(hipSetDevice(h->cfg.device));
  HIPCHK(hipStreamSynchronize(h->stream));
  return pipe_check(h);
}

extern "C" int paxisim_kernel_time(paxisim* h, double* ms, uint64_t* launches, int reset) {
  if (!h) return fail(PAXISIM_EINVAL, "null handle");
  HIPCHK(hipSetDevice(h->cfg.device));
  int rc = flush_events(h);
  if (rc) return rc;
  if (ms) *ms = h->kernel_ms;
  if (launches) *launches = h->launches;
  if (reset) {
    h->kernel_ms = 0;
    h->launches = 0;
  }
  return 0;
}

extern "C" int paxisim_inject(paxisim* h, uint64_t cluster, uint32_t replica, uint32_t cid) {
  if (!h) return fail(PAXISIM_EINVAL, "null handle");
  if (cluster >= h->cfg.clusters || replica >= h->P.N || cid < 1 || cid > CMD_MASK)
    return fail(PAXISIM_EINVAL, "bad inject (cluster %llu, replica %u, cid %u)", (unsigned long long)cluster,
                replica, cid);
  HIPCHK(hipSetDevice(h->cfg.device));
  if (h->P.compact) {
    const int rc = wake(h, cluster);
    if (rc) return rc;
  }
  uint32_t st = 0;
  inject_kernel<<<1, 64, 0, h->stream>>>(h->P, cluster, replica, h->t % h->P.D, cid, (uint32_t*)h->d_scratch);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(&st, h->d_scratch, sizeof st, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  if (st) return fail(PAXISIM_EINVAL, "client mailbox full");
  return 0;
}

extern "C" int paxisim_read_inbox(paxisim* h, uint64_t cluster, uint32_t replica, paxisim_inbox_record* out,
                                  uint32_t cap, uint32_t* n_out) {
  if (!h || !n_out || (cap && !out)) return fail(PAXISIM_EINVAL, "null argument");
  if (cluster >= h->cfg.clusters || replica >= h->P.N) return fail(PAXISIM_ERANGE, "bad inbox");
  HIPCHK(hipSetDevice(h->cfg.device));
  if (const int rc = pipe_check(h)) return rc;   // results only of launches that fully ran
  HIPCHK(hipStreamSynchronize(h->stream));
  const uint32_t maxn = h->P.NS * h->P.M;   // a bucket set holds at most this many
  paxisim_inbox_record* d = nullptr;
  HIPCHK(hipMalloc(&d, maxn * sizeof(paxisim_inbox_record) + 64));
  uint32_t* dn = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(d) + maxn * sizeof(paxisim_inbox_record));
  read_inbox_kernel<<<1, 64, 0, h->stream>>>(h->P, cluster, replica, h->t % h->P.D, d, maxn, dn);
  hipError_t e = hipGetLastError();
  uint32_t n = 0;
  if (e == hipSuccess) e = hipMemcpyAsync(&n, dn, sizeof n, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  if (e == hipSuccess && cap)
    e = hipMemcpy(out, d, (n < cap ? n : cap) * sizeof(paxisim_inbox_record), hipMemcpyDeviceToHost);
  (void)hipFree(d);
  if (e != hipSuccess) return fail(PAXISIM_EDEVICE, "read_inbox: %s", hipGetErrorString(e));
  *n_out = n;
  return 0;
}

extern "C" int paxisim_commands(paxisim* h, uint64_t cluster, const uint32_t* cids, uint32_t n, uint32_t* keys,
                                uint32_t* writes) {
  if (!h || (n && (!cids || !keys || !writes))) return fail(PAXISIM_EINVAL, "null argument");
  if (cluster >= h->cfg.clusters) return fail(PAXISIM_ERANGE, "bad cluster");
  if (n == 0) return 0;
  HIPCHK(hipSetDevice(h->cfg.device));
  if (const int rc = pipe_check(h)) return rc;   // results only of launches that fully ran
  uint32_t* d = nullptr;
  HIPCHK(hipMalloc(&d, 3ull * n * sizeof(uint32_t)));
  hipError_t e = hipMemcpyAsync(d, cids, n * sizeof(uint32_t), hipMemcpyHostToDevice, h->stream);
  if (e == hipSuccess) {
    command_kernel<<<(n + 255) / 256, 256, 0, h->stream>>>(h->P, cluster, d, n, d + n, d + 2 * n);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpyAsync(keys, d + n, n * sizeof(uint32_t), hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(writes, d + 2 * n, n * sizeof(uint32_t), hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  (void)hipFree(d);
  if (e != hipSuccess) return fail(PAXISIM_EDEVICE, "commands: %s", hipGetErrorString(e));
  return 0;
}

extern "C" int paxisim_deliver(paxisim* h, uint64_t cluster, uint32_t replica, uint32_t src,
                               const paxisim_inbox_record* recs, uint32_t n) {
  if (!h || (n && !recs)) return fail(PAXISIM_EINVAL, "null argument");
  if (cluster >= h->cfg.clusters || replica >= h->P.N || src > h->P.N)
    return fail(PAXISIM_EINVAL, "bad deliver (cluster %llu, replica %u, src %u)", (unsigned long long)cluster,
                replica, src);
  if (n == 0) return 0;
  if (n > h->P.M) return fail(PAXISIM_EINVAL, "mailbox full");
  HIPCHK(hipSetDevice(h->cfg.device));
  if (h->P.compact) {
    const int rc = wake(h, cluster);
    if (rc) return rc;
  }
  paxisim_inbox_record* d = nullptr;
  HIPCHK(hipMalloc(&d, n * sizeof(paxisim_inbox_record)));
  hipError_t e = hipMemcpyAsync(d, recs, n * sizeof(paxisim_inbox_record), hipMemcpyHostToDevice, h->stream);
  uint32_t st = 0;
  if (e == hipSuccess) {
    deliver_kernel<<<1, 64, 0, h->stream>>>(h->P, cluster, replica, src, h->t % h->P.D, d, n,
                                            (uint32_t*)h->d_scratch);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpyAsync(&st, h->d_scratch, sizeof st, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  (void)hipFree(d);
  if (e != hipSuccess) return fail(PAXISIM_EDEVICE, "deliver: %s", hipGetErrorString(e));
  if (st) return fail(PAXISIM_EINVAL, "mailbox full");
  return 0;
}

extern "C" int paxisim_read_log(paxisim* h, uint64_t cluster, uint32_t replica, uint32_t key, int32_t slot_lo,
                                uint32_t n, paxisim_log_entry* out) {
  if (!h || !out) return fail(PAXISIM_EINVAL, "null argument");
  if (cluster >= h->cfg.clusters || replica >= h->P.N || key >= h->P.NK) return fail(PAXISIM_ERANGE, "bad entry");
  if (n == 0) return 0;
  HIPCHK(hipSetDevice(h->cfg.device));
  if (const int rc = pipe_check(h)) return rc;   // results only of launches that fully ran
  paxisim_log_entry* d = nullptr;
  HIPCHK(hipMalloc(&d, n * sizeof(paxisim_log_entry)));
  read_log_kernel<<<(n + 63) / 64, 64, 0, h->stream>>>(h->P, cluster, replica, key, slot_lo, n, d);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipMemcpyAsync(out, d, n * sizeof(paxisim_log_entry), hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  (void)hipFree(d);
  if (e != hipSuccess) return fail(PAXISIM_EDEVICE, "read_log: %s", hipGetErrorString(e));
  for (uint32_t i = 0; i < n; i++) out[i].ballot = expand_ballot(h, (uint32_t)out[i].ballot);
  return 0;
}

extern "C" int paxisim_stats_get(paxisim* h, paxisim_stats* out) {
  if (!h || !out) return fail(PAXISIM_EINVAL, "null argument");
  HIPCHK(hipSetDevice(h->cfg.device));
  if (const int rc = pipe_check(h)) return rc;   // results only of launches that fully ran
  uint64_t red[NRED];
  HIPCHK(hipMemsetAsync(h->d_scratch, 0, sizeof(uint64_t) * NRED, h->stream));
  stats_kernel<<<(unsigned)(h->P.C / 256 + 1), 256, 0, h->stream>>>(h->P, h->d_scratch);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(red, h->d_scratch, sizeof red, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  memset(out, 0, sizeof *out);
  out->steps = h->t;
  out->clusters = h->cfg.clusters;
  for (int k = 0; k < PAXISIM_NMSG; k++) {
    out->delivered[k] = red[ST_DELIV0 + k];
    out->delivered_total += red[ST_DELIV0 + k];
  }
  out->client_requests = red[ST_CLIENT];
  out->sent = red[ST_SENT];
  out->dropped = red[ST_DROPPED];
  out->discarded = red[ST_DISCARDED];
  out->commits = red[ST_COMMITS];
  out->replies = red[ST_REPLIES];
  out->agree_compared = red[ST_AGC];
  out->agree_missed = red[ST_AGM];
  out->agree_mismatch = red[ST_AGB];
  for (int b = 0; b < 8; b++) out->flagged[b] = red[NSTAT + b];
  return 0;
}

extern "C" int paxisim_read_state(paxisim* h, uint64_t lo, uint64_t n, paxisim_replica_state* out) {
  if (!h || !out) return fail(PAXISIM_EINVAL, "null argument");
  if (lo + n > h->cfg.clusters || lo + n < lo) return fail(PAXISIM_ERANGE, "cluster range");
  if (n == 0) return 0;
  HIPCHK(hipSetDevice(h->cfg.device));
  if (const int rc = pipe_check(h)) return rc;   // results only of launches that fully ran
  const size_t cnt = (size_t)n * h->P.N;
  paxisim_replica_state* d = nullptr;
  HIPCHK(hipMalloc(&d, cnt * sizeof(paxisim_replica_state)));
  gather_kernel<<<(unsigned)((cnt + 255) / 256), 256, 0, h->stream>>>(h->P, lo, n, d);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipMemcpyAsync(out, d, cnt * sizeof(paxisim_replica_state), hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  (void)hipFree(d);
  if (e != hipSuccess) return fail(PAXISIM_EDEVICE, "read_state: %s", hipGetErrorString(e));
  for (size_t i = 0; i < cnt; i++) out[i].ballot = expand_ballot(h, (uint32_t)out[i].ballot);
  return 0;
}

extern "C" int paxisim_read_instances(paxisim* h, uint64_t lo, uint64_t n, paxisim_instance_state* out) {
  if (!h || !out) return fail(PAXISIM_EINVAL, "null argument");
  if (lo + n > h->cfg.clusters || lo + n < lo) return fail(PAXISIM_ERANGE, "cluster range");
  if (n == 0) return 0;
  HIPCHK(hipSetDevice(h->cfg.device));
  if (const int rc = pipe_check(h)) return rc;   // results only of launches that fully ran
  const uint32_t ni = h->P.protocol == PAXISIM_EPAXOS ? h->P.N * h->P.N : h->P.NI;   // per cluster; EPaxos: (replica, owner log)
  const size_t cnt = (size_t)n * ni;
  paxisim_instance_state* d = nullptr;
  HIPCHK(hipMalloc(&d, cnt * sizeof(paxisim_instance_state)));
  gather_inst_kernel<<<(unsigned)((cnt + 255) / 256), 256, 0, h->stream>>>(h->P, lo, n, d);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipMemcpyAsync(out, d, cnt * sizeof(paxisim_instance_state), hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  (void)hipFree(d);
  if (e != hipSuccess) return fail(PAXISIM_EDEVICE, "read_instances: %s", hipGetErrorString(e));
  for (size_t i = 0; i < cnt; i++) out[i].ballot = expand_ballot(h, (uint32_t)out[i].ballot);
  return 0;
}

extern "C" int paxisim_check(paxisim* h, uint64_t* violations) {
  if (!h || !violations) return fail(PAXISIM_EINVAL, "null argument");
  HIPCHK(hipSetDevice(h->cfg.device));
  if (const int rc = pipe_check(h)) return rc;   // results only of launches that fully ran
  HIPCHK(hipMemsetAsync(h->d_scratch, 0, sizeof(uint64_t), h->stream));
  check_kernel<<<(unsigned)(h->P.C / 256 + 1), 256, 0, h->stream>>>(h->P, h->d_scratch);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(violations, h->d_scratch, sizeof(uint64_t), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return 0;
}

extern "C" int paxisim_occupancy(paxisim* h, int* blocks_per_cu, uint32_t* lds_bytes, uint32_t* staged) {
  if (!h || !blocks_per_cu) return fail(PAXISIM_EINVAL, "null argument");
  HIPCHK(hipSetDevice(h->cfg.device));
  HIPCHK(h->ops.occupancy(h->P, blocks_per_cu));
  *blocks_per_cu *= (int)h->P.G;    // 64-cluster tiles resident per CU
  if (lds_bytes) *lds_bytes = h->P.lds_bytes;
  if (staged) *staged = h->P.J;
  return 0;
}

extern "C" int paxisim_device_bytes(paxisim* h, uint64_t* bytes) {
  if (!h || !bytes) return fail(PAXISIM_EINVAL, "null argument");
  *bytes = h->arena_bytes;
  return 0;
}

// Completed ABD operations of one cluster, 5 words per op {key, is_write,
// value, start, end}, replicas in index order, each in completion order.
extern "C" int paxisim_history(paxisim* h, uint64_t cluster, uint32_t* buf, uint32_t cap_ops, uint32_t* n_out) {
  if (!h || !n_out) return fail(PAXISIM_EINVAL, "null argument");
  if (cluster >= h->cfg.clusters) return fail(PAXISIM_ERANGE, "cluster");
  HIPCHK(hipSetDevice(h->cfg.device));
  if (const int rc = pipe_check(h)) return rc;   // results only of launches that fully ran
  HIPCHK(hipStreamSynchronize(h->stream));   // step kernels run on the non-blocking h->stream
  const Params& P = h->P;
  std::vector<uint32_t> len(P.N);
  for (uint32_t r = 0; r < P.N; r++)
    HIPCHK(hipMemcpy(&len[r], &P.execute[rc_host(P, r, cluster)], 4, hipMemcpyDeviceToHost));
  uint32_t n = 0;
  for (uint32_t r = 0; r < P.N && P.H; r++) {
    std::vector<uint4> tmp(len[r]);
    if (len[r])
      HIPCHK(hipMemcpy(tmp.data(), &P.hist[((size_t)r * P.C + cluster) * P.H], len[r] * sizeof(uint4),
                       hipMemcpyDeviceToHost));
    for (uint32_t j = 0; j < len[r]; j++, n++) {
      if (!buf || n >= cap_ops) continue;
      uint32_t* o = buf + 5 * (size_t)n;
      o[0] = tmp[j].x & 0x7FFFFFFFu;
      o[1] = tmp[j].x >> 31;
      o[2] = tmp[j].y;
      o[3] = tmp[j].z;
      o[4] = tmp[j].w;
    }
  }
  *n_out = n;
  return 0;
}

// History.ReadFile (history.go:115-178) into the device history of one replica.
extern "C" int paxisim_history_load(paxisim* h, uint64_t cluster, uint32_t replica, const uint32_t* ops, uint32_t n) {
  if (!h || (n && !ops)) return fail(PAXISIM_EINVAL, "null argument");
  if (cluster >= h->cfg.clusters || replica >= h->P.N) return fail(PAXISIM_ERANGE, "bad replica");
  if (h->P.protocol != PAXISIM_ABD) return fail(PAXISIM_EUNSUPP, "op history is kept by ABD only");
  if (n > h->P.H) return fail(PAXISIM_EINVAL, "%u ops exceed history capacity %u", n, h->P.H);
  HIPCHK(hipSetDevice(h->cfg.device));
  HIPCHK(hipStreamSynchronize(h->stream));
  const Params& P = h->P;
  std::vector<uint4> tmp(n ? n : 1);
  for (uint32_t j = 0; j < n; j++) {
    const uint32_t* o = ops + 5 * (size_t)j;
    if (o[0] >= h->P.keys || o[1] > 1u) return fail(PAXISIM_EINVAL, "op %u: bad key (keys = %u) or is_write", j, h->P.keys);
    tmp[j] = make_uint4(o[0] | (o[1] << 31), o[2], o[3], o[4]);
  }
  if (n)
    HIPCHK(hipMemcpy(&P.hist[((size_t)replica * P.C + cluster) * P.H], tmp.data(), n * sizeof(uint4),
                     hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(&P.execute[rc_host(P, replica, cluster)], &n, 4, hipMemcpyHostToDevice));
  return 0;
}

extern "C" int paxisim_linearizable(paxisim* h, uint64_t* anomalies, uint64_t* ops, uint64_t* skipped) {
  if (!h) return fail(PAXISIM_EINVAL, "null handle");
  if (h->P.protocol != PAXISIM_ABD || h->P.H == 0)
    return fail(PAXISIM_EUNSUPP, "linearizability scan needs protocol ABD with history > 0");
  HIPCHK(hipSetDevice(h->cfg.device));
  if (const int rc = pipe_check(h)) return rc;   // results only of launches that fully ran
  HIPCHK(hipStreamSynchronize(h->stream));
  const Params& P = h->P;
  // clusters per launch: each gets a stage of N*H ops (its history grouped by key).
  // The stage takes up to a quarter of the free HBM (2-16 GiB): fewer, longer
  // launches leave less of each launch's last round of workgroups idle
  // (config 3: 21 -> 6 launches); PAXISIM_LIN_STAGE_MB overrides (A/B).
  const size_t cap = (size_t)P.N * P.H;
  size_t budget = 2ull << 30, freeb = 0, totb = 0;
  if (hipMemGetInfo(&freeb, &totb) == hipSuccess) budget = std::max(budget, std::min<size_t>(freeb / 4, 16ull << 30));
  if (const char* e = getenv("PAXISIM_LIN_STAGE_MB")) budget = std::max<size_t>(1, (size_t)atoll(e)) << 20;
  const uint64_t chunk = std::max<uint64_t>(1, std::min<uint64_t>(P.clusters, budget / (cap * sizeof(uint4))));
  uint4* stage = nullptr;
  uint2* big = nullptr;
  unsigned long long* out = nullptr;
  uint8_t* bws = nullptr;
  size_t bws_bytes = 0;
  const size_t nout = LIN_NOUT + 8;
  auto cleanup = [&]() {
    (void)hipFree(stage);
    (void)hipFree(big);
    (void)hipFree(out);
    (void)hipFree(bws);
  };
  hipError_t e = hipMalloc(&stage, chunk * cap * sizeof(uint4));
  if (e == hipSuccess) e = hipMalloc(&big, chunk * P.keys * sizeof(uint2));
  if (e == hipSuccess) e = hipMalloc(&out, nout * sizeof(unsigned long long));
  if (e == hipSuccess) e = hipMemsetAsync(out, 0, nout * sizeof(unsigned long long), h->stream);
  const uint32_t lds = LIN_LW * LIN_SORT_BYTES;
  unsigned long long tot[LIN_NOUT] = {0};
  for (uint64_t c0 = 0; e == hipSuccess && c0 < P.clusters; c0 += chunk) {
    const uint64_t nc = std::min<uint64_t>(chunk, P.clusters - c0);
    if ((e = hipMemsetAsync(out + LIN_BIG, 0, 2 * sizeof(unsigned long long), h->stream)) != hipSuccess) break;
    lin_cluster_kernel<<<(unsigned)nc, LIN_LW * 64, lds, h->stream>>>(P, c0, stage, out, big);
    unsigned long long bc[2] = {0, 0};
    if ((e = hipGetLastError()) != hipSuccess) break;
    if ((e = hipMemcpyAsync(bc, out + LIN_BIG, sizeof bc, hipMemcpyDeviceToHost, h->stream)) != hipSuccess) break;
    if ((e = hipStreamSynchronize(h->stream)) != hipSuccess) break;
    if (bc[0]) {   // partitions above LIN_SMAX ops: one wave each, scratch in HBM
      tot[LIN_BIG] += bc[0];
      tot[LIN_NMAX] = std::max<unsigned long long>(tot[LIN_NMAX], bc[1]);
      const uint32_t nw = (uint32_t)((bc[1] + 63u) / 64u);     // bc[1] <= LIN_VMAX (larger: skipped)
      const size_t per = lin_scratch_bytes(nw, true);
      const uint32_t waves = (uint32_t)std::max<unsigned long long>(
          1, std::min<unsigned long long>(std::min<unsigned long long>(bc[0], 2048), (2ull << 30) / per));
      const size_t need = (size_t)waves * per;
      if (need > bws_bytes) {
        (void)hipFree(bws);
        bws = nullptr;
        bws_bytes = 0;
        if ((e = hipMalloc(&bws, need)) != hipSuccess) break;
        bws_bytes = need;
      }
      if (nw <= 64u) lin_big_kernel<1><<<waves, 64, 0, h->stream>>>(stage, big, (uint32_t)bc[0], bws, nw, out);
      else lin_big_kernel<LIN_WPL_MAX><<<waves, 64, 0, h->stream>>>(stage, big, (uint32_t)bc[0], bws, nw, out);
      if ((e = hipGetLastError()) != hipSuccess) break;
    }
  }
  uint64_t res[LIN_NOUT + 8] = {0};
  if (e == hipSuccess) e = hipMemcpyAsync(res, out, sizeof res, hipMemcpyDeviceToHost, h->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  cleanup();
  if (e != hipSuccess) return fail(PAXISIM_EDEVICE, "linearizable: %s", hipGetErrorString(e));
#ifdef PXS_LIN_STAMPS
  fprintf(stderr, "lin stamps (wave-cycles): p1 %llu p2 %llu sort %llu run %llu | add %llu look %llu merge %llu reach %llu\n",
          (unsigned long long)res[LIN_NOUT + 0], (unsigned long long)res[LIN_NOUT + 1], (unsigned long long)res[LIN_NOUT + 2],
          (unsigned long long)res[LIN_NOUT + 3], (unsigned long long)res[LIN_NOUT + 4], (unsigned long long)res[LIN_NOUT + 5],
          (unsigned long long)res[LIN_NOUT + 6], (unsigned long long)res[LIN_NOUT + 7]);
#endif
  h->lin_big = tot[LIN_BIG];
  h->lin_nmax = tot[LIN_NMAX];
  if (anomalies) *anomalies = res[LIN_ANOM];
  if (ops) *ops = res[LIN_OPS];
  if (skipped) *skipped = res[LIN_SKIP];   // partitions above LIN_VMAX ops (not checked)
  return 0;
}

// ---------------------------------------------------------------------------
// Multi-GPU behind the C-ABI: clusters shard by range across
// handles (cluster_base), the data path has no collective, and the statistics
// are summed (max for time) with one RCCL all-reduce.  RCCL is opened at run
// time, so the library loads without it and only these calls need it; a
// process that already holds librccl.so.1 (e.g. through torch) shares it.
// ---------------------------------------------------------------------------
namespace {
struct Rccl {
  bool ok = false;
  ncclResult_t (*get_unique_id)(ncclUniqueId*);
  ncclResult_t (*init_rank)(ncclComm_t*, int, ncclUniqueId, int);
  ncclResult_t (*init_all)(ncclComm_t*, int, const int*);
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t);
  ncclResult_t (*group_start)();
  ncclResult_t (*group_end)();
  ncclResult_t (*destroy)(ncclComm_t);
  const char* (*error_string)(ncclResult_t);
};
Rccl& rccl() {
  static Rccl r;
  static bool tried = false;
  if (tried) return r;
  tried = true;
  void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!h) return r;
  auto sym = [&](const char* n) { return dlsym(h, n); };
  r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(sym("ncclGetUniqueId"));
  r.init_rank = reinterpret_cast<decltype(r.init_rank)>(sym("ncclCommInitRank"));
  r.init_all = reinterpret_cast<decltype(r.init_all)>(sym("ncclCommInitAll"));
  r.all_reduce = reinterpret_cast<decltype(r.all_reduce)>(sym("ncclAllReduce"));
  r.group_start = reinterpret_cast<decltype(r.group_start)>(sym("ncclGroupStart"));
  r.group_end = reinterpret_cast<decltype(r.group_end)>(sym("ncclGroupEnd"));
  r.destroy = reinterpret_cast<decltype(r.destroy)>(sym("ncclCommDestroy"));
  r.error_string = reinterpret_cast<decltype(r.error_string)>(sym("ncclGetErrorString"));
  r.ok = r.get_unique_id && r.init_rank && r.init_all && r.all_reduce && r.group_start && r.group_end && r.destroy &&
         r.error_string;
  return r;
}
}  // namespace

#define RCCLCHK(expr)                                                                      \
  do {                                                                                     \
    ncclResult_t r_ = (expr);                                                              \
    if (r_ != ncclSuccess) return fail(PAXISIM_EDEVICE, "%s: %s", #expr, rccl().error_string(r_)); \
  } while (0)

struct paxisim_dist {
  std::vector<paxisim*> h;           // handles driven by this process, one per device
  std::vector<ncclComm_t> comm;
  std::vector<void*> buf;            // per member: device buffer for the reduction
};

constexpr uint32_t DIST_MAXV = 64;   // u64 sums + f64 maxes per reduction

extern "C" int paxisim_dist_unique_id(unsigned char id[128]) {
  if (!id) return fail(PAXISIM_EINVAL, "null argument");
  if (!rccl().ok) return fail(PAXISIM_EUNSUPP, "RCCL (librccl.so.1) not available");
  ncclUniqueId u;
  RCCLCHK(rccl().get_unique_id(&u));
  memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
  return 0;
}

static int dist_alloc(paxisim_dist* d) {
  for (paxisim* h : d->h) {
    void* b = nullptr;
    HIPCHK(hipSetDevice(h->cfg.device));
    HIPCHK(hipMalloc(&b, 2 * DIST_MAXV * sizeof(uint64_t)));
    d->buf.push_back(b);
  }
  return 0;
}

extern "C" int paxisim_dist_destroy(paxisim_dist* d) {
  if (!d) return 0;
  for (size_t i = 0; i < d->comm.size(); i++) (void)rccl().destroy(d->comm[i]);
  for (size_t i = 0; i < d->buf.size(); i++) {
    (void)hipSetDevice(d->h[i]->cfg.device);
    (void)hipFree(d->buf[i]);
  }
  delete d;
  return 0;
}

// Single process, one handle per device (ncclCommInitAll)
extern "C" int paxisim_dist_init(paxisim* const* handles, int n, paxisim_dist** out) {
  if (!handles || n < 1 || !out) return fail(PAXISIM_EINVAL, "bad argument");
  if (!rccl().ok) return fail(PAXISIM_EUNSUPP, "RCCL (librccl.so.1) not available");
  std::vector<int> devs;
  for (int i = 0; i < n; i++) {
    if (!handles[i]) return fail(PAXISIM_EINVAL, "null handle %d", i);
    for (int d : devs)
      if (d == handles[i]->cfg.device) return fail(PAXISIM_EINVAL, "two handles on device %d", d);
    devs.push_back(handles[i]->cfg.device);
  }
  paxisim_dist* d = new (std::nothrow) paxisim_dist();
  if (!d) return fail(PAXISIM_ENOMEM, "oom");
  d->h.assign(handles, handles + n);
  d->comm.resize(n);
  ncclResult_t r = rccl().init_all(d->comm.data(), n, devs.data());
  if (r != ncclSuccess) {
    d->comm.clear();
    paxisim_dist_destroy(d);
    return fail(PAXISIM_EDEVICE, "ncclCommInitAll: %s", rccl().error_string(r));
  }
  int rc = dist_alloc(d);
  if (rc) {
    paxisim_dist_destroy(d);
    return rc;
  }
  *out = d;
  return 0;
}

// One handle per process: every rank passes the id one rank obtained from
// paxisim_dist_unique_id (the caller ships it, e.g. over its launcher)
extern "C" int paxisim_dist_init_rank(paxisim* h, const unsigned char id[128], int nranks, int rank,
                                      paxisim_dist** out) {
  if (!h || !id || nranks < 1 || rank < 0 || rank >= nranks || !out) return fail(PAXISIM_EINVAL, "bad argument");
  if (!rccl().ok) return fail(PAXISIM_EUNSUPP, "RCCL (librccl.so.1) not available");
  HIPCHK(hipSetDevice(h->cfg.device));
  paxisim_dist* d = new (std::nothrow) paxisim_dist();
  if (!d) return fail(PAXISIM_ENOMEM, "oom");
  d->h.push_back(h);
  d->comm.resize(1);
  ncclUniqueId u;
  memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
  ncclResult_t r = rccl().init_rank(&d->comm[0], nranks, u, rank);
  if (r != ncclSuccess) {
    d->comm.clear();
    paxisim_dist_destroy(d);
    return fail(PAXISIM_EDEVICE, "ncclCommInitRank: %s", rccl().error_string(r));
  }
  int rc = dist_alloc(d);
  if (rc) {
    paxisim_dist_destroy(d);
    return rc;
  }
  *out = d;
  return 0;
}

// Sum sums_in[i] (i < n) and max maxes_in[j] (j < m) over every member of
// every rank; member k's inputs are at sums_in[k*n], maxes_in[k*m].  The
// result (the same on every member) goes to sums_out[0..n), maxes_out[0..m).
extern "C" int paxisim_dist_allreduce(paxisim_dist* d, const uint64_t* sums_in, uint32_t n, const double* maxes_in,
                                      uint32_t m, uint64_t* sums_out, double* maxes_out) {
  if (!d || n > DIST_MAXV || m > DIST_MAXV || (n && (!sums_in || !sums_out)) || (m && (!maxes_in || !maxes_out)))
    return fail(PAXISIM_EINVAL, "bad argument");
  const size_t k = d->h.size();
  for (size_t i = 0; i < k; i++) {
    paxisim* h = d->h[i];
    HIPCHK(hipSetDevice(h->cfg.device));
    uint64_t* b = static_cast<uint64_t*>(d->buf[i]);
    if (n) HIPCHK(hipMemcpyAsync(b, sums_in + i * n, n * 8, hipMemcpyHostToDevice, h->stream));
    if (m) HIPCHK(hipMemcpyAsync(b + DIST_MAXV, maxes_in + i * m, m * 8, hipMemcpyHostToDevice, h->stream));
  }
  RCCLCHK(rccl().group_start());
  for (size_t i = 0; i < k; i++) {
    uint64_t* b = static_cast<uint64_t*>(d->buf[i]);
    if (n) (void)rccl().all_reduce(b, b, n, ncclUint64, ncclSum, d->comm[i], d->h[i]->stream);
    if (m) (void)rccl().all_reduce(b + DIST_MAXV, b + DIST_MAXV, m, ncclFloat64, ncclMax, d->comm[i], d->h[i]->stream);
  }
  RCCLCHK(rccl().group_end());
  for (size_t i = 0; i < k; i++) {
    paxisim* h = d->h[i];
    HIPCHK(hipSetDevice(h->cfg.device));
    uint64_t* b = static_cast<uint64_t*>(d->buf[i]);
    if (i == 0 && n) HIPCHK(hipMemcpyAsync(sums_out, b, n * 8, hipMemcpyDeviceToHost, h->stream));
    if (i == 0 && m) HIPCHK(hipMemcpyAsync(maxes_out, b + DIST_MAXV, m * 8, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
  }
  return 0;
}

// paxisim_stats summed over every handle of the job (u64 fields), and the
// largest step-kernel time of any handle (kernel_ms_max may be NULL)
extern "C" int paxisim_dist_stats(paxisim_dist* d, paxisim_stats* out, double* kernel_ms_max) {
  if (!d || !out) return fail(PAXISIM_EINVAL, "null argument");
  constexpr uint32_t NV = sizeof(paxisim_stats) / sizeof(uint64_t);
  static_assert(sizeof(paxisim_stats) % sizeof(uint64_t) == 0 && NV <= DIST_MAXV, "stats layout");
  const size_t k = d->h.size();
  std::vector<uint64_t> in(k * NV);
  std::vector<double> tin(k);
  for (size_t i = 0; i < k; i++) {
    paxisim_stats s;
    int rc = paxisim_stats_get(d->h[i], &s);
    if (rc) return rc;
    memcpy(&in[i * NV], &s, sizeof s);
    double ms = 0;
    if ((rc = paxisim_kernel_time(d->h[i], &ms, nullptr, 0))) return rc;
    tin[i] = ms;
  }
  uint64_t res[NV];
  double tmax = 0;
  int rc = paxisim_dist_allreduce(d, in.data(), NV, tin.data(), 1, res, &tmax);
  if (rc) return rc;
  memcpy(out, res, sizeof *out);
  if (kernel_ms_max) *kernel_ms_max = tmax;
  return 0;
}

#if (defined(PXS_WAVE_TIMES) || defined(PXS_TALLY)) && !defined(PXS_STAMPS)
constexpr uint32_t DBG_PER = 48;   // the stamps build's buffer size (paxisim_dev.h); two words per block used
#endif
#if defined(PXS_STAMPS) || defined(PXS_WAVE_TIMES) || defined(PXS_TALLY)
// Diagnostic builds only: per (block, replica) {setup, loop, barrier cycles, loop trips, records, steps}
// (PXS_STAMPS), per block the serial kernel's start and end clock (PXS_WAVE_TIMES, tools/wave_times.py), or
// per block the access-class tallies (PXS_TALLY, tools/tally.py).
extern "C" int paxisim_dbg_enable(paxisim* h) {
  HIPCHK(hipSetDevice(h->cfg.device));
  const size_t n = (h->P.C / LANES) * 16 * DBG_PER;
  HIPCHK(hipMalloc(&h->P.dbg, n * 8));
  HIPCHK(hipMemset(h->P.dbg, 0, n * 8));
  return 0;
}
extern "C" int paxisim_dbg_read(paxisim* h, unsigned long long* out) {
  HIPCHK(hipSetDevice(h->cfg.device));
  HIPCHK(hipStreamSynchronize(h->stream));
  const size_t n = (h->P.C / LANES) * 16 * DBG_PER;
  HIPCHK(hipMemcpy(out, h->P.dbg, n * 8, hipMemcpyDeviceToHost));
  HIPCHK(hipMemset(h->P.dbg, 0, n * 8));
  return 0;
}
#endif
