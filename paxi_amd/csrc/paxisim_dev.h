// paxisim_dev.h — device-side layout, PRNG and shared helpers of the HIP path.
//
// Execution model: one workgroup = N waves x 64 lanes.  Wave r
// plays replica r, lane l plays cluster 64*blockIdx.x + l, so all replicas of
// a cluster live in one workgroup and exchange messages through memory the
// workgroup owns.  A workgroup advances its 64 clusters S steps per launch
// with one __syncthreads() per step.
//
// Per launch the workgroup's hot state (log windows, mailbox counts, client
// worker tables, poison flags) is copied from its HBM image into LDS and
// back; message records stay in HBM in a block-contiguous region and are
// prefetched one message ahead; replica scalars and socket fault state live
// in registers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/paxisim.h"

namespace pxs {

constexpr uint32_t PMAX = 32;   // pending requests per replica (p.requests)
constexpr uint32_t FMAX = 32;   // forwards table per replica (node.forwards)
constexpr uint32_t CKI = 16;    // checkpoint interval (executed slots)
constexpr uint32_t CKR = 8;     // checkpoints kept per replica
constexpr uint32_t GMAX = 8;    // live entries below execute kept per instance
constexpr uint32_t AGMAX = 8;   // agreement-ring arrivals buffered per replica-step
constexpr uint32_t NO_ID = 0xFFu;
constexpr uint32_t POL_NONE = 0xFFu;   // consecutive.last == "" (policy.go:50)
constexpr uint32_t LANES = 64;
constexpr uint32_t LDS_MAX = 160u * 1024u;
constexpr uint32_t T_MAX = 1u << 28;   // slow_until is packed in 28 bits

// log entry, LDS form: {ballot, cmd | flags, ack mask}
constexpr uint32_t CMD_MASK = 0x07FFFFFFu;
constexpr uint32_t EF_EXISTS = 1u << 27, EF_COMMIT = 1u << 28, EF_QUORUM = 1u << 29;
constexpr uint32_t EF_REQSELF = 1u << 30;   // request == (cmd, client): kept implicit
constexpr uint32_t EF_REQEXT = 1u << 31;    // request in the HBM side table

enum { PUR_ORDER = 1, PUR_LINK = 2, PUR_SLOWD = 3, PUR_FLAKY = 4 };

// per-replica counter slots in Params::stats ([slot][r][C])
enum {
  ST_DELIV0 = 0,                    // 16 slots: delivered by message type
  ST_CLIENT = PAXISIM_NMSG,
  ST_SENT, ST_DROPPED, ST_DISCARDED, ST_COMMITS, ST_REPLIES,
  ST_AGC, ST_AGM, ST_AGB,           // agreement checkpoints compared / missed / mismatched
  NSTAT
};

// Byte layout of a workgroup's LDS image (identical in HBM, one per block).
// Regions a/b/c belong to the protocol:
//   Paxos: log window ballot / cmd|flags / ack mask, each [r][W][lane] u32
//   ABD:   KV value / KV version [r][K][lane] u32, op table [r][OW][6][lane] u32
struct Image {
  uint32_t off_a, off_b, off_c, off_wcur, off_wiss, off_poison, off_cnt, bytes;
};

__host__ __device__ inline Image image_layout(uint32_t bytes_a, uint32_t bytes_b, uint32_t bytes_c, uint32_t N,
                                              uint32_t WK, uint32_t D) {
  Image m;
  m.off_a = 0;
  m.off_b = m.off_a + bytes_a;
  m.off_c = m.off_b + bytes_b;
  m.off_wcur = m.off_c + bytes_c;
  m.off_wiss = m.off_wcur + WK * LANES * 4u;
  m.off_poison = m.off_wiss + WK * LANES * 4u;
  m.off_cnt = m.off_poison + LANES * 4u;
  m.bytes = (m.off_cnt + D * N * (N + 1u) * LANES + 15u) & ~15u;
  return m;
}

// ABD op table: a power of two >= 2*outstanding, at least 4
__host__ __device__ inline uint32_t abd_ow(uint32_t outstanding) {
  uint32_t ow = 4;
  while (ow < 2u * outstanding) ow <<= 1;
  return ow;
}
constexpr uint32_t ABD_OPF = 6;   // op fields: tag, req, state|get<<2|set<<17, value, version, start
enum { ABD_FREE = 0, ABD_GET = 1, ABD_SET = 2, ABD_DONE = 3 };

// A scripted fault as the device reads it: the 40-byte paxisim_fault repacked
// into three 16-byte-aligned words by paxisim_fault_add, so every load of the
// table is a naturally aligned uint4 (the ABI struct is only 8-byte aligned).
struct alignas(16) DevFault {
  uint4 a;   // kind, src, dst, param
  uint4 b;   // cluster_lo (lo, hi), cluster_hi (lo, hi)
  uint4 c;   // step_from, step_to, 0, 0
};
__host__ inline DevFault dev_fault(const paxisim_fault& f) {
  DevFault d;
  d.a = make_uint4(f.kind, f.src, f.dst, f.param);
  d.b = make_uint4((uint32_t)f.cluster_lo, (uint32_t)(f.cluster_lo >> 32), (uint32_t)f.cluster_hi,
                   (uint32_t)(f.cluster_hi >> 32));
  d.c = make_uint4(f.step_from, f.step_to, 0u, 0u);
  return d;
}

struct Params {
  uint32_t protocol, N, Z, W, M, D, NS, WK, max_requests;
  uint32_t keys, write_ppm, locality_ppm, H, OW;
  uint32_t dist, conflicts;             // workload key distribution (paxisim_distribution)
  uint32_t key_cdf[PAXISIM_MAX_KEYS];   // TABLE inverse CDF
  uint32_t NK, NI;       // Paxos instances per replica (WPaxos: keys, else 1); per cluster NI = NK*N
  uint32_t adaptive, policy_thr;
  uint32_t policy, policy_interval;   // paxisim_policy; MAJORITY interval in steps
  double policy_alpha;                // EMA alpha
  uint32_t wk_magic;     // floor((2^32-1)/WK): (x % WK) by multiply-high + one correction
  uint64_t C;            // allocated cluster lanes (multiple of 64)
  uint64_t clusters;     // live clusters
  uint64_t cluster_base, seed;
  uint32_t q1, q2, fz, thrifty, ephemeral, rwc, max_delay, nfaults;
  uint32_t drop_ppm, drop_len, slow_ppm, slow_len, slow_min, slow_max;
  uint32_t npz[PAXISIM_MAX_ZONES], zmask[PAXISIM_MAX_ZONES];
  uint32_t zone_of[PAXISIM_MAX_N];   // 0-based zone of each replica
  uint32_t target[PAXISIM_MAX_WORKERS];
  uint32_t start_step[PAXISIM_MAX_WORKERS];   // first request of worker w at this step
  uint32_t late_workers;                      // mask of workers with start_step > 0
  // workload keys (sim_core.h wl_key), per worker w: zone z of its target, the
  // count nk of that zone's keys {k = z mod Z} and floor((2^32-1)/nk); and
  // floor((2^32-1)/keys): (x % d) as a multiply-high and one correction
  uint32_t wzone[PAXISIM_MAX_WORKERS], wnk[PAXISIM_MAX_WORKERS], wnk_magic[PAXISIM_MAX_WORKERS];
  uint32_t keys_magic;
  Image img;
  uint32_t J, off_stage;   // LDS stage: J staged picks per replica at LDS byte off_stage ([r][J][64] x 16 B)
  uint32_t lds_bytes;      // LDS per cluster group (16-B multiple): the image + the stage
  uint32_t lds_tail;       // serial kernel: the image bytes [lds_tail, bytes) are staged in LDS (PXS_CLIENT_LDS)
  uint32_t off_wscr;       // serial kernel, WPaxos (wlds): LDS byte offset of the replica-step instance scratch [K][5][lane]
  uint32_t G;              // cluster groups (64-cluster tiles) per workgroup
  uint32_t rec_per_block;  // D*N*NS*M*64
  const DevFault* faults;
  // Paxos instance scalars [NI][C] (Multi-Paxos: NI = N); node scalars flags/nfwd [N][C]
  uint32_t *ballot, *slot, *execute, *meta, *flags, *npend, *nfwd;
  uint64_t* digest;
  uint32_t* kc;          // [C] per-cluster PRNG key
  uint32_t* pend;        // [PMAX][NI][C]
  uint32_t* fwd;         // [FMAX][N][C]
  uint32_t *link_drop, *link_slow;  // [dst][N][C]: drop_until; slow_until | delay << 28
  uint32_t* ck_e;        // [CKR][NI][C]
  uint64_t* ck_d;        // [CKR][NI][C]
  uint4* gst;            // entries below execute {slot, ballot, until | commit << 31, 0}: [GMAX][NI][C], per-key instances [NI][C][GMAX]
  // WPaxos kpaxos instances, one 32-B state + a W-entry window + PMAX pending per
  // (blk, key, r, lane): {ballot, slot, execute, active|exists<<1|p1acks<<16,
  // npend, digest lo, digest hi, policy last|hits<<8}; entries {ballot, cmd|flags, acks, request}
  uint4* wst;            // [blk][K][N][64] x wst_str uint4 (wlds = 0): {ballot..meta}, {npend, digest, pol|cmask}
  uint32_t wst_str;      // uint4s between instances: 2, or (wcoloc) the co-located block's size / 16
  uint32_t wlog_str;     // u32s between instances' windows: W * 4, or (wcoloc) the block's size / 4
  uint32_t wlds;         // 1: instance scalars in the tile image (region a, LDS during a launch), digests in wdig
  uint32_t wcoloc;       // 1 (wlds = 0): an instance's scalars and window in one block (PAXISIM_WCOLOC)
  uint64_t* wdig;        // [blk][K][N][64] instance digests (wlds = 1)
  uint32_t* wlog;        // [blk][K][N][64][W][4]; wcoloc: 32 B into each instance's block, after its wst
  uint32_t* wpend;       // [blk][K][N][64][PMAX]
  uint4* wpx;            // [blk][K][N][64][3] majority {hits u16 x 16 (2 x uint4), {sum, start step}} / ema {s lo, s hi, zone}
  uint32_t* stats;       // [NSTAT][N][C]
  unsigned long long* agr;  // [AR][NK][C] first executor's digest per checkpoint: k << 40 | 40-bit digest fold;
                            // the C index is the local cluster id (not the slot: compaction leaves it in place)
  uint32_t AR;           // checkpoints kept per (cluster, instance); 0 = no agreement ring
  uint4* agq;            // [2][AGMAX][N][C] a step's ring arrivals {entry lo, entry hi, key, 0}, by step parity
  uint32_t off_agn;      // LDS byte offset of the arrival counts [2][N][lane] u8 (per tile, outside the image)
  uint32_t* reqx;        // [blk][N][W][64] request side table (Paxos)
  uint4* hist;           // [N][C][H] completed ABD ops {key|write<<31, value, start, end}
  uint8_t* image;        // [blk][img.bytes]
  unsigned long long* dbg;  // diagnostic build only (PXS_STAMPS): per-wave phase totals
  uint4* rec;            // [blk][D][dst][src][M][64]
  // Live-cluster compaction.  Every per-cluster array above is
  // indexed by the cluster's *slot*; slot_of / cl_of map local cluster ids to
  // slots and back.  Slots >= *bound hold quiescent (frozen) clusters that no
  // launch touches; frz[s] is the step a frozen slot stopped at, qf[s] = 1 when
  // the slot ended its last launch with an empty mailbox (a fixed point).
  uint32_t* slot_of;     // [C] cluster -> slot
  uint32_t* cl_of;       // [C] slot -> cluster
  uint32_t* frz;         // [C] per slot
  uint32_t* qf;          // [C] per slot
  uint32_t* bound;       // device scalar: slots [0, *bound) are stepped
  uint32_t compact;      // protocol supports compaction and it is enabled
  // Phase binning (serial kernel): each launch sums the records a
  // cluster's replicas handle per (step mod phase_period) in LDS (at l_cnt +
  // ph_rel), and ends by writing the busiest residue to phase[slot]; compaction
  // then groups live clusters by it, so a wave's lanes have their bursts together.
  uint32_t phase_sort, phase_period, ph_rel;
  uint32_t* phase;       // [C] per slot
  uint32_t variant;      // per-key protocol run by the WPaxos kernel: WPAXOS, M2PAXOS or KPAXOS
  uint32_t zfirst[PAXISIM_MAX_ZONES];   // replica index of "z.1" (KPaxos static leaders)
  uint32_t key_min;      // Bconfig.Min: key value of key index 0 (ORDER / UNIFORM / CONFLICT)
  // the workload's key space (paxisim.h paxisim_workload)
  uint32_t kspace, kspace_magic;   // ORDER / UNIFORM / CONFLICT range over [0, kspace)
  uint32_t conflict_key;           // index of CONFLICT's literal key 0 (kspace when key_min != 0)
  uint32_t key_tail;               // TABLE: draws >= key_tail (nonzero) lie beyond [0, keys)
  uint32_t move_every, move_tables, move_loop;   // moving Mu: table of command cid is (cid-1) / move_every
  const uint32_t* move_cdf;        // [move_tables][PAXISIM_MAX_KEYS]
  // EPaxos (epaxos_kernel.h)
  uint4* ep_inst;        // [blk][r][o][W][64] x 4 uint4
  uint32_t* ep_sce;      // [3][o][r][C] slot, committed, executed
  uint32_t* ep_cf;       // [2][o][K][r][C] conflicts {slot or -1, seq}
  uint32_t* ep_max;      // [K][r][C] maxSeqPerKey, -1 = absent
  // Database (db.go) of the log-based protocols when P.kv
  uint32_t kv;
  uint32_t* kv_val;      // [K][r][C] value = command id of the last write, 0 = nil
  uint32_t* kv_ver;      // [r][C] database.version
  uint32_t* wrep;        // [WK][C] Reply.Value of each worker's last reply (0 = nil)
};

// Persistent scalars of the kpaxos instance (blk, k, r, lane) in the record
// form {a = ballot, slot, execute, active|exists<<1|wovf,ghost<<2|p1acks<<16;
// b = npend, digest lo, digest hi, policy|committed window<<16}, from either
// layout: the HBM table wst, or (wlds) five words in the tile image,
// [(k*N + r)*5 + word][lane] = {ballot, slot, execute, meta | npend << 4,
// policy | committed window << 16}, and the digest in wdig.
constexpr uint32_t WP_WORDS = 5;
// Instance index of (blk, key k, replica r, lane) in the per-instance HBM
// arrays (wst, wdig, wlog, wpend, wpx).  Key-major keeps one key's 64 lanes
// together; lane-major (PXS_WP_LANEMAJOR) keeps one lane's K instances
// together, so the instances a replica-step binds share few lines.
#ifndef PXS_WP_LANEMAJOR
#define PXS_WP_LANEMAJOR 0
#endif
__device__ __forceinline__ size_t wp_si(const Params& P, uint64_t blk, uint32_t k, uint32_t r, uint32_t lane) {
  if (PXS_WP_LANEMAJOR) return ((blk * P.N + r) * 64u + lane) * P.keys + k;
  return ((blk * P.keys + k) * P.N + r) * 64u + lane;
}
__device__ __forceinline__ uint32_t* wp_img(const Params& P, uint64_t blk, uint32_t k, uint32_t r, uint32_t lane) {
  return reinterpret_cast<uint32_t*>(P.image + (size_t)blk * P.img.bytes + P.img.off_a) +
         ((size_t)(k * P.N + r) * WP_WORDS << 6) + lane;
}
__device__ __forceinline__ void wp_read(const Params& P, uint64_t blk, uint32_t k, uint32_t r, uint32_t lane, uint4& a,
                                        uint4& b) {
  const size_t si = wp_si(P, blk, k, r, lane);
  if (!P.wlds) {
    a = P.wst[(size_t)P.wst_str * si];
    b = P.wst[(size_t)P.wst_str * si + 1];
    return;
  }
  const uint32_t* w = wp_img(P, blk, k, r, lane);
  const uint64_t d = P.wdig[si];
  a = make_uint4(w[0], w[64], w[128], w[192] & 0xFFFF000Fu);
  b = make_uint4((w[192] >> 4) & 0x3Fu, (uint32_t)d, (uint32_t)(d >> 32), w[256]);
}
__device__ __forceinline__ void wp_write(const Params& P, uint64_t blk, uint32_t k, uint32_t r, uint32_t lane,
                                         const uint4& a, const uint4& b) {
  const size_t si = wp_si(P, blk, k, r, lane);
  if (!P.wlds) {
    P.wst[(size_t)P.wst_str * si] = a;
    P.wst[(size_t)P.wst_str * si + 1] = b;
    return;
  }
  uint32_t* w = wp_img(P, blk, k, r, lane);
  w[0] = a.x; w[64] = a.y; w[128] = a.z; w[192] = (a.w & 0xFFFF000Fu) | (b.x << 4); w[256] = b.w;
  P.wdig[si] = (uint64_t)b.y | ((uint64_t)b.z << 32);
}

// slot of local cluster c
__device__ __forceinline__ uint64_t slot_of(const Params& P, uint64_t c) { return P.slot_of[c]; }

// ---- PRNG ------------------------------------------------
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z ^= z >> 30; z *= 0xbf58476d1ce4e5b9ULL;
  z ^= z >> 27; z *= 0x94d049bb133111ebULL;
  z ^= z >> 31;
  return z;
}
__host__ __device__ __forceinline__ uint32_t fmix32(uint32_t h) {
  h ^= h >> 16; h *= 0x85ebca6bu;
  h ^= h >> 13; h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}
__host__ __device__ __forceinline__ uint32_t cluster_key(uint64_t seed, uint64_t gid) {
  return (uint32_t)mix64(seed ^ mix64(gid + 0x9E3779B97F4A7C15ULL));
}
__device__ __forceinline__ uint32_t step_key(uint32_t kc, uint32_t t) { return fmix32(kc ^ (t * 0x9E3779B1u)); }
__device__ __forceinline__ uint32_t draw(uint32_t hs, uint32_t tag) { return fmix32(hs ^ tag); }
__device__ __forceinline__ uint32_t tag(uint32_t p, uint32_t a, uint32_t b) { return (p << 28) | (a << 20) | b; }
__device__ __forceinline__ bool ppm_hit(uint32_t x, uint32_t ppm) { return __umulhi(x, 1000000u) < ppm; }
__device__ __forceinline__ bool ppm_hit16(uint32_t x16, uint32_t ppm) { return ((x16 * 15625u) >> 10) < ppm; }

// ---- ballots: (n << 4) | replica, 0 = none (ballot.go:12-52) -------------
__device__ __forceinline__ uint32_t bal_id(uint32_t b) { return b ? (b & 15u) : NO_ID; }
__device__ __forceinline__ uint32_t bal_next(uint32_t b, uint32_t self) { return (((b >> 4) + 1u) << 4) | self; }

// ---- requests: cid | origin << 27 (message.go:24-30) ---------------------
__device__ __forceinline__ uint32_t req_cid(uint32_t q) { return q & CMD_MASK; }
__device__ __forceinline__ uint32_t req_origin(uint32_t q) { return q >> 27; }
__device__ __forceinline__ uint32_t mkreq(uint32_t cid, uint32_t o) { return cid | (o << 27); }

// ---- message records: {hdr = type | n << 8 | key << 16, ballot, slot, cid} --
// n: P1b payload records (ABD: the key); key: the WPaxos kpaxos instance
__device__ __forceinline__ uint32_t hdr_type(uint32_t h) { return h & 0xFFu; }
__device__ __forceinline__ uint32_t hdr_n(uint32_t h) { return (h >> 8) & 0xFFu; }
__device__ __forceinline__ uint32_t hdr_key(uint32_t h) { return h >> 16; }
// records of one message: a P1b and the EPaxos messages carry payload records
// (ABD keeps its key in bits 8-15, so the count is read only for those types)
__device__ __forceinline__ uint32_t rec_len(uint32_t h) {
  const uint32_t t = hdr_type(h);
  return 1u + ((t == PAXISIM_MSG_P1B || (t >= PAXISIM_MSG_PREACCEPT && t <= PAXISIM_MSG_COMMIT)) ? hdr_n(h) : 0u);
}

// ---- quorum predicates on an ack mask (quorum.go:55-119) -----------------
// One definition for the kernels and the host (paxisim_quorum exports it, so
// a caller can check the predicates the kernels use against quorum.go).
__host__ __device__ __forceinline__ bool quorum_check(uint32_t kind, uint32_t N, uint32_t Z, const uint32_t* npz,
                                                      const uint32_t* zmask, uint32_t fz, uint32_t mask) {
  const int size = __builtin_popcount(mask);
  if (kind == PAXISIM_Q_MAJORITY) return size > (int)(N / 2);
  uint32_t zones_any = 0, zones_maj = 0;
  bool col = false;
  for (uint32_t z = 0; z < Z; z++) {
    const uint32_t c = (uint32_t)__builtin_popcount(mask & zmask[z]);
    zones_any += c > 0;
    zones_maj += c > npz[z] / 2;
    col |= c == npz[z];
  }
  switch (kind) {
    case PAXISIM_Q_ALL: return size == (int)N;
    case PAXISIM_Q_FAST: return size >= (int)(N * 3 / 4);
    case PAXISIM_Q_GRID_ROW: return zones_any == Z;
    case PAXISIM_Q_ZONE_MAJORITY: return zones_maj > 0;
    case PAXISIM_Q_GRID_COLUMN: return col;
    case PAXISIM_Q_FGRID_Q1: return (int)zones_maj >= (int)Z - (int)fz;
    case PAXISIM_Q_FGRID_Q2: return (int)zones_maj >= (int)fz + 1;
  }
  return false;
}
__device__ __forceinline__ bool quorum_ok(const Params& P, uint32_t kind, uint32_t mask) {
  return quorum_check(kind, P.N, P.Z, P.npz, P.zmask, P.fz, mask);
}

// ---- loads retired on the spot ----------------------------------------------
// vmcnt counts stores as well as loads, and the compiler's waitcnt pass merges
// control-flow paths conservatively: a load left in flight in a rarely taken
// branch makes it wait on vmcnt (and so on every record store issued since) at
// the next join of the step loop.  Loads off the staged path are therefore
// consumed where they are issued.
__device__ __forceinline__ uint32_t ldg(const uint32_t* p) {
  uint32_t v = *p;
  asm volatile("" : "+v"(v));
  return v;
}
__device__ __forceinline__ uint64_t ldg(const uint64_t* p) {
  uint64_t v = *p;
  asm volatile("" : "+v"(v));
  return v;
}
__device__ __forceinline__ uint4 ldg(const uint4* p) {
  uint4 v = *p;
  asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w));
  return v;
}

// ---- scripted faults (uniform across the wave: scalar loads) -------------
__device__ __forceinline__ bool scripted(const Params& P, uint32_t kind, uint64_t gid, uint32_t src,
                                         uint32_t dst, uint32_t t, uint32_t* param) {
  bool hit = false;
  for (uint32_t i = 0; i < P.nfaults; i++) {
    paxisim_fault f;
    {
      const uint4 a = ldg(&P.faults[i].a);
      const uint4 b = ldg(&P.faults[i].b);
      const uint4 c = ldg(&P.faults[i].c);
      f.kind = a.x; f.src = a.y; f.dst = a.z; f.param = a.w;
      f.cluster_lo = (uint64_t)b.x | ((uint64_t)b.y << 32);
      f.cluster_hi = (uint64_t)b.z | ((uint64_t)b.w << 32);
      f.step_from = c.x; f.step_to = c.y;
    }
    if (f.kind != kind || f.src != src) continue;
    if (kind != PAXISIM_FAULT_CRASH && f.dst != PAXISIM_ALL_DST && f.dst != dst) continue;
    if (gid < f.cluster_lo || gid >= f.cluster_hi) continue;
    if (t < f.step_from || t >= f.step_to) continue;
    hit = true;
    if (param && f.param > *param) *param = f.param;
  }
  return hit;
}

// ---- diagnostic build (PXS_STAMPS): s_memtime phase and per-handler stamps ----
#ifdef PXS_STAMPS
constexpr uint32_t DBG_PER = 48;   // per (block, replica): 16 phase totals, 16 handler cycles, 16 handler runs
__device__ __forceinline__ unsigned long long stamp() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}
// cycles a wave spent in handler path k this trip (its lanes' branch runs once)
__device__ __forceinline__ void stamp_case(const Params& P, uint32_t blk, uint32_t r, uint32_t k, uint32_t c0) {
  const unsigned long long d = (uint32_t)stamp() - c0;   // 32-bit: a 64-bit stamp spilled trips a gfx950 codegen bug
  if (!P.dbg) return;
  const unsigned long long act = __ballot(1);
  if ((threadIdx.x & 63u) == (uint32_t)(__ffsll((long long)act) - 1)) {
    unsigned long long* q = &P.dbg[((size_t)blk * 16 + r) * DBG_PER];
    atomicAdd(&q[16 + k], d);
    atomicAdd(&q[32 + k], 1ull);
  }
}
#define PXS_CASE_T0 const uint32_t pxs_c0 = (uint32_t)stamp();
#define PXS_CASE_T1(k) if constexpr (NT != 0) stamp_case(P, x.blk, x.r, (k), pxs_c0);   // (NT = 0: a spill codegen bug)
// sub-handler regions (slots the Multi-Paxos kernels leave free: 5, 9-13)
#define PXS_SUB_T0(v) const uint32_t v = (uint32_t)stamp();
#define PXS_SUB_T1(v, k) if constexpr (NT != 0) stamp_case(P, x.blk, x.r, (k), v);
#else
#define PXS_CASE_T0
#define PXS_CASE_T1(k)
#define PXS_SUB_T0(v)
#define PXS_SUB_T1(v, k)
#endif

// The serial kernel keeps the client tables (wcur / wiss) in the HBM image
// (0) or stages them into LDS with the mailbox counts (1, A/B).
#ifndef PXS_CLIENT_LDS
#define PXS_CLIENT_LDS 1   // (A/B r3: the HBM tables cost config 2 6%, configs 4 and 5 4%)
#endif

// The serial kernel's WPaxos replica-step scratch (wpaxos_kernel.h step_begin):
// the current replica's instance scalars in LDS.  Off: the scratch costs more
// in tiles per CU (8 -> 5 on config 5) than it saves (A/B r3: -35%).
#ifndef PXS_WP_SCRATCH
#define PXS_WP_SCRATCH 0
#endif

// Phase binning of live clusters at compaction; the default,
// overridden at run time by PAXISIM_PHASE_SORT=0/1
#ifndef PXS_PHASE_SORT
#define PXS_PHASE_SORT 1   // (A/B r4h, config 2: 12.87-13.17 -> 16.05-16.33 G msgs/s)
#endif

// ---- SoA addressing --------------------------------------------------------
__device__ __forceinline__ size_t rc(const Params& P, uint32_t r, uint64_t c) { return (size_t)r * P.C + c; }
__device__ __forceinline__ size_t krc(const Params& P, uint32_t k, uint32_t r, uint64_t c) {
  return ((size_t)k * P.N + r) * P.C + c;
}

// ---- diagnostic build (PXS_TALLY): the HBM requests of each
// access class.  At every instrumented load or store the active lanes count
// the distinct 128-B lines (loads) or 32-B sectors (stores) their addresses
// fall in - the requests the instruction sends to L2 (a
// scattered read is one 128-B request, a scattered 16- or 32-B write one 32-B
// one) - and the first active lane adds (lane accesses, units) to the block's
// words in P.dbg, loads and stores apart.  tools/tally.py turns them into bytes per message. ----
enum TallyClass : uint32_t {
  TC_REC_LD, TC_REC_ST, TC_INST_LD, TC_INST_ST, TC_ENT_LD, TC_ENT_ST, TC_ROW_LD, TC_ROW_ST, TC_CNT, TC_KV_LD,
  TC_KV_ST, TC_FWD, TC_PEND, TC_CKPT, TC_AGREE, TC_REPLY, TC_GHOST, TC_LINK, TC_OTHER, TC_N
};
#ifdef PXS_TALLY
constexpr uint32_t TALLY_PER = 48;   // = DBG_PER; a block's 16 x 48 words in P.dbg hold [class][load, store][lanes, units]
__device__ __noinline__ void tally_at(unsigned long long* dbg, uint32_t blk, uint32_t cls, const void* p, bool store) {
  if (!dbg) return;
  const unsigned long long unit = (unsigned long long)(uintptr_t)p >> (store ? 5 : 7);
  unsigned long long m = __ballot(1);
  const unsigned long long lanes = __popcll(m);
  const int first = __ffsll((long long)m) - 1;
  unsigned long long n = 0;
  while (m) {
    const int f = __ffsll((long long)m) - 1;
    const unsigned long long u0 = __shfl(unit, f);
    m &= ~__ballot(unit == u0);
    n++;
  }
  if ((int)(threadIdx.x & 63u) == first) {
    unsigned long long* q = &dbg[(size_t)blk * 16 * TALLY_PER + 4 * cls + (store ? 2 : 0)];
    atomicAdd(&q[0], lanes);
    atomicAdd(&q[1], n);
  }
}
#define PXS_TALLY_AT(P, blk, cls, ptr, st) tally_at((P).dbg, (blk), (cls), (const void*)(ptr), (st))
#else
#define PXS_TALLY_AT(P, blk, cls, ptr, st)
#endif

}  // namespace pxs
