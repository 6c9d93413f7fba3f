// paxisim_dev.h — device-side layout, PRNG and shared helpers of the HIP path.
//
// Execution model: one workgroup = N waves x 64 lanes.  Wave r
// plays replica r, lane l plays cluster (64*blockIdx.x + l).  All state is
// structure-of-arrays with the cluster index fastest, so a wave's access to a
// field is one contiguous 256-byte (u32) run.  A workgroup owns its 64
// clusters for the whole launch and advances them S steps, with one
// __syncthreads() per step: messages sent in step t become visible to their
// receivers in step t+1+delay through the bucketed mailboxes.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/paxisim.h"

namespace pxs {

constexpr uint32_t PMAX = 32;   // pending requests per replica (p.requests)
constexpr uint32_t FMAX = 32;   // forwards table per replica (node.forwards)
constexpr uint32_t CKI = 16;    // checkpoint interval (executed slots)
constexpr uint32_t CKR = 8;     // checkpoints kept per replica
constexpr uint32_t NO_ID = 0xFFu;
constexpr uint32_t LANES = 64;

constexpr uint32_t E_EXISTS = 1u, E_COMMIT = 2u, E_QUORUM = 4u;

enum { PUR_ORDER = 1, PUR_LINK = 2, PUR_SLOWD = 3, PUR_FLAKY = 4 };

// per-replica counter slots in Params::stats ([slot][r][C])
enum {
  ST_DELIV0 = 0,                    // 16 slots: delivered by message type
  ST_CLIENT = PAXISIM_NMSG,
  ST_SENT, ST_DROPPED, ST_DISCARDED, ST_COMMITS, ST_REPLIES,
  NSTAT
};

struct Params {
  uint32_t N, Z, W, M, D, NS, WK, max_requests;
  uint64_t C;            // allocated cluster lanes (multiple of 64)
  uint64_t clusters;     // live clusters
  uint64_t cluster_base, seed;
  uint32_t q1, q2, fz, thrifty, ephemeral, rwc, max_delay, nfaults;
  uint32_t drop_ppm, drop_len, slow_ppm, slow_len, slow_min, slow_max;
  uint32_t npz[PAXISIM_MAX_ZONES], zmask[PAXISIM_MAX_ZONES];
  uint32_t target[PAXISIM_MAX_WORKERS];
  const paxisim_fault* faults;
  // replica scalars [r][C]
  uint32_t *ballot, *slot, *execute, *meta, *flags, *npend, *nfwd;
  uint64_t* digest;
  // per-cluster [C]
  uint64_t* kc;
  uint32_t* poison;
  // dynamic tables
  uint32_t* pend;        // [PMAX][N][C]
  uint32_t* fwd;         // [FMAX][N][C]
  uint32_t *drop_until, *slow_until, *slow_delay;  // [dst][N][C]
  uint32_t* ck_e;        // [CKR][N][C]
  uint64_t* ck_d;        // [CKR][N][C]
  uint32_t* stats;       // [NSTAT][N][C]
  uint32_t *wk_cur, *wk_issued;  // [WK][C]
  uint4* log;            // [N][C][W]
  uint4* rec;            // [D][N dst][NS src][M][C]
  uint8_t* cnt;          // [D][N dst][NS src][C]
};

// ---- PRNG ------------------------------------------------
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z ^= z >> 30; z *= 0xbf58476d1ce4e5b9ULL;
  z ^= z >> 27; z *= 0x94d049bb133111ebULL;
  z ^= z >> 31;
  return z;
}
__host__ __device__ __forceinline__ uint64_t cluster_key(uint64_t seed, uint64_t gid) {
  return mix64(seed ^ mix64(gid + 0x9E3779B97F4A7C15ULL));
}
__device__ __forceinline__ uint64_t draw(uint64_t kc, uint32_t t, uint32_t tag) {
  return mix64(kc ^ mix64(((uint64_t)t << 32) | tag));
}
__device__ __forceinline__ uint32_t tag(uint32_t p, uint32_t a, uint32_t b) {
  return (p << 28) | (a << 20) | b;
}
__device__ __forceinline__ bool ppm_hit(uint32_t x, uint32_t ppm) {
  return __umulhi(x, 1000000u) < ppm;
}

// ---- ballots: (n << 4) | replica, 0 = none (ballot.go:12-52) -------------
__device__ __forceinline__ uint32_t bal_id(uint32_t b) { return b ? (b & 15u) : NO_ID; }
__device__ __forceinline__ uint32_t bal_next(uint32_t b, uint32_t self) {
  return (((b >> 4) + 1u) << 4) | self;
}

// ---- requests: cid | origin << 27 (message.go:24-30) ---------------------
__device__ __forceinline__ uint32_t req_cid(uint32_t q) { return q & 0x07FFFFFFu; }
__device__ __forceinline__ uint32_t req_origin(uint32_t q) { return q >> 27; }
__device__ __forceinline__ uint32_t mkreq(uint32_t cid, uint32_t o) { return cid | (o << 27); }

// ---- message records: {hdr = type | n << 8, ballot, slot, cid} ------------
__device__ __forceinline__ uint32_t hdr_type(uint32_t h) { return h & 0xFFu; }
__device__ __forceinline__ uint32_t hdr_n(uint32_t h) { return h >> 8; }

// ---- quorum predicates on an ack mask (quorum.go:55-119) -----------------
__device__ __forceinline__ bool quorum_ok(const Params& P, uint32_t kind, uint32_t mask) {
  const int size = __popc(mask);
  uint32_t zones_any = 0, zones_maj = 0;
  bool col = false;
  for (uint32_t z = 0; z < P.Z; z++) {
    const uint32_t c = (uint32_t)__popc(mask & P.zmask[z]);
    zones_any += c > 0;
    zones_maj += c > P.npz[z] / 2;
    col |= c == P.npz[z];
  }
  switch (kind) {
    case PAXISIM_Q_MAJORITY: return size > (int)(P.N / 2);
    case PAXISIM_Q_ALL: return size == (int)P.N;
    case PAXISIM_Q_FAST: return size >= (int)(P.N * 3 / 4);
    case PAXISIM_Q_GRID_ROW: return zones_any == P.Z;
    case PAXISIM_Q_ZONE_MAJORITY: return zones_maj > 0;
    case PAXISIM_Q_GRID_COLUMN: return col;
    case PAXISIM_Q_FGRID_Q1: return (int)zones_maj >= (int)P.Z - (int)P.fz;
    case PAXISIM_Q_FGRID_Q2: return (int)zones_maj >= (int)P.fz + 1;
  }
  return false;
}

// ---- scripted faults (uniform across the wave: scalar loads) -------------
__device__ __forceinline__ bool scripted(const Params& P, uint32_t kind, uint64_t gid, uint32_t src,
                                         uint32_t dst, uint32_t t, uint32_t* param) {
  bool hit = false;
  for (uint32_t i = 0; i < P.nfaults; i++) {
    const paxisim_fault f = P.faults[i];
    if (f.kind != kind || f.src != src) continue;
    if (kind != PAXISIM_FAULT_CRASH && f.dst != PAXISIM_ALL_DST && f.dst != dst) continue;
    if (gid < f.cluster_lo || gid >= f.cluster_hi) continue;
    if (t < f.step_from || t >= f.step_to) continue;
    hit = true;
    if (param && f.param > *param) *param = f.param;
  }
  return hit;
}

// ---- SoA addressing --------------------------------------------------------
__device__ __forceinline__ size_t rc(const Params& P, uint32_t r, uint64_t c) { return (size_t)r * P.C + c; }
__device__ __forceinline__ size_t krc(const Params& P, uint32_t k, uint32_t r, uint64_t c) {
  return ((size_t)k * P.N + r) * P.C + c;
}
__device__ __forceinline__ uint4* log_at(const Params& P, uint32_t r, uint64_t c, int32_t s) {
  return &P.log[((size_t)r * P.C + c) * P.W + ((uint32_t)s & (P.W - 1u))];
}
__device__ __forceinline__ size_t box(const Params& P, uint32_t b, uint32_t dst, uint32_t src) {
  return ((size_t)b * P.N + dst) * P.NS + src;
}
__device__ __forceinline__ uint4* rec_at(const Params& P, size_t bx, uint32_t k, uint64_t c) {
  return &P.rec[(bx * P.M + k) * P.C + c];
}
__device__ __forceinline__ uint8_t* cnt_at(const Params& P, size_t bx, uint64_t c) {
  return &P.cnt[bx * P.C + c];
}

}  // namespace pxs
