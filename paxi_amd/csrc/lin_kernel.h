// lin_kernel.h — History.Linearizable on gfx950 (history.go:55-71), no size cap.
//
// The reference's checker (checker.go:69-104, lib/graph.go:180-232) runs on
// every (cluster, key) partition of the completed-operation history:
//   ops stable-sorted by start (sort.Sort(byTime)); add() draws happens-before
//   edges into each new vertex; a read looks ahead for concurrent writes, is
//   merged into the first vertex holding the value it returned, and Cycle()
//   (a DFS over the vertices) reports an anomaly, after which the edges u->v
//   with u.start > v.end among the DFS path's vertices are removed.
// Vertices are iterated in insertion order where Go ranges over a map (the
// oracle does the same), so a vertex is named by its insertion
// number and "the first vertex in insertion order" is the lowest set bit.
//
// One wave checks one partition.  The adjacency matrix is a bit matrix with
// one row of nw = ceil(cap/64) u64 words per vertex; bit sets that a DFS or a
// search reads whole (present, gray, black, reach frontier) are spread one
// word per lane (lane w holds word w), so a row scan is one load per lane and
// a ballot.  Per read the wave pays O(n/64) for add/match/merge; Cycle() runs
// only when the graph can hold a cycle:
//   - add() gives the new vertex only incoming edges, so it never closes one;
//   - merge(read, w) adds edges s->w, so an acyclic graph gains a cycle iff w
//     reaches itself afterwards: a breadth-first reach from w over the rows;
//   - after an anomaly the graph may still be cyclic, and then Cycle() runs at
//     every read until it finds none, as in the reference.
// When a cycle exists the exact insertion-order DFS runs, so the removed
// edges are exactly the reference's.
//
// lin_cluster_kernel: one workgroup per cluster.  Its LIN_LW waves read the
// cluster's history once (a pass over the key words, then one over the ops)
// and write it to an HBM stage grouped by key, each key in canonical order
// (replica 0's ops, then replica 1's, ... each in completion order: per-wave
// counts and a stable ballot-ranked placement); then they take the keys in
// turn and check partitions of up to LIN_SMAX ops in LDS.  Larger ones go to
// a list that lin_big_kernel checks with the same code on an HBM scratch.
#pragma once
#include "paxisim_dev.h"

namespace pxs {

// PXS_LIN_STAMPS (diagnostic build): s_memtime cycles of the checker's phases,
// summed over waves into out[LIN_NOUT + k] (paxisim_linearizable prints them)
#ifdef PXS_LIN_STAMPS
__device__ __forceinline__ uint32_t lin_now() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return (uint32_t)t;
}
#define LIN_T0(v) const uint32_t v = lin_now();
#define LIN_T1(v, k) lst[k] += lin_now() - v;
#else
#define LIN_T0(v)
#define LIN_T1(v, k)
#endif
enum { LS_P1 = 0, LS_P2, LS_SORT, LS_RUN, LS_ADD, LS_LOOK, LS_MERGE, LS_REACH };

#ifndef PXS_LIN_LW
#define PXS_LIN_LW 2   // (A/B r4w, config 3 scan: 2 waves 0.926 s, 4 waves 0.962 s, 8 waves 1.079 s)
#endif
constexpr uint32_t LIN_LW = PXS_LIN_LW;    // waves per cluster workgroup
#ifndef PXS_LIN_MINW
// waves per SIMD the cluster kernel's registers must allow.  A/B r4t: 8 waves
// (64 VGPRs, 9 spilled) 0.99 -> 0.96 s; round 5 (the cyclic-state shortcut's
// fields, gpurun_out/r5c/ab_lin): 8 waves spill 40 VGPRs and scan in 0.82 s,
// 7 waves (72 VGPRs, 16 spilled) 0.49 s, 6 (80, 2) 0.50 s, 5 (84, 0) 0.52 s
#define PXS_LIN_MINW 7
#endif
constexpr uint32_t LIN_SMAX = 128;         // partitions checked in LDS by the cluster kernel
constexpr uint32_t LIN_WPL_MAX = 4;        // bit-set words per lane: up to 4096 * 4 vertices
constexpr uint32_t LIN_VMAX = 4096u * LIN_WPL_MAX;   // larger partitions are counted as skipped
constexpr uint16_t LIN_NOV = 0xFFFFu;      // sorted op not (yet) a vertex
constexpr uint32_t LIN_SORT_BYTES = LIN_SMAX * (16u + 4u);   // cluster kernel, per wave: sorted ops + start copies
enum { LIN_ANOM = 0, LIN_OPS, LIN_BIG, LIN_NMAX, LIN_PARTS, LIN_SKIP, LIN_NOUT = 8 };

// A wave's scratch for one partition of capacity cap = 64 * nw ops (cap <=
// LIN_VMAX: vertex ids and DFS resume positions fit 16 bits).
struct LinScratch {
  uint4* ops;        // [cap] sorted by start: {key | write << 31, value, start, end (refined)}
  uint16_t* vid;     // [cap] sorted index -> vertex (insertion number) or LIN_NOV
  uint16_t* opv;     // [cap] vertex -> sorted index
  uint32_t* vst;     // [cap] vertex start
  uint32_t* ven;     // [cap] vertex end (refined by merges)
  uint32_t* vvl;     // [cap] vertex value | write << 31
  uint32_t* stk;     // [cap] DFS stack: vertex | resume position << 16
  uint64_t* rows;    // [cap][nw] successor bit rows
  uint32_t nw;
};
__host__ __device__ inline size_t lin_scratch_bytes(uint32_t nw, bool) {
  const size_t cap = 64u * (size_t)nw;
  return cap * (16u + 2u + 2u + 4u * 4u) + cap * nw * 8u;
}
__device__ inline LinScratch lin_scratch(uint8_t* p, uint32_t nw, bool) {
  const size_t cap = 64u * (size_t)nw;
  LinScratch s;
  s.rows = reinterpret_cast<uint64_t*>(p); p += cap * nw * 8u;
  s.ops = reinterpret_cast<uint4*>(p); p += cap * 16u;
  s.vst = reinterpret_cast<uint32_t*>(p); p += cap * 4u;
  s.ven = reinterpret_cast<uint32_t*>(p); p += cap * 4u;
  s.vvl = reinterpret_cast<uint32_t*>(p); p += cap * 4u;
  s.stk = reinterpret_cast<uint32_t*>(p); p += cap * 4u;
  s.vid = reinterpret_cast<uint16_t*>(p); p += cap * 2u;
  s.opv = reinterpret_cast<uint16_t*>(p);
  s.nw = nw;
  return s;
}

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }
// A lane-distributed bit set of up to 4096 * WPL bits: word w lives in lane
// w & 63, element w >> 6 of that lane's array (wave-uniform w).
template <int WPL>
struct LSet {
  uint64_t m[WPL];
  __device__ __forceinline__ static LSet zero() {
    LSet r;
#pragma unroll
    for (int j = 0; j < WPL; j++) r.m[j] = 0;
    return r;
  }
  __device__ __forceinline__ LSet operator&(const LSet& o) const {
    LSet r;
#pragma unroll
    for (int j = 0; j < WPL; j++) r.m[j] = m[j] & o.m[j];
    return r;
  }
  __device__ __forceinline__ LSet operator~() const {
    LSet r;
#pragma unroll
    for (int j = 0; j < WPL; j++) r.m[j] = ~m[j];
    return r;
  }
  __device__ __forceinline__ LSet& operator|=(const LSet& o) {
#pragma unroll
    for (int j = 0; j < WPL; j++) m[j] |= o.m[j];
    return *this;
  }
  __device__ __forceinline__ bool lane_any() const {
    uint64_t v = 0;
#pragma unroll
    for (int j = 0; j < WPL; j++) v |= m[j];
    return v != 0;
  }
  __device__ __forceinline__ uint64_t elem(uint32_t j) const {   // m[j], j wave-uniform
    uint64_t v = m[0];
#pragma unroll
    for (int k = 1; k < WPL; k++) v = j == (uint32_t)k ? m[k] : v;
    return v;
  }
  // word w := v on its lane
  __device__ __forceinline__ void put_word(uint32_t w, uint64_t v) {
    if (lane_id() != (w & 63u)) return;
#pragma unroll
    for (int k = 0; k < WPL; k++)
      if ((w >> 6) == (uint32_t)k) m[k] = v;
  }
};
// word w of a lane-distributed bit set (wave-uniform w)
template <int WPL>
__device__ __forceinline__ uint64_t mword(const LSet<WPL>& s, uint32_t w) {
  const uint64_t m = s.elem(w >> 6);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)m, (int)(w & 63u));
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(m >> 32), (int)(w & 63u));
  return (uint64_t)lo | ((uint64_t)hi << 32);
}
template <int WPL>
__device__ __forceinline__ bool mbit(const LSet<WPL>& s, uint32_t v) { return (mword(s, v >> 6) >> (v & 63u)) & 1u; }
template <int WPL>
__device__ __forceinline__ LSet<WPL> mset(LSet<WPL> s, uint32_t v) {
  const uint32_t w = v >> 6;
  if (lane_id() == (w & 63u)) {
#pragma unroll
    for (int k = 0; k < WPL; k++)
      if ((w >> 6) == (uint32_t)k) s.m[k] |= 1ull << (v & 63u);
  }
  return s;
}
template <int WPL>
__device__ __forceinline__ LSet<WPL> mclr(LSet<WPL> s, uint32_t v) {
  const uint32_t w = v >> 6;
  if (lane_id() == (w & 63u)) {
#pragma unroll
    for (int k = 0; k < WPL; k++)
      if ((w >> 6) == (uint32_t)k) s.m[k] &= ~(1ull << (v & 63u));
  }
  return s;
}
// OR over the wave's 64 lanes, uniform result.  DPP row shifts fold each row of
// 16 lanes into its lane 15, row_bcast:15 / row_bcast:31 carry those into lane
// 63, and one readlane broadcasts it: VALU ops only (a __shfl_xor ladder is
// six ds_bpermute round trips through the LDS crossbar per 32-bit half).
__device__ __forceinline__ uint32_t or_reduce32(uint32_t v) {
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);   // row_shr:1
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);   // row_shr:2
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);   // row_shr:4
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);   // row_shr:8
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);   // row_bcast:15
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);   // row_bcast:31
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
__device__ __forceinline__ uint64_t or_reduce(uint64_t v) {
  return (uint64_t)or_reduce32((uint32_t)v) | ((uint64_t)or_reduce32((uint32_t)(v >> 32)) << 32);
}
__device__ __forceinline__ uint32_t first_lane(uint64_t ballot) { return (uint32_t)__builtin_ctzll(ballot); }
__device__ __forceinline__ uint64_t readlane64(uint64_t v, uint32_t l) {
  return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)l) |
         ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), (int)l) << 32);
}

// The checker over one partition held in s.ops[0, n) (sorted).  Returns the
// number of anomalous reads (checker.go:97: len(anomaly)).  Lanes write what
// other lanes read next (rows, vertex fields, the DFS stack): LDS serves one
// wave's accesses in order; with the scratch in HBM (G) a fence orders them.
template <bool G, int WPL>
struct LinCheck {
  using Set = LSet<WPL>;
  LinScratch s;
  uint32_t n, nv;       // ops, vertices inserted so far
  Set present;          // lane-distributed vertex set
  Set writes;           // lane-distributed: vertices that are writes (have an input)
  __device__ __forceinline__ void sync() const {
    if (G) __threadfence_block();
  }
  __device__ __forceinline__ bool hb_ops(uint32_t a, uint32_t b) const {   // operation.go:12-14 on sorted ops
    return s.ops[a].w < s.ops[b].z;
  }
  // checker.add (checker.go:21-33): edges v -> o from every vertex that happened before o
  __device__ void add(uint32_t o) {
    if (s.vid[o] != LIN_NOV) return;                     // already in graph from lookahead
    const uint4 op = s.ops[o];
    const uint32_t id = nv++;
    if (lane_id() == 0) {
      s.vid[o] = (uint16_t)id;
      s.opv[id] = (uint16_t)o;
      s.vst[id] = op.z;
      s.ven[id] = op.w;
      s.vvl[id] = op.y;
    }
    for (uint32_t w = lane_id(); w < s.nw; w += 64u) s.rows[(size_t)id * s.nw + w] = 0;
    present = mset(present, id);
    if (op.x >> 31) writes = mset(writes, id);
    for (uint32_t b = 0; b < id; b += 64u) {             // the new vertex is not before itself
      const uint32_t v = b + lane_id();
      const uint64_t pw = mword(present, b >> 6);
      if (v < id && ((pw >> (v & 63u)) & 1u) && s.ven[v] < op.z)
        s.rows[(size_t)v * s.nw + (id >> 6)] |= 1ull << (id & 63u);
    }
    sync();
  }
  // graph.Remove (graph.go:36-48)
  __device__ void remove(uint32_t r) {
    present = mclr(present, r);
    for (uint32_t w = lane_id(); w < s.nw; w += 64u) s.rows[(size_t)r * s.nw + w] = 0;
    for (uint32_t b = 0; b < nv; b += 64u) {
      const uint32_t v = b + lane_id();
      if (v < nv) s.rows[(size_t)v * s.nw + (r >> 6)] &= ~(1ull << (r & 63u));
    }
    sync();
  }
  // match (checker.go:44-52): the first vertex whose input equals the read's
  // output (a read has no input: only writes match a read's value)
  __device__ uint32_t match(uint32_t out) const {
    for (uint32_t b = 0; b < nv; b += 64u) {
      const uint32_t v = b + lane_id();
      const uint64_t pw = mword(present & writes, b >> 6);
      const bool hit = v < nv && ((pw >> (v & 63u)) & 1u) && s.vvl[v] == out;
      const uint64_t m = __ballot(hit);
      if (m) return b + first_lane(m);
    }
    return LIN_NOV;
  }
  // merge (checker.go:55-67): the write inherits the read's incoming edges
  __device__ void merge(uint32_t r, uint32_t m) {
    for (uint32_t b = 0; b < nv; b += 64u) {
      const uint32_t v = b + lane_id();
      if (v < nv && v != m && ((s.rows[(size_t)v * s.nw + (r >> 6)] >> (r & 63u)) & 1u))
        s.rows[(size_t)v * s.nw + (m >> 6)] |= 1ull << (m & 63u);
    }
    if (lane_id() == 0 && s.ven[r] < s.ven[m]) {         // refine response time of the merged vertex
      s.ven[m] = s.ven[r];
      s.ops[s.opv[m]].w = s.ven[r];
    }
    sync();
    remove(r);
  }
  // Does m reach itself?  Breadth-first over the rows, one word a lane.
  __device__ bool reaches_self(uint32_t m) const {
    Set R = mset(Set::zero(), m), F = R;
    for (;;) {
      Set nx = Set::zero();
      for (uint32_t w = 0; w < s.nw; w++) {
        uint64_t acc = 0;
        for (uint32_t b = 0; b < nv; b += 64u) {
          const uint64_t fw = mword(F, b >> 6);
          if (!fw) continue;
          const uint32_t v = b + lane_id();
          if ((fw >> (v & 63u)) & 1u) acc |= s.rows[(size_t)v * s.nw + w];
        }
        acc = or_reduce(acc);
        if (w == (m >> 6) && ((acc >> (m & 63u)) & 1u)) return true;
        nx.put_word(w, acc);
      }
      nx = nx & present & ~R;
      if (!__ballot(nx.lane_any())) return false;
      R |= nx;
      F = nx;
    }
  }
  // Cycle() (graph.go:212-232): DFS from each white vertex in insertion order,
  // visit (180-193) walking successors in insertion order; on a back edge the
  // gray vertices (the DFS path) are returned in `gray`.
  __device__ bool cycle(Set& gray) const {
    Set black = Set::zero();
    gray = Set::zero();
    for (uint32_t rb = 0; rb < nv; rb += 64u) {
      uint64_t roots = mword(present & ~black, rb >> 6);
      while (roots) {
        const uint32_t root = rb + (uint32_t)__builtin_ctzll(roots);
        roots &= roots - 1u;
        if (mbit(black, root)) continue;                 // reached from an earlier root
        uint32_t sp = 0, v = root, k = 0;
        gray = mset(gray, root);
        for (;;) {
          // the first successor u >= k of v that is not black: word j*64 + lane
          uint32_t u = ~0u;
#pragma unroll
          for (int j = 0; j < WPL; j++) {
            const uint32_t w = (uint32_t)j * 64u + lane_id();
            uint64_t c = 0;
            if (w < s.nw && w * 64u + 63u >= k) {
              c = s.rows[(size_t)v * s.nw + w] & ~black.m[j];
              if (w * 64u < k) c &= ~0ull << (k - w * 64u);
            }
            const uint64_t bl = __ballot(c != 0);
            if (bl) {
              const uint32_t f = first_lane(bl);
              u = ((uint32_t)j * 64u + f) * 64u + (uint32_t)__builtin_ctzll(readlane64(c, f));
              break;
            }
          }
          if (u == ~0u) {                                // v done: black, back to its parent
            gray = mclr(gray, v);
            black = mset(black, v);
            if (sp == 0) break;
            const uint32_t top = s.stk[--sp];
            v = top & 0xFFFFu;
            k = top >> 16;
            continue;
          }
          if (mbit(gray, u)) return true;
          if (lane_id() == 0) s.stk[sp] = v | ((u + 1u) << 16);
          sync();
          sp++;
          gray = mset(gray, u);
          v = u;
          k = 0;
        }
      }
    }
    return false;
  }
  // checker.go:93-100: remove the edges u->v between gray vertices with u.start > v.end
  __device__ void cut(const Set& gray) {
    for (uint32_t b = 0; b < nv; b += 64u) {
      const uint32_t u = b + lane_id();
      const uint64_t gw = mword(gray, b >> 6);
      if (u >= nv || !((gw >> (u & 63u)) & 1u)) continue;
      const uint32_t su = s.vst[u];
      for (uint32_t w = 0; w < s.nw; w++) {
        uint64_t e = s.rows[(size_t)u * s.nw + w] & mword(gray, w), keep = ~0ull;
        while (e) {
          const uint32_t t = (uint32_t)__builtin_ctzll(e);
          e &= e - 1u;
          if (su > s.ven[w * 64u + t]) keep &= ~(1ull << t);
        }
        if (keep != ~0ull) s.rows[(size_t)u * s.nw + w] &= keep;
      }
    }
    sync();
  }
  // checker.linearizable (checker.go:69-104) over the sorted ops
  __device__ uint32_t run() {
    nv = 0;
    present = writes = Set::zero();
    for (uint32_t i = lane_id(); i < n; i += 64u) s.vid[i] = LIN_NOV;
    sync();
    bool maybe_cyclic = false;
    uint32_t anomalies = 0;
    for (uint32_t i = 0; i < n; i++) {
      add(i);
      const uint4 o = s.ops[i];
      if (o.x >> 31) continue;                           // a write: nothing more
      for (uint32_t j = i + 1; j < n && !hb_ops(i, j) && !hb_ops(j, i); j++)   // look ahead
        if (s.ops[j].x >> 31) add(j);                    // concurrent writes
      const uint32_t r = s.vid[i];
      const uint32_t m = match(o.y);
      if (m != LIN_NOV) merge(r, m);
      bool cyc = false;
      Set gray;
      const bool was_cyclic = maybe_cyclic;
      if (maybe_cyclic) cyc = cycle(gray);
      else if (m != LIN_NOV && reaches_self(m)) cyc = cycle(gray);
      if (cyc) {
        anomalies++;
        cut(gray);
        // still cyclic: Cycle() at every read.  When the graph was acyclic
        // before this read's merge, every cycle runs through the merged vertex
        // m (the merge's edges s -> m are the only new ones), so a reach from
        // m decides it; otherwise the full DFS does.
        if (!was_cyclic) {
          maybe_cyclic = reaches_self(m);
        } else {
          Set g2;
          maybe_cyclic = cycle(g2);
        }
      } else {
        maybe_cyclic = false;
      }
    }
    return anomalies;
  }
};

// ---------------------------------------------------------------------------
// LinReg: the same checker for partitions of at most 128 ops with the whole
// graph in registers.  Lane l owns vertices l and 64 + l (slot j = v >> 6):
// their successor rows (2 x 2 words), start, refined end and value; the sorted
// ops are held the same way (op o at lane o & 63, slot o >> 6).  Vertex sets
// are two wave-uniform words.  A DFS step then reads a row with four
// readlanes and works on scalars, add / merge / remove / cut are one pass of
// per-lane register work, and nothing touches LDS after the sort - where
// LinCheck pays an LDS round trip per dependent access (round-4 profile:
// lin_cluster_kernel 1.26 s for config 3's 1.68 G ops).  The semantics are
// LinCheck's line for line (checker.go:69-104, lib/graph.go:180-232).
// ---------------------------------------------------------------------------
// two-word vertex set / row (v < 128): explicit fields, no dynamically indexed arrays
struct B2 {
  uint64_t lo, hi;
  __device__ __forceinline__ uint64_t w(uint32_t i) const { return i ? hi : lo; }
  __device__ __forceinline__ bool has(uint32_t v) const { return ((v >> 6 ? hi : lo) >> (v & 63u)) & 1u; }
  // (value selects, not a selected field: a store through a selected pointer
  // would put the owning struct in scratch memory)
  __device__ __forceinline__ void set(uint32_t v) {
    const uint64_t b = 1ull << (v & 63u);
    const bool h = (v >> 6) != 0;
    lo |= h ? 0ull : b;
    hi |= h ? b : 0ull;
  }
  __device__ __forceinline__ void clr(uint32_t v) {
    const uint64_t b = ~(1ull << (v & 63u));
    const bool h = (v >> 6) != 0;
    lo &= h ? ~0ull : b;
    hi &= h ? b : ~0ull;
  }
  __device__ __forceinline__ bool any() const { return (lo | hi) != 0; }
};
__device__ __forceinline__ B2 b2(uint64_t lo, uint64_t hi) { B2 r; r.lo = lo; r.hi = hi; return r; }

struct LinReg {
  // per lane, slot j in {0, 1} (fields suffixed 0 / 1)
  uint4 op0, op1;            // sorted op j*64+lane: {key | write << 31, value, start, end (refined)}
  uint32_t vid0, vid1;       // sorted op -> vertex, or LIN_NOV
  B2 row0, row1;             // successor rows of vertex j*64+lane
  uint32_t vst0, vst1, ven0, ven1, vvl0, vvl1, opv0, opv1;
  // a lower bound of the (refined) ends of the vertex's successors: an edge
  // u -> t with u.start > t.end - the only kind cut() removes - can exist only
  // where vst > msc (run(): the cyclic-state shortcut)
  uint32_t msc0, msc1;
  uint32_t stk0, stk1;       // DFS stack entry sp at lane sp & 63, slot sp >> 6
  // wave-uniform
  B2 present, writes;
  uint32_t n, nv;
#ifdef PXS_LIN_STAMPS
  uint32_t lst[8];
#endif

  __device__ __forceinline__ static uint32_t rl(uint32_t v, uint32_t l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
  }
  // slot select of a lane field; the asm barriers keep LLVM from turning the
  // select of two fields into a load through a selected pointer (which puts
  // the whole struct in scratch memory)
  __device__ __forceinline__ static uint32_t pick(uint32_t i, uint32_t a0, uint32_t a1) {
    asm volatile("" : "+v"(a0), "+v"(a1));
    return (i >> 6) ? a1 : a0;
  }
  __device__ __forceinline__ static uint64_t pick64(uint32_t i, uint64_t a0, uint64_t a1) {
    asm volatile("" : "+v"(a0), "+v"(a1));
    return (i >> 6) ? a1 : a0;
  }
  __device__ __forceinline__ uint32_t op_x(uint32_t o) const { return rl(pick(o, op0.x, op1.x), o & 63u); }
  __device__ __forceinline__ uint32_t op_y(uint32_t o) const { return rl(pick(o, op0.y, op1.y), o & 63u); }
  __device__ __forceinline__ uint32_t op_z(uint32_t o) const { return rl(pick(o, op0.z, op1.z), o & 63u); }
  __device__ __forceinline__ uint32_t op_w(uint32_t o) const { return rl(pick(o, op0.w, op1.w), o & 63u); }
  __device__ __forceinline__ uint32_t vid_of(uint32_t o) const { return rl(pick(o, vid0, vid1), o & 63u); }
  __device__ __forceinline__ uint32_t ven_of(uint32_t v) const { return rl(pick(v, ven0, ven1), v & 63u); }
  __device__ __forceinline__ bool hb_ops(uint32_t a, uint32_t b) const { return op_w(a) < op_z(b); }   // operation.go:12-14
  __device__ __forceinline__ uint64_t row_of(uint32_t v, uint32_t w) const {   // word w of vertex v's row
    return readlane64(w ? pick64(v, row0.hi, row1.hi) : pick64(v, row0.lo, row1.lo), v & 63u);
  }

  // the sorted ops of the partition from the wave's LDS sort buffer
  __device__ __forceinline__ void load(const uint4* sorted, uint32_t cnt) {
    n = cnt;
    nv = 0;
    present = b2(0, 0);
    writes = b2(0, 0);
    const uint32_t l = lane_id();
    op0 = l < n ? sorted[l] : make_uint4(0u, 0u, 0u, 0u);
    op1 = l + 64u < n ? sorted[l + 64u] : make_uint4(0u, 0u, 0u, 0u);
    vid0 = vid1 = LIN_NOV;
    row0 = b2(0, 0);
    row1 = b2(0, 0);
    vst0 = vst1 = ven0 = ven1 = vvl0 = vvl1 = opv0 = opv1 = 0;
    msc0 = msc1 = ~0u;
    stk0 = stk1 = 0;
  }
  // checker.add (checker.go:21-33)
  __device__ __forceinline__ void add(uint32_t o) {
    if (vid_of(o) != LIN_NOV) return;
    const uint32_t oz = op_z(o), ow = op_w(o), oy = op_y(o), ox = op_x(o);
    const uint32_t id = nv++;
    const uint32_t l = lane_id();
    const bool own_o = l == (o & 63u), own_id = l == (id & 63u);
    vid0 = own_o && !(o >> 6) ? id : vid0;
    vid1 = own_o && (o >> 6) ? id : vid1;
    const bool n0 = own_id && !(id >> 6), n1 = own_id && (id >> 6);
    vst0 = n0 ? oz : vst0; ven0 = n0 ? ow : ven0; vvl0 = n0 ? oy : vvl0; opv0 = n0 ? o : opv0;
    vst1 = n1 ? oz : vst1; ven1 = n1 ? ow : ven1; vvl1 = n1 ? oy : vvl1; opv1 = n1 ? o : opv1;
    row0.lo = n0 ? 0ull : row0.lo; row0.hi = n0 ? 0ull : row0.hi;
    row1.lo = n1 ? 0ull : row1.lo; row1.hi = n1 ? 0ull : row1.hi;
    msc0 = n0 ? ~0u : msc0; msc1 = n1 ? ~0u : msc1;
    // v -> id for every present vertex that ended before o started (id is not yet present)
    if (l < id && present.has(l) && ven0 < oz) { row0.set(id); msc0 = min(msc0, ow); }
    if (l + 64u < id && present.has(l + 64u) && ven1 < oz) { row1.set(id); msc1 = min(msc1, ow); }
    present.set(id);
    if (ox >> 31) writes.set(id);
  }
  // graph.Remove (graph.go:36-48)
  __device__ __forceinline__ void remove(uint32_t r) {
    present.clr(r);
    const uint32_t l = lane_id();
    const bool z0 = l == (r & 63u) && !(r >> 6), z1 = l == (r & 63u) && (r >> 6);
    row0.lo = z0 ? 0ull : row0.lo; row0.hi = z0 ? 0ull : row0.hi;
    row1.lo = z1 ? 0ull : row1.lo; row1.hi = z1 ? 0ull : row1.hi;
    row0.clr(r);
    row1.clr(r);
  }
  // match (checker.go:44-52): the first write vertex in insertion order holding the value
  __device__ __forceinline__ uint32_t match(uint32_t out) const {
    const uint32_t l = lane_id();
    const uint64_t m0 = __ballot(l < nv && present.has(l) && writes.has(l) && vvl0 == out);
    if (m0) return first_lane(m0);
    const uint64_t m1 = __ballot(l + 64u < nv && present.has(l + 64u) && writes.has(l + 64u) && vvl1 == out);
    if (m1) return 64u + first_lane(m1);
    return LIN_NOV;
  }
  // merge (checker.go:55-67)
  __device__ __forceinline__ void merge(uint32_t r, uint32_t m) {
    const uint32_t l = lane_id();
    const uint32_t er = ven_of(r), em = ven_of(m), emin = er < em ? er : em;
    // the edges into m (old, and the read's inherited ones) now end at emin
    if (l < nv && l != m && (row0.has(r) || row0.has(m))) msc0 = min(msc0, emin);
    if (l + 64u < nv && l + 64u != m && (row1.has(r) || row1.has(m))) msc1 = min(msc1, emin);
    if (l < nv && l != m && row0.has(r)) row0.set(m);
    if (l + 64u < nv && l + 64u != m && row1.has(r)) row1.set(m);
    if (er < em) {                                        // refine the merged vertex's response time
      const uint32_t om = rl(pick(m, opv0, opv1), m & 63u);
      ven0 = l == (m & 63u) && !(m >> 6) ? er : ven0;
      ven1 = l == (m & 63u) && (m >> 6) ? er : ven1;
      op0.w = l == (om & 63u) && !(om >> 6) ? er : op0.w;
      op1.w = l == (om & 63u) && (om >> 6) ? er : op1.w;
    }
    remove(r);
  }
  // Does m reach itself?  Breadth-first over the rows of the frontier.
  __device__ __forceinline__ bool reaches_self(uint32_t m) const {
    const uint32_t l = lane_id();
    B2 R = b2(0, 0);
    R.set(m);
    B2 F = R;
    for (;;) {
      uint64_t a0 = 0, a1 = 0;
      if (F.has(l)) { a0 |= row0.lo; a1 |= row0.hi; }
      if (F.has(l + 64u)) { a0 |= row1.lo; a1 |= row1.hi; }
      B2 nx = b2(or_reduce(a0), or_reduce(a1));
      if (nx.has(m)) return true;
      nx.lo &= present.lo & ~R.lo;
      nx.hi &= present.hi & ~R.hi;
      if (!nx.any()) return false;
      R.lo |= nx.lo; R.hi |= nx.hi;
      F = nx;
    }
  }
  // Cycle() (graph.go:212-232): DFS from each white vertex in insertion order,
  // visit (180-193) walking successors in insertion order; on a back edge the
  // gray vertices (the DFS path) are returned in `gray`.
  __device__ __forceinline__ bool cycle(B2& gray) {
    B2 black = b2(0, 0);
    gray = b2(0, 0);
    const uint32_t l = lane_id();
    for (uint32_t rb = 0; rb < 2; rb++) {
      uint64_t roots = present.w(rb) & ~black.w(rb);
      while (roots) {
        const uint32_t root = rb * 64u + (uint32_t)__builtin_ctzll(roots);
        roots &= roots - 1u;
        if (black.has(root)) continue;                   // reached from an earlier root
        uint32_t sp = 0, v = root, k = 0;
        gray.set(root);
        for (;;) {
          // the first successor u >= k of v that is not black
          uint32_t u = ~0u;
          if (k < 64u) {
            uint64_t c = row_of(v, 0) & ~black.lo;
            c &= ~0ull << k;
            if (c) u = (uint32_t)__builtin_ctzll(c);
          }
          if (u == ~0u) {
            uint64_t c = row_of(v, 1) & ~black.hi;
            if (k >= 128u) c = 0;                       // resumed after vertex 127: no successor left
            else if (k > 64u) c &= ~0ull << (k - 64u);
            if (c) u = 64u + (uint32_t)__builtin_ctzll(c);
          }
          if (u == ~0u) {                                // v done: black, back to its parent
            gray.clr(v);
            black.set(v);
            if (sp == 0) break;
            --sp;
            const uint32_t top = rl(pick(sp, stk0, stk1), sp & 63u);
            v = top & 0xFFFFu;
            k = top >> 16;
            continue;
          }
          if (gray.has(u)) return true;
          const uint32_t e = v | ((u + 1u) << 16);
          stk0 = l == (sp & 63u) && !(sp >> 6) ? e : stk0;
          stk1 = l == (sp & 63u) && (sp >> 6) ? e : stk1;
          sp++;
          gray.set(u);
          v = u;
          k = 0;
        }
      }
    }
    return false;
  }
  // checker.go:93-100: remove the edges u->t between gray vertices with u.start > t.end;
  // returns whether any edge was removed
  __device__ __forceinline__ bool cut(const B2& gray) {
    const uint32_t l = lane_id();
    const bool g0 = gray.has(l), g1 = gray.has(l + 64u);
    bool ch = false;
    for (uint32_t w = 0; w < 2; w++) {
      for (uint64_t g = gray.w(w); g; g &= g - 1u) {
        const uint32_t t = w * 64u + (uint32_t)__builtin_ctzll(g);
        const uint32_t et = ven_of(t);
        if (g0 && vst0 > et && row0.has(t)) { row0.clr(t); ch = true; }
        if (g1 && vst1 > et && row1.has(t)) { row1.clr(t); ch = true; }
      }
    }
    return __ballot(ch) != 0;
  }
  // May the graph hold an edge u -> t with u.start > t.end (one cut() would remove)?
  __device__ __forceinline__ bool inverted_any() const {
    const uint32_t l = lane_id();
    return __ballot((present.has(l) && vst0 > msc0) || (present.has(l + 64u) && vst1 > msc1)) != 0;
  }
  // checker.linearizable (checker.go:69-104) over the sorted ops
  __device__ __forceinline__ uint32_t run() {
    bool maybe_cyclic = false;
    uint32_t anomalies = 0;
    for (uint32_t i = 0; i < n; i++) {
      LIN_T0(ta)
      add(i);
      LIN_T1(ta, LS_ADD)
      if (op_x(i) >> 31) continue;                       // a write: nothing more
      LIN_T0(tl)
      for (uint32_t j = i + 1; j < n && !hb_ops(i, j) && !hb_ops(j, i); j++)   // look ahead
        if (op_x(j) >> 31) add(j);                       // concurrent writes
      LIN_T1(tl, LS_LOOK)
      LIN_T0(tm)
      const uint32_t r = vid_of(i);
      const uint32_t m = match(op_y(i));
      if (m != LIN_NOV) merge(r, m);
      LIN_T1(tm, LS_MERGE)
      bool cyc = false;
      B2 gray = b2(0, 0);
      const bool was_cyclic = maybe_cyclic;
      LIN_T0(tr)
      // Cyclic-state shortcut (round 5).  Between checks the graph loses only
      // edges into the merged read, a sink, so a cycle found before is still
      // there and Cycle() finds one: an anomaly.  cut() then removes nothing
      // when no edge u -> t has u.start > t.end anywhere (msc), and the graph
      // stays cyclic - no DFS needed.  (Config 3: every cyclic-state read;
      // tools/lin_model.py: DFS steps 2.67 -> 0.08 per op, anomalies equal.)
      if (maybe_cyclic && !inverted_any()) {
        anomalies++;
        LIN_T1(tr, LS_REACH)
        continue;
      }
      if (maybe_cyclic) cyc = cycle(gray);
      else if (m != LIN_NOV && reaches_self(m)) cyc = cycle(gray);
      LIN_T1(tr, LS_REACH)
      if (cyc) {
        anomalies++;
        if (!cut(gray)) {
          maybe_cyclic = true;                            // the graph is the one just found cyclic
        } else if (!was_cyclic) {
          maybe_cyclic = reaches_self(m);
        } else {
          B2 g2;
          maybe_cyclic = cycle(g2);
        }
      } else {
        maybe_cyclic = false;
      }
    }
    return anomalies;
  }
};

// Stable sort of src[0, n) by start into s.ops (sort.Sort(byTime): ties keep
// canonical order): each op's rank counts the ops before it.
// The start times are first copied into the scratch's stack array (free
// until run()), so the n^2 rank comparisons read the scratch, not the stage.
template <bool G>
__device__ inline void lin_sort(const uint4* src, uint32_t n, LinScratch& s) {
  for (uint32_t i = lane_id(); i < n; i += 64u) s.stk[i] = src[i].z;
  if (G) __threadfence_block();
  __builtin_amdgcn_wave_barrier();
  for (uint32_t i = lane_id(); i < n; i += 64u) {
    const uint4 o = src[i];
    uint32_t rk = 0;
    for (uint32_t j = 0; j < n; j++) {
      const uint32_t sj = s.stk[j];
      rk += (sj < o.z || (sj == o.z && j < i)) ? 1u : 0u;
    }
    s.ops[rk] = o;
  }
  if (G) __threadfence_block();
}

// Canonical op index -> its history record (replica-major; len[r] ops each).
__device__ __forceinline__ const uint4* hist_at(const Params& P, uint64_t c, const uint32_t* len, uint32_t idx) {
  uint32_t r = 0;
  while (idx >= len[r]) idx -= len[r++];
  return &P.hist[((size_t)r * P.C + c) * P.H + idx];
}

// grid: one workgroup (LIN_LW waves) per cluster c0 + blockIdx.x.  stage:
// [grid][N*H] ops, the cluster's history grouped by key (its own region of
// the launch's workspace).  Dynamic LDS: LIN_LW sort buffers (LIN_SORT_BYTES);
// partitions of at most LIN_SMAX ops are checked in registers (LinReg).
__global__ void __launch_bounds__(LIN_LW * 64, PXS_LIN_MINW) lin_cluster_kernel(Params P, uint64_t c0, uint4* stage_all,
                                                                   unsigned long long* out, uint2* big) {
  extern __shared__ uint4 lds_lin[];
  __shared__ uint32_t len[PAXISIM_MAX_N];
  __shared__ uint32_t cnt[LIN_LW][PAXISIM_MAX_KEYS];   // per wave slice, per key
  __shared__ uint32_t koff[PAXISIM_MAX_KEYS + 1];
  const uint64_t c = c0 + blockIdx.x;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t K = P.keys;
  const uint32_t cap = P.N * P.H;
  uint4* stage = stage_all + (size_t)blockIdx.x * cap;
  uint8_t* wsp = reinterpret_cast<uint8_t*>(lds_lin) + wave * LIN_SORT_BYTES;
#ifdef PXS_LIN_STAMPS
  uint32_t lst[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
  LIN_T0(tp1)
  if (threadIdx.x < P.N) len[threadIdx.x] = P.execute[rc(P, threadIdx.x, c)];
  for (uint32_t k = threadIdx.x; k < LIN_LW * PAXISIM_MAX_KEYS; k += blockDim.x) (&cnt[0][0])[k] = 0;
  __syncthreads();
  uint32_t tot = 0;
  for (uint32_t r = 0; r < P.N; r++) tot += len[r];
  // pass 1: per-key counts of each wave's slice of the canonical sequence (key words only)
  const uint32_t per = (tot + LIN_LW - 1u) / LIN_LW;
  const uint32_t lo = wave * per < tot ? wave * per : tot, hi = lo + per < tot ? lo + per : tot;
  for (uint32_t i = lo + lane_id(); i < hi; i += 64u) {
    const uint32_t key = *reinterpret_cast<const uint32_t*>(hist_at(P, c, len, i)) & 0x7FFFFFFFu;
    if (key < K) atomicAdd(&cnt[wave][key], 1u);       // (paxisim_history_load admits keys < K only)
  }
  __syncthreads();
  if (threadIdx.x == 0) {                              // key-major, wave-minor exclusive scan
    uint32_t acc = 0;
    for (uint32_t k = 0; k < K; k++) {
      koff[k] = acc;
      for (uint32_t w = 0; w < LIN_LW; w++) {
        const uint32_t v = cnt[w][k];
        cnt[w][k] = acc;
        acc += v;
      }
    }
    koff[K] = acc;
  }
  __syncthreads();
  LIN_T1(tp1, LS_P1)
  LIN_T0(tp2)
  // pass 2: stable placement by key.  Each wave walks its slice in 64-op
  // chunks; an op goes to its key's running offset for this wave plus its
  // rank among the chunk's ops of that key (a ballot per distinct key).
  for (uint32_t i0 = lo; i0 < hi; i0 += 64u) {
    const uint32_t i = i0 + lane_id();
    const uint4 o = i < hi ? *hist_at(P, c, len, i) : make_uint4(0u, 0u, 0u, 0u);
    const bool act = i < hi && (o.x & 0x7FFFFFFFu) < K;
    const uint32_t key = act ? (o.x & 0x7FFFFFFFu) : 0xFFFFFFFFu;
    uint64_t todo = __ballot(act);
    while (todo) {
      const uint32_t kk = (uint32_t)__builtin_amdgcn_readlane((int)key, (int)first_lane(todo));
      const uint64_t m = __ballot(key == kk);
      const uint32_t base = cnt[wave][kk];
      if (key == kk) stage[base + (uint32_t)__popcll(m & ((1ull << lane_id()) - 1ull))] = o;
      __builtin_amdgcn_wave_barrier();
      if (lane_id() == 0) cnt[wave][kk] = base + (uint32_t)__popcll(m);
      todo &= ~m;
    }
  }
  __threadfence_block();
  __syncthreads();
  LIN_T1(tp2, LS_P2)
  // pass 3: the keys in turn, one wave each
  unsigned long long anomalies = 0, ops = 0;
  for (uint32_t k = wave; k < K; k += LIN_LW) {
    const uint32_t n = koff[k + 1] - koff[k];
    if (!n) continue;
    if (n > LIN_VMAX) {                                // beyond the bit sets: reported, not checked
      if (lane_id() == 0) atomicAdd(&out[LIN_SKIP], 1ull);
      continue;
    }
    ops += n;
    if (n > LIN_SMAX) {                                // the big path
      if (lane_id() == 0) {
        const uint32_t slot = (uint32_t)atomicAdd(&out[LIN_BIG], 1ull);
        big[slot] = make_uint2(blockIdx.x * cap + koff[k], n);
        atomicMax(&out[LIN_NMAX], (unsigned long long)n);
      }
      continue;
    }
    LinScratch srt;                                      // the sort's LDS buffers: ops and start copies
    srt.ops = reinterpret_cast<uint4*>(wsp);
    srt.stk = reinterpret_cast<uint32_t*>(wsp + LIN_SMAX * 16u);
    LIN_T0(tso)
    lin_sort<false>(stage + koff[k], n, srt);
    __builtin_amdgcn_wave_barrier();
    LinReg g;
    g.load(srt.ops, n);
    LIN_T1(tso, LS_SORT)
    LIN_T0(tru)
#ifdef PXS_LIN_STAMPS
    for (int q = 0; q < 8; q++) g.lst[q] = 0;
#endif
    anomalies += g.run();
    LIN_T1(tru, LS_RUN)
#ifdef PXS_LIN_STAMPS
    for (int q = LS_ADD; q < 8; q++) lst[q] += g.lst[q];
#endif
    __builtin_amdgcn_wave_barrier();                     // the next key's sort reuses the buffer
  }
  if (lane_id() == 0) {
    if (anomalies) atomicAdd(&out[LIN_ANOM], anomalies);
    if (ops) atomicAdd(&out[LIN_OPS], ops);
#ifdef PXS_LIN_STAMPS
    for (int q = 0; q < 8; q++) atomicAdd(&out[LIN_NOUT + q], (unsigned long long)lst[q]);
#endif
  }
}

// grid-stride over the big partitions {stage offset, ops}: one wave each,
// scratch in HBM (slot = blockIdx.x), capacity 64 * nw ops; WPL bit-set words
// per lane (nw <= 64 * WPL).
template <int WPL>
__global__ void __launch_bounds__(64) lin_big_kernel(const uint4* stage_all, const uint2* big, uint32_t nbig,
                                                     uint8_t* ws, uint32_t nw, unsigned long long* out) {
  const LinScratch s = lin_scratch(ws + (size_t)blockIdx.x * lin_scratch_bytes(nw, false), nw, false);
  unsigned long long anomalies = 0;
  for (uint32_t b = blockIdx.x; b < nbig; b += gridDim.x) {
    LinCheck<true, WPL> g;
    g.s = s;
    g.n = big[b].y;
    lin_sort<true>(stage_all + big[b].x, g.n, g.s);
    anomalies += g.run();
  }
  if (lane_id() == 0 && anomalies) atomicAdd(&out[LIN_ANOM], anomalies);
}

}  // namespace pxs
