// lin_kernel.h — History.Linearizable on gfx950 (history.go:55-71).
//
// One thread checks one (cluster, key) partition of the completed-operation
// history with the reference's graph algorithm, checker.go:69-104:
//   ops sorted by start (stable); add() draws happens-before edges into each
//   new vertex; a read looks ahead for concurrent writes, is merged into the
//   write whose value it returned, and a cycle in the graph is an anomaly,
//   after which the cycle's edges u->v with u.start > v.end are removed.
// Vertex iteration is in insertion order (Go's map order is random; the
// oracle uses the same insertion order).  The graph is a
// 128x128 bit matrix; partitions with more than LIN_MAXV operations are
// skipped and counted.  The recursive DFS of lib/graph.go:180-193 becomes an
// explicit stack.  Workspace is per thread in HBM, field-major so that the
// threads of a wave touch consecutive words.
#pragma once
#include "paxisim_dev.h"

namespace pxs {

constexpr uint32_t LIN_MAXV = 128;
constexpr uint32_t LIN_WORDS = LIN_MAXV / 64;   // u64 words per bit row

struct LinWs {
  uint64_t* adj;     // [LIN_MAXV][LIN_WORDS][T]
  uint32_t* vin;     // [LIN_MAXV][T] write value (input)
  uint32_t* vout;    // [LIN_MAXV][T] read value (output)
  uint32_t* vstart;  // [LIN_MAXV][T]
  uint32_t* vend;    // [LIN_MAXV][T]
  uint32_t* vw;      // [LIN_MAXV][T] 1 = write (has input), 0 = read (has output)
  uint32_t* order;   // [LIN_MAXV][T] insertion order
  uint32_t* stk;     // [LIN_MAXV][T] DFS stack: vertex | next order index << 16
  uint64_t T;
};

struct Bits {
  uint64_t w[LIN_WORDS];
  __device__ __forceinline__ bool get(uint32_t i) const {
    bool b = false;
#pragma unroll
    for (uint32_t k = 0; k < LIN_WORDS; k++) b |= (k == (i >> 6)) && ((w[k] >> (i & 63u)) & 1u);
    return b;
  }
  __device__ __forceinline__ void set(uint32_t i) {
#pragma unroll
    for (uint32_t k = 0; k < LIN_WORDS; k++)
      if (k == (i >> 6)) w[k] |= 1ull << (i & 63u);
  }
  __device__ __forceinline__ void clr(uint32_t i) {
#pragma unroll
    for (uint32_t k = 0; k < LIN_WORDS; k++)
      if (k == (i >> 6)) w[k] &= ~(1ull << (i & 63u));
  }
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (uint32_t k = 0; k < LIN_WORDS; k++) w[k] = 0;
  }
};

struct Lin {
  const LinWs& ws;
  uint64_t tid;
  uint32_t n, norder;
  Bits present;
  __device__ Lin(const LinWs& w, uint64_t t) : ws(w), tid(t), n(0), norder(0) { present.zero(); }
  __device__ __forceinline__ size_t at(uint32_t v) const { return (size_t)v * ws.T + tid; }
  __device__ __forceinline__ size_t adj_at(uint32_t v, uint32_t k) const {
    return ((size_t)v * LIN_WORDS + k) * ws.T + tid;
  }
  __device__ __forceinline__ bool edge(uint32_t u, uint32_t v) const {
    return (ws.adj[adj_at(u, v >> 6)] >> (v & 63u)) & 1u;
  }
  __device__ __forceinline__ void set_edge(uint32_t u, uint32_t v) { ws.adj[adj_at(u, v >> 6)] |= 1ull << (v & 63u); }
  __device__ __forceinline__ void clr_edge(uint32_t u, uint32_t v) { ws.adj[adj_at(u, v >> 6)] &= ~(1ull << (v & 63u)); }
  __device__ __forceinline__ bool happen_before(uint32_t a, uint32_t b) const {   // operation.go:12-14
    return ws.vend[at(a)] < ws.vstart[at(b)];
  }
  __device__ __forceinline__ void add_vertex(uint32_t v) {
    if (present.get(v)) return;
    present.set(v);
    ws.order[at(norder++)] = v;
  }
  __device__ __forceinline__ void chk_add(uint32_t o) {                            // checker.go:21-33
    if (present.get(o)) return;
    add_vertex(o);
    for (uint32_t k = 0; k < norder; k++) {
      const uint32_t v = ws.order[at(k)];
      if (happen_before(v, o)) set_edge(v, o);
    }
  }
  __device__ __forceinline__ void remove(uint32_t v) {                             // graph.go:36-48
    if (!present.get(v)) return;
    present.clr(v);
    for (uint32_t k = 0; k < LIN_WORDS; k++) ws.adj[adj_at(v, k)] = 0;
    uint32_t j = 0;
    for (uint32_t k = 0; k < norder; k++) {
      const uint32_t u = ws.order[at(k)];
      clr_edge(u, v);
      if (u != v) ws.order[at(j++)] = u;
    }
    norder = j;
  }
  // Cycle() (graph.go:212-232): returns true and leaves `gray` = the DFS stack
  __device__ bool cycle(Bits& gray) {
    Bits black;
    black.zero();
    gray.zero();
    for (uint32_t s = 0; s < norder; s++) {
      const uint32_t root = ws.order[at(s)];
      if (gray.get(root) || black.get(root)) continue;
      uint32_t sp = 0;
      gray.set(root);
      ws.stk[at(sp++)] = root;
      while (sp) {                                                                  // visit(): graph.go:180-193
        const uint32_t top = ws.stk[at(sp - 1)];
        const uint32_t v = top & 0xFFFFu;
        uint32_t k = top >> 16;
        uint32_t u = 0;
        bool next = false;
        for (; k < norder; k++) {
          u = ws.order[at(k)];
          if (edge(v, u) && !black.get(u)) { next = true; break; }
        }
        if (!next) {
          gray.clr(v);
          black.set(v);
          sp--;
          continue;
        }
        ws.stk[at(sp - 1)] = v | ((k + 1u) << 16);
        if (gray.get(u)) return true;
        gray.set(u);
        ws.stk[at(sp++)] = u;
      }
    }
    return false;
  }
};

// grid: one thread per (cluster, key) of clusters [c0, c0+nc)
__global__ void lin_kernel(Params P, LinWs ws, uint64_t c0, uint64_t nc, uint64_t* out) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t anomalies = 0, checked = 0, skipped = 0;
  if (tid < nc * P.keys) {
    const uint64_t c = c0 + tid / P.keys;
    const uint32_t key = (uint32_t)(tid % P.keys);
    Lin g(ws, tid);
    // gather the partition in canonical order, then stable-sort by start (sort.Sort(byTime))
    uint32_t n = 0;
    bool over = false;
    for (uint32_t r = 0; r < P.N; r++) {
      const uint32_t len = P.execute[rc(P, r, c)];
      const uint4* h = &P.hist[((size_t)r * P.C + c) * P.H];
      for (uint32_t j = 0; j < len; j++) {
        const uint4 o = h[j];
        if ((o.x & 0x7FFFFFFFu) != key) continue;
        if (n == LIN_MAXV) { over = true; break; }
        const uint32_t w = o.x >> 31;
        uint32_t p = n++;
        while (p > 0 && ws.vstart[g.at(p - 1)] > o.z) {          // insertion sort: stable
          ws.vin[g.at(p)] = ws.vin[g.at(p - 1)];
          ws.vout[g.at(p)] = ws.vout[g.at(p - 1)];
          ws.vstart[g.at(p)] = ws.vstart[g.at(p - 1)];
          ws.vend[g.at(p)] = ws.vend[g.at(p - 1)];
          ws.vw[g.at(p)] = ws.vw[g.at(p - 1)];
          p--;
        }
        ws.vin[g.at(p)] = w ? o.y : 0u;
        ws.vout[g.at(p)] = w ? 0u : o.y;
        ws.vstart[g.at(p)] = o.z;
        ws.vend[g.at(p)] = o.w;
        ws.vw[g.at(p)] = w;
      }
      if (over) break;
    }
    if (over) {
      skipped = 1;
    } else if (n) {
      checked = n;
      for (uint32_t v = 0; v < n; v++)
        for (uint32_t k = 0; k < LIN_WORDS; k++) ws.adj[g.adj_at(v, k)] = 0;
      for (uint32_t i = 0; i < n; i++) {                          // checker.go:73-102
        g.chk_add(i);
        if (ws.vw[g.at(i)]) continue;                              // writes: nothing more
        for (uint32_t j = i + 1; j < n && !g.happen_before(i, j) && !g.happen_before(j, i); j++)
          if (ws.vw[g.at(j)]) g.chk_add(j);                        // look-ahead concurrent writes
        int match = -1;                                            // match: checker.go:44-52
        for (uint32_t k = 0; k < g.norder; k++) {
          const uint32_t v = ws.order[g.at(k)];
          if (ws.vw[g.at(v)] && ws.vin[g.at(v)] == ws.vout[g.at(i)]) { match = (int)v; break; }
        }
        if (match >= 0) {                                          // merge: checker.go:55-67
          const uint32_t mw = (uint32_t)match;
          for (uint32_t k = 0; k < g.norder; k++) {
            const uint32_t s2 = ws.order[g.at(k)];
            if (g.edge(s2, i) && s2 != mw) g.set_edge(s2, mw);
          }
          if (ws.vend[g.at(i)] < ws.vend[g.at(mw)]) ws.vend[g.at(mw)] = ws.vend[g.at(i)];
          g.remove(i);
        }
        Bits gray;
        if (g.cycle(gray)) {
          anomalies++;
          for (uint32_t a = 0; a < g.norder; a++) {
            const uint32_t u = ws.order[g.at(a)];
            if (!gray.get(u)) continue;
            for (uint32_t b = 0; b < g.norder; b++) {
              const uint32_t v = ws.order[g.at(b)];
              if (gray.get(v) && g.edge(u, v) && ws.vstart[g.at(u)] > ws.vend[g.at(v)]) g.clr_edge(u, v);
            }
          }
        }
      }
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    anomalies += __shfl_down(anomalies, o, 64);
    checked += __shfl_down(checked, o, 64);
    skipped += __shfl_down(skipped, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    if (anomalies) atomicAdd((unsigned long long*)&out[0], (unsigned long long)anomalies);
    if (checked) atomicAdd((unsigned long long*)&out[1], (unsigned long long)checked);
    if (skipped) atomicAdd((unsigned long long*)&out[2], (unsigned long long)skipped);
  }
}

}  // namespace pxs
