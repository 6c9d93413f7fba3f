// Residency probe: how many workgroups of a given shape share a CU at once.
// Each workgroup records {start, end (100 MHz clock), HW_ID, XCC_ID} and spins ~1 ms.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <vector>
#include <algorithm>

__global__ void probe(unsigned long long* out, int spin, int scratch_idx) {
  extern __shared__ unsigned int lds[];
  volatile unsigned int priv[64];   // forces a private (scratch) segment when indexed at run time
  for (int i = 0; i < 64; i++) priv[i] = i * threadIdx.x;
  unsigned long long t0, t1;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  lds[threadIdx.x] = threadIdx.x;
  __syncthreads();
  for (int i = 0; i < spin; i++) __builtin_amdgcn_s_sleep(100);
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  if (threadIdx.x == 0) {
    out[blockIdx.x * 4 + 0] = t0;
    out[blockIdx.x * 4 + 1] = t1;
    out[blockIdx.x * 4 + 2] = __builtin_amdgcn_s_getreg((4) | (0 << 6) | ((32 - 1) << 11));
    out[blockIdx.x * 4 + 3] = __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((32 - 1) << 11)) + lds[5] +
                              (scratch_idx >= 0 ? ((unsigned long long)priv[scratch_idx & 63] << 40) : 0ull);
  }
}

int main(int argc, char** argv) {
  const int threads = atoi(argv[1]), lds = atoi(argv[2]), attr = atoi(argv[3]);
  const int blocks = 512;
  unsigned long long* d;
  hipMalloc(&d, blocks * 4 * 8);
  hipFuncSetAttribute((const void*)probe, hipFuncAttributeMaxDynamicSharedMemorySize, attr);
  int occ = 0;
  hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)probe, threads, lds);
  const int use_scratch = argc > 4 ? atoi(argv[4]) : 0;
  probe<<<blocks, threads, lds>>>(d, 2000, use_scratch ? 7 : -1);
  hipError_t e = hipDeviceSynchronize();
  std::vector<unsigned long long> h(blocks * 4);
  hipMemcpy(h.data(), d, blocks * 32, hipMemcpyDeviceToHost);
  std::map<unsigned long long, std::vector<std::pair<unsigned long long, unsigned long long>>> cu;
  for (int b = 0; b < blocks; b++) {
    unsigned long long hw = h[b * 4 + 2], key = ((h[b * 4 + 3] & 0xFull) << 16) | ((hw >> 8) & 0xFF);
    cu[key].push_back({h[b * 4], h[b * 4 + 1]});
  }
  int maxconc = 0;
  for (auto& kv : cu) {
    auto v = kv.second;
    for (auto& a : v) {
      int c = 0;
      for (auto& b : v) c += (b.first <= a.first && a.first < b.second);
      maxconc = std::max(maxconc, c);
    }
  }
  printf("scratch=%d threads=%d lds=%d attr=%d: err=%s occupancy_api=%d distinct_cus=%zu max_concurrent_per_cu=%d\n", use_scratch, threads, lds,
         attr, hipGetErrorString(e), occ, cu.size(), maxconc);
  return 0;
}
