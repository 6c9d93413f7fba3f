// Residency probe 2: does a workgroup of 5 waves that needs ~V VGPRs share a CU with another?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <vector>
#include <algorithm>

template <int V, int MINW>
__global__ void __launch_bounds__(320, MINW) probe(unsigned long long* out, int spin, const unsigned* in) {
  extern __shared__ unsigned int lds[];
  unsigned long long t0, t1;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  unsigned r[V];
#pragma unroll
  for (int k = 0; k < V; k++) r[k] = in[k * 320 + threadIdx.x];
  lds[threadIdx.x] = threadIdx.x;
  __syncthreads();
  for (int i = 0; i < spin; i++) {
    __builtin_amdgcn_s_sleep(100);
#pragma unroll
    for (int k = 0; k < V; k++) r[k] = r[k] * 3u + r[(k + 1) % V];
  }
  unsigned acc = 0;
#pragma unroll
  for (int k = 0; k < V; k++) acc ^= r[k];
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  if (threadIdx.x == 0) {
    out[blockIdx.x * 4 + 0] = t0;
    out[blockIdx.x * 4 + 1] = t1;
    out[blockIdx.x * 4 + 2] = __builtin_amdgcn_s_getreg((4) | (0 << 6) | ((32 - 1) << 11));
    out[blockIdx.x * 4 + 3] = __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((32 - 1) << 11)) + ((unsigned long long)acc << 32);
  }
}

template <int V, int MINW>
void run(int lds) {
  const int blocks = 512;
  unsigned long long* d;
  unsigned* in;
  (void)hipMalloc(&d, blocks * 4 * 8);
  (void)hipMalloc(&in, 320 * 256 * 4);
  (void)hipMemset(in, 1, 320 * 256 * 4);
  (void)hipFuncSetAttribute((const void*)probe<V, MINW>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  int occ = 0;
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)probe<V, MINW>, 320, lds);
  probe<V, MINW><<<blocks, 320, lds>>>(d, 200, in);
  hipError_t e = hipDeviceSynchronize();
  std::vector<unsigned long long> h(blocks * 4);
  (void)hipMemcpy(h.data(), d, blocks * 32, hipMemcpyDeviceToHost);
  std::map<unsigned long long, std::vector<std::pair<unsigned long long, unsigned long long>>> cu;
  for (int b = 0; b < blocks; b++) {
    unsigned long long hw = h[b * 4 + 2], key = ((h[b * 4 + 3] & 0xFull) << 16) | ((hw >> 8) & 0xFF);
    cu[key].push_back({h[b * 4], h[b * 4 + 1]});
  }
  int maxconc = 0;
  for (auto& kv : cu)
    for (auto& a : kv.second) {
      int c = 0;
      for (auto& b : kv.second) c += (b.first <= a.first && a.first < b.second);
      maxconc = std::max(maxconc, c);
    }
  printf("V=%d minwaves=%d lds=%d: err=%s occupancy_api=%d max_concurrent_per_cu=%d\n", V, MINW, lds, hipGetErrorString(e),
         occ, maxconc);
  (void)hipFree(d);
  (void)hipFree(in);
}

int main() {
  run<100, 3>(77312);
  run<100, 4>(0);
  run<100, 4>(46592);
  run<100, 5>(0);
  run<100, 6>(0);
  run<20, 8>(0);
  return 0;
}
