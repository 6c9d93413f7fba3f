// copy_bw: the achievable HBM bandwidth of this MI355X (SURVEY.md §8d asks
// for it beside the 8 TB/s spec peak the roofline fraction is priced on).
// A grid-stride uint4 copy between two 4 GiB buffers, 256 threads a block,
// 8 x 256 CUs of blocks; bytes = read + write.  Prints one JSON line.
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe/copy_bw tools/probe/copy_bw.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void copy_kernel(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) b[i] = a[i];
}

__global__ void read_kernel(const uint4* __restrict__ a, size_t n, unsigned* out) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  unsigned acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint4 v = a[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;   // keeps the loads
}

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
  const size_t bytes = 4ull << 30, n = bytes / sizeof(uint4);
  uint4 *a = nullptr, *b = nullptr;
  unsigned* o = nullptr;
  CHK(hipMalloc(&a, bytes));
  CHK(hipMalloc(&b, bytes));
  CHK(hipMalloc(&o, 4));
  CHK(hipMemset(a, 1, bytes));
  CHK(hipMemset(b, 0, bytes));
  int cus = 0;
  CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const unsigned grid = (unsigned)cus * 8u, block = 256;
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  float best_copy = 1e30f, best_read = 1e30f;
  for (int rep = 0; rep < 12; rep++) {
    float ms = 0;
    CHK(hipEventRecord(e0));
    copy_kernel<<<grid, block>>>(a, b, n);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    CHK(hipEventElapsedTime(&ms, e0, e1));
    if (rep >= 2 && ms < best_copy) best_copy = ms;
    CHK(hipEventRecord(e0));
    read_kernel<<<grid, block>>>(a, n, o);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    CHK(hipEventElapsedTime(&ms, e0, e1));
    if (rep >= 2 && ms < best_read) best_read = ms;
  }
  printf("{\"probe\": \"copy_bw\", \"cus\": %d, \"buffer_bytes\": %zu, \"copy_GBps\": %.1f, \"read_GBps\": %.1f, "
         "\"copy_ms\": %.3f, \"read_ms\": %.3f, \"method\": \"best of 10 timed launches (2 warm-up), uint4 grid-stride, "
         "bytes = read + write for copy\"}\n",
         cus, bytes, 2.0 * bytes / (best_copy * 1e6), (double)bytes / (best_read * 1e6), best_copy, best_read);
  return 0;
}
