// scatter_probe: calibrates rocprofv3's FETCH_SIZE / WRITE_SIZE for the access
// pattern of the step kernels - each lane touching 16 to 64 bytes of its own
// cache line, lines far apart (MI355X_MICROARCH.md: "other access widths are
// uncalibrated: calibrate on a known byte count in your own access pattern").
// Every kernel touches N lanes x one line each, chosen by a hash over a 16 GiB
// buffer (far beyond the L2 and the 256 MiB MALL), one launch per pattern:
//   rd16 / rd32 / rd64 / rd128: each lane reads 16 / 32 / 64 / 128 B of its line
//   wr16 / wr32 / wr64: each lane writes 16 / 32 / 64 B of its line
//   rmw16: each lane reads then writes the same 16 B
// Launch k (in that order) is dispatch k of the trace; bytes "touched" per lane
// are printed so FETCH_SIZE / WRITE_SIZE per dispatch can be divided by them.
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe/scatter_probe tools/probe/scatter_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

__device__ __forceinline__ uint32_t fmix(uint32_t h) {
  h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
  return h;
}
__device__ __forceinline__ size_t line_of(uint32_t i, uint32_t salt, size_t nlines) {
  return (((size_t)fmix(i ^ salt) << 20) ^ fmix(i * 0x9E3779B1u + salt)) % nlines;
}

template <int NV>
__global__ void rd(const uint4* __restrict__ a, size_t nlines, uint32_t n, uint32_t salt, unsigned* out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint4* p = a + line_of(i, salt, nlines) * 8;
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < NV; k++) { const uint4 v = p[k]; acc ^= v.x ^ v.y ^ v.z ^ v.w; }
  if (acc == 0x12345678u) out[0] = acc;
}
template <int NV>
__global__ void wr(uint4* __restrict__ a, size_t nlines, uint32_t n, uint32_t salt) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint4* p = a + line_of(i, salt, nlines) * 8;
#pragma unroll
  for (int k = 0; k < NV; k++) p[k] = make_uint4(i, k, salt, 1u);
}
__global__ void rmw(uint4* __restrict__ a, size_t nlines, uint32_t n, uint32_t salt) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint4* p = a + line_of(i, salt, nlines) * 8;
  uint4 v = *p;
  v.x += 1u;
  *p = v;
}

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
  const size_t bytes = 16ull << 30, nlines = bytes / 128;
  const uint32_t n = 1u << 24;   // lanes per launch (16 M lines touched)
  uint4* a = nullptr;
  unsigned* o = nullptr;
  CHK(hipMalloc(&a, bytes));
  CHK(hipMalloc(&o, 4));
  CHK(hipMemset(a, 1, bytes));
  CHK(hipDeviceSynchronize());
  const unsigned block = 256, grid = (n + block - 1) / block;
  const char* names[] = {"rd16", "rd32", "rd64", "rd128", "wr16", "wr32", "wr64", "rmw16"};
  const int touched[] = {16, 32, 64, 128, 16, 32, 64, 16};
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  printf("{\"probe\": \"scatter\", \"lanes_per_launch\": %u, \"buffer_bytes\": %zu, \"launches\": [", n, bytes);
  for (int k = 0; k < 8; k++) {
    const uint32_t salt = 0x1000u * (k + 1);
    float ms = 0;
    CHK(hipEventRecord(e0));
    switch (k) {
      case 0: rd<1><<<grid, block>>>(a, nlines, n, salt, o); break;
      case 1: rd<2><<<grid, block>>>(a, nlines, n, salt, o); break;
      case 2: rd<4><<<grid, block>>>(a, nlines, n, salt, o); break;
      case 3: rd<8><<<grid, block>>>(a, nlines, n, salt, o); break;
      case 4: wr<1><<<grid, block>>>(a, nlines, n, salt); break;
      case 5: wr<2><<<grid, block>>>(a, nlines, n, salt); break;
      case 6: wr<4><<<grid, block>>>(a, nlines, n, salt); break;
      default: rmw<<<grid, block>>>(a, nlines, n, salt); break;
    }
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    CHK(hipEventElapsedTime(&ms, e0, e1));
    printf("%s{\"dispatch\": %d, \"name\": \"%s\", \"bytes_touched_per_lane\": %d, \"ms\": %.3f}", k ? ", " : "",
           k, names[k], touched[k], ms);
  }
  printf("]}\n");
  return 0;
}
