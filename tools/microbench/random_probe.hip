// random_probe.hip — microbenchmark: random 64-B bucket reads / atomics over
// tables of growing size on one MI355X (what the ClaimSet / FPSet probes cost
// as a function of footprint).  Diagnostic only; not part of the product.
//
//   hipcc -O3 --offload-arch=gfx950 random_probe.hip -o random_probe && ./random_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));   \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

// one lane reads a whole 64-B bucket (4 x 16-B loads)
__global__ void k_lane_bucket(const ulonglong2* __restrict__ t, uint64_t nb, uint64_t n, uint64_t seed,
                              unsigned long long* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t b = __umul64hi(mix(seed + i), nb);
  const ulonglong2* p = t + b * 4;
  const ulonglong2 a = p[0], c = p[1], d = p[2], e = p[3];
  const unsigned long long x = a.x ^ a.y ^ c.x ^ c.y ^ d.x ^ d.y ^ e.x ^ e.y;
  if (x == 0x1234567ull) out[0] = x;
}
// 4 lanes cooperate: each reads 16 B of the same bucket
__global__ void k_quad_bucket(const ulonglong2* __restrict__ t, uint64_t nb, uint64_t n, uint64_t seed,
                              unsigned long long* __restrict__ out) {
  const uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x);
  const uint64_t q = i >> 2;
  if (q >= n) return;
  const uint64_t b = __umul64hi(mix(seed + q), nb);
  const ulonglong2 a = t[b * 4 + (i & 3)];
  const unsigned long long x = a.x ^ a.y;
  if (x == 0x1234567ull) out[0] = x;
}
// one 8-B load per lane (random)
__global__ void k_lane_8b(const unsigned long long* __restrict__ t, uint64_t nb, uint64_t n, uint64_t seed,
                          unsigned long long* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t b = __umul64hi(mix(seed + i), nb);
  const unsigned long long x = t[b * 8];
  if (x == 0x1234567ull) out[0] = x;
}
// random 64-bit atomicMax (with return)
__global__ void k_atomic(unsigned long long* __restrict__ t, uint64_t nb, uint64_t n, uint64_t seed,
                         unsigned long long* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t b = __umul64hi(mix(seed + i), nb);
  const unsigned long long x = atomicMax(t + b * 8 + 1, (unsigned long long)i);
  if (x == 0x1234567ull) out[0] = x;
}
// random 64-bit atomicCAS (with return), mostly failing
__global__ void k_cas(unsigned long long* __restrict__ t, uint64_t nb, uint64_t n, uint64_t seed,
                      unsigned long long* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t b = __umul64hi(mix(seed + i), nb);
  const unsigned long long x = atomicCAS(t + b * 8, 1ull, (unsigned long long)i);
  if (x == 0x1234567ull) out[0] = x;
}

template <class K, class T>
static int timeit(const char* name, K kern, T* tab, uint64_t nb, uint64_t n, int lanes_per_op,
                  unsigned long long* out, uint64_t table_bytes) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const uint64_t threads = n * lanes_per_op;
  const unsigned grid = (unsigned)((threads + 255) / 256);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, tab, nb, n, 1ull, out);  // warm
  CK(hipEventRecord(a));
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, tab, nb, n, 7ull + r, out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  const double ops = 3.0 * n / (ms * 1e-3);
  printf("%-12s table %8.2f GB  %7.2f G ops/s  (%6.1f GB/s of 64-B lines)\n", name, table_bytes / 1e9,
         ops / 1e9, ops * 64 / 1e9);
  fflush(stdout);
  return 0;
}

int main() {
  const uint64_t n = 1ull << 28;   // ops per launch
  unsigned long long* out;
  CK(hipMalloc(&out, 64));
  const double gbs[] = {0.25, 1, 4, 16, 32, 64};
  for (double gb : gbs) {
    const uint64_t bytes = (uint64_t)(gb * 1e9) / 64 * 64;
    const uint64_t nb = bytes / 64;
    void* tab;
    CK(hipMalloc(&tab, bytes));
    CK(hipMemset(tab, 0, bytes));
    timeit("lane-64B", k_lane_bucket, (const ulonglong2*)tab, nb, n, 1, out, bytes);
    timeit("quad-16B", k_quad_bucket, (const ulonglong2*)tab, nb, n, 4, out, bytes);
    timeit("lane-8B", k_lane_8b, (const unsigned long long*)tab, nb, n, 1, out, bytes);
    timeit("atomicMax", k_atomic, (unsigned long long*)tab, nb, n, 1, out, bytes);
    timeit("atomicCAS", k_cas, (unsigned long long*)tab, nb, n, 1, out, bytes);
    CK(hipFree(tab));
  }
  return 0;
}
