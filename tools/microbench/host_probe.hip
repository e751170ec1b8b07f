// host_probe.hip — microbenchmark: what a kernel pays to read pinned HOST
// memory directly (random 8-B / 64-B lookups, sequential streaming) against a
// hipMemcpyAsync stream of the same buffer.  Sizes the seen-set spill tier
// (DESIGN.md §4.5): cold fingerprint runs in pinned host RAM, probed by the
// GPU.  Diagnostic only; not part of the product.
//
//   hipcc -O3 --offload-arch=gfx950 host_probe.hip -o host_probe && ./host_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

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

// one 8-B load per lane at a random line
__global__ void k_rand8(const unsigned long long* __restrict__ t, uint64_t nlines, uint64_t n, uint64_t seed,
                        unsigned long long* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t b = __umul64hi(mix(seed + i), nlines);
  const unsigned long long x = t[b * 8];
  if (x == 0x1234567ull) out[0] = x;
}
// one lane reads a whole random 64-B line (4 x 16 B)
__global__ void k_rand64(const ulonglong2* __restrict__ t, uint64_t nlines, uint64_t n, uint64_t seed,
                         unsigned long long* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t b = __umul64hi(mix(seed + i), nlines);
  const ulonglong2* p = t + b * 4;
  const ulonglong2 a = p[0], c = p[1], d = p[2], e = p[3];
  const unsigned long long x = a.x ^ a.y ^ c.x ^ c.y ^ d.x ^ d.y ^ e.x ^ e.y;
  if (x == 0x1234567ull) out[0] = x;
}
// sorted random: lane i reads line floor(i * nlines / n) + small jitter
// (the shape of a sorted query batch probing a sorted run)
__global__ void k_sorted64(const ulonglong2* __restrict__ t, uint64_t nlines, uint64_t n, uint64_t seed,
                           unsigned long long* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t b = (uint64_t)((double)i / (double)n * (double)nlines) + (mix(seed + i) & 3);
  if (b >= nlines) b = nlines - 1;
  const ulonglong2* p = t + b * 4;
  const ulonglong2 a = p[0], c = p[1], d = p[2], e = p[3];
  const unsigned long long x = a.x ^ a.y ^ c.x ^ c.y ^ d.x ^ d.y ^ e.x ^ e.y;
  if (x == 0x1234567ull) out[0] = x;
}
// streaming read: grid-stride 16-B loads
__global__ void k_stream(const ulonglong2* __restrict__ t, uint64_t n16, unsigned long long* __restrict__ out) {
  unsigned long long x = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
    const ulonglong2 a = t[i];
    x ^= a.x ^ a.y;
  }
  if (x == 0x1234567ull) out[0] = x;
}

template <class K, class T>
static int timeit(const char* name, K kern, T* tab, uint64_t nlines, uint64_t n, unsigned long long* out) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const unsigned grid = (unsigned)((n + 255) / 256);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, tab, nlines, n, 1ull, out);  // warm
  CK(hipEventRecord(a));
  for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, tab, nlines, n, 7ull + r, out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  const double ops = 2.0 * n / (ms * 1e-3);
  printf("%-10s %7.1f M ops/s  (%6.2f GB/s of 64-B lines)\n", name, ops / 1e6, ops * 64 / 1e9);
  fflush(stdout);
  return 0;
}

int main() {
  const uint64_t bytes = 4ull << 30;
  const uint64_t nlines = bytes / 64;
  unsigned long long* out;
  CK(hipMalloc(&out, 64));
  void* dev;
  CK(hipMalloc(&dev, bytes));
  const unsigned flags[] = {hipHostMallocDefault, hipHostMallocNonCoherent, hipHostMallocCoherent};
  const char* fname[] = {"default", "noncoherent", "coherent"};
  for (int f = 0; f < 3; ++f) {
    void* host;
    CK(hipHostMalloc(&host, bytes, flags[f]));
    memset(host, 0, bytes);
    printf("== pinned host %.1f GB, %s\n", bytes / 1e9, fname[f]);
    for (uint64_t n : {1ull << 20, 1ull << 24}) {
      printf("-- %llu ops per launch\n", (unsigned long long)n);
      timeit("rand-8B", k_rand8, (const unsigned long long*)host, nlines, n, out);
      timeit("rand-64B", k_rand64, (const ulonglong2*)host, nlines, n, out);
      timeit("sorted-64B", k_sorted64, (const ulonglong2*)host, nlines, n, out);
    }
    {
      hipEvent_t a, b;
      CK(hipEventCreate(&a));
      CK(hipEventCreate(&b));
      CK(hipEventRecord(a));
      hipLaunchKernelGGL(k_stream, dim3(4096), dim3(256), 0, 0, (const ulonglong2*)host, bytes / 16, out);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      printf("kernel stream read   %6.2f GB/s\n", bytes / (ms * 1e-3) / 1e9);
      CK(hipEventRecord(a));
      CK(hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, 0));
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms, a, b));
      printf("memcpy H2D           %6.2f GB/s\n", bytes / (ms * 1e-3) / 1e9);
      CK(hipEventRecord(a));
      CK(hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, 0));
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms, a, b));
      printf("memcpy D2H           %6.2f GB/s\n", bytes / (ms * 1e-3) / 1e9);
      fflush(stdout);
    }
    CK(hipHostFree(host));
  }
  return 0;
}
