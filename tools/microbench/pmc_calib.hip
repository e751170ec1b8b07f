// pmc_calib.hip — PMC calibration of HBM byte counters on MI355X (gfx950):
// one kernel per access shape, each moving a KNOWN number of accesses over a
// 32 GiB table (far beyond the 256 MiB Infinity Cache), so that
// rocprofv3's FETCH_SIZE / WRITE_SIZE (and the raw TCC_EA0 request counters)
// can be divided by the access count.  MI355X_MICROARCH.md §HBM: "Other
// access widths are uncalibrated: calibrate on a known byte count in your
// own access pattern".  Diagnostic only; not part of the product.
//
//   hipcc -O3 --offload-arch=gfx950 pmc_calib.hip -o pmc_calib
//   rocprofv3 --pmc FETCH_SIZE -- ./pmc_calib      (one counter set per run)
//
// The shapes are the ones the product's kernels issue:
//   c_stream_load16  coalesced 16 B/lane loads (the guide's reference shape)
//   c_stream_store16 coalesced 16 B/lane stores (reference for WRITE_SIZE)
//   c_rand_load16    one random 16-B load per lane (ClaimSet probe, k_claim)
//   c_rand_load8     one random 8-B load per lane
//   c_rand_cas_new   random 64-bit CAS that succeeds (a new fingerprint)
//   c_rand_cas_fail  random 64-bit CAS that fails (no write)
//   c_rand_store_agent random 8-B agent-scope atomic store (k_claim's claim word)
//   c_rand_store8    random plain 8-B store
//   c_rand_max       random 64-bit atomicMax (settle pass A)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      return 1;                                                                \
    }                                                                          \
  } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
// random 16-B-aligned pair index in [0, npairs)
__device__ __forceinline__ uint64_t rpair(uint64_t i, uint64_t seed, uint64_t npairs) {
  return __umul64hi(mix(seed + i), npairs);
}

__global__ void c_stream_load16(const ulonglong2* __restrict__ t, uint64_t n, unsigned long long* out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const ulonglong2 v = t[i];
  if ((v.x ^ v.y) == 0x1234567ull) out[0] = v.x;
}
__global__ void c_stream_store16(ulonglong2* __restrict__ t, uint64_t n, unsigned long long* out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) t[i] = make_ulonglong2(i, ~i);
}
__global__ void c_rand_load16(const ulonglong2* __restrict__ t, uint64_t npairs, uint64_t n, uint64_t seed,
                              unsigned long long* out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const ulonglong2 v = t[rpair(i, seed, npairs)];
  if ((v.x ^ v.y) == 0x1234567ull) out[0] = v.x;
}
__global__ void c_rand_load8(const unsigned long long* __restrict__ t, uint64_t npairs, uint64_t n,
                             uint64_t seed, unsigned long long* out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const unsigned long long v = t[2 * rpair(i, seed, npairs)];
  if (v == 0x1234567ull) out[0] = v;
}
__global__ void c_rand_cas_new(unsigned long long* __restrict__ t, uint64_t npairs, uint64_t n,
                               uint64_t seed, unsigned long long* out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const unsigned long long v = atomicCAS(t + 2 * rpair(i, seed, npairs), 0ull, (unsigned long long)i + 1);
  if (v == 0x1234567ull) out[0] = v;
}
__global__ void c_rand_cas_fail(unsigned long long* __restrict__ t, uint64_t npairs, uint64_t n,
                                uint64_t seed, unsigned long long* out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  // the table's odd words stay 0: expecting 1 never matches
  const unsigned long long v = atomicCAS(t + 2 * rpair(i, seed, npairs) + 1, 1ull, (unsigned long long)i);
  if (v == 0x1234567ull) out[0] = v;
}
__global__ void c_rand_store_agent(unsigned long long* __restrict__ t, uint64_t npairs, uint64_t n,
                                   uint64_t seed, unsigned long long* out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  __hip_atomic_store(t + 2 * rpair(i, seed, npairs), (unsigned long long)i, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__global__ void c_rand_store8(unsigned long long* __restrict__ t, uint64_t npairs, uint64_t n,
                              uint64_t seed, unsigned long long* out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) t[2 * rpair(i, seed, npairs)] = i;
}
__global__ void c_rand_max(unsigned long long* __restrict__ t, uint64_t npairs, uint64_t n, uint64_t seed,
                           unsigned long long* out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const unsigned long long v = atomicMax(t + 2 * rpair(i, seed, npairs), (unsigned long long)i);
  if (v == 0x1234567ull) out[0] = v;
}

int main() {
  const uint64_t table_bytes = 32ull << 30;
  const uint64_t npairs = table_bytes / 16;
  const uint64_t n_rand = 1ull << 26;         // random accesses per kernel
  const uint64_t n_stream = 1ull << 28;       // 16-B lanes per streaming kernel (4 GiB)
  void* tab = nullptr;
  unsigned long long* out = nullptr;
  CK(hipMalloc(&tab, table_bytes));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(tab, 0, table_bytes));
  CK(hipDeviceSynchronize());
  const dim3 B(256);
  const dim3 Gr((unsigned)((n_rand + 255) / 256)), Gs((unsigned)((n_stream + 255) / 256));
  auto ev = [&](const char* name, auto launch, uint64_t accesses, uint64_t bytes_req) -> int {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a));
    launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("%-20s accesses %12llu requested_bytes %14llu  %8.3f ms  %8.2f G/s\n", name,
           (unsigned long long)accesses, (unsigned long long)bytes_req, ms, accesses / (ms * 1e6));
    fflush(stdout);
    return 0;
  };
  ulonglong2* t2 = (ulonglong2*)tab;
  unsigned long long* t8 = (unsigned long long*)tab;
  if (ev("c_stream_load16", [&] { hipLaunchKernelGGL(c_stream_load16, Gs, B, 0, 0, t2, n_stream, out); },
         n_stream, n_stream * 16)) return 1;
  if (ev("c_stream_store16", [&] { hipLaunchKernelGGL(c_stream_store16, Gs, B, 0, 0, t2, n_stream, out); },
         n_stream, n_stream * 16)) return 1;
  CK(hipMemset(tab, 0, table_bytes));
  CK(hipDeviceSynchronize());
  if (ev("c_rand_load16", [&] { hipLaunchKernelGGL(c_rand_load16, Gr, B, 0, 0, t2, npairs, n_rand, 11ull, out); },
         n_rand, n_rand * 16)) return 1;
  if (ev("c_rand_load8", [&] { hipLaunchKernelGGL(c_rand_load8, Gr, B, 0, 0, t8, npairs, n_rand, 12ull, out); },
         n_rand, n_rand * 8)) return 1;
  if (ev("c_rand_cas_new", [&] { hipLaunchKernelGGL(c_rand_cas_new, Gr, B, 0, 0, t8, npairs, n_rand, 13ull, out); },
         n_rand, n_rand * 8)) return 1;
  if (ev("c_rand_cas_fail", [&] { hipLaunchKernelGGL(c_rand_cas_fail, Gr, B, 0, 0, t8, npairs, n_rand, 14ull, out); },
         n_rand, n_rand * 8)) return 1;
  if (ev("c_rand_store_agent", [&] { hipLaunchKernelGGL(c_rand_store_agent, Gr, B, 0, 0, t8, npairs, n_rand, 15ull, out); },
         n_rand, n_rand * 8)) return 1;
  if (ev("c_rand_store8", [&] { hipLaunchKernelGGL(c_rand_store8, Gr, B, 0, 0, t8, npairs, n_rand, 16ull, out); },
         n_rand, n_rand * 8)) return 1;
  if (ev("c_rand_max", [&] { hipLaunchKernelGGL(c_rand_max, Gr, B, 0, 0, t8, npairs, n_rand, 17ull, out); },
         n_rand, n_rand * 8)) return 1;
  CK(hipFree(tab));
  CK(hipFree(out));
  return 0;
}
