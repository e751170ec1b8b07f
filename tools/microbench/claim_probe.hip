// claim_probe.hip — microbenchmark of ClaimSet lookups as k_settle_rec does
// them (diagnostic only; not part of the product).  Fills a 2^31-slot
// ClaimSet to ~34% with random fingerprints, then looks up present ones.
//
//   hipcc -O3 --offload-arch=gfx950 -I../../tla-kubernetes_amd/csrc claim_probe.hip -o claim_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "fpset_dev.h"

using namespace kc;

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
  return normalize_fp(z ^ (z >> 31));
}

__global__ void k_fill(ClaimEntry* t, uint64_t ns, uint64_t n, unsigned long long* stats) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int r = claimset_claim(t, ns, mix(i), make_claim(2, i), 2);
  if (r != CL_NEW) atomicAdd(stats, 1ull);
}
// as k_settle_rec: claimset_get per lane
__global__ void k_get(const ClaimEntry* t, uint64_t ns, uint64_t n, uint64_t seed, unsigned long long* out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t q = (mix(seed + i) % (n)) ;
  const unsigned long long c = claimset_get(t, ns, mix(q));
  if (c == 0x1234567ull) out[0] = c;
}
// as k_settle_rec: one 256-thread workgroup per tile of `per` records
__global__ void k_tile(const ClaimEntry* t, uint64_t ns, const unsigned long long* rec, uint64_t per,
                       unsigned int* out) {
  __shared__ unsigned int sh[256];
  sh[threadIdx.x] = 0;
  __syncthreads();
  for (uint64_t k = threadIdx.x; k < per; k += 256) {
    const unsigned long long fp = rec[blockIdx.x * per + k];
    const unsigned long long c = claimset_get(t, ns, fp);
    if (c & 1) atomicOr(&sh[k & 255], 1u << (c & 31));
  }
  __syncthreads();
  out[(uint64_t)blockIdx.x * 256 + threadIdx.x] = sh[threadIdx.x];
}
__global__ void k_mkrec(unsigned long long* rec, uint64_t n, uint64_t nfill) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) rec[i] = mix(mix(i + 12345) % nfill);
}
// probe-length histogram
__global__ void k_len(const ClaimEntry* t, uint64_t ns, uint64_t n, unsigned long long* hist) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t fp = mix(i);
  uint64_t k = bucket_of(fp, ns);
  int len = 1;
  while (t[k].fp != fp && len < 63) { k = (k + 1 == ns) ? 0 : k + 1; ++len; }
  atomicAdd(&hist[len], 1ull);
}

int main() {
  const uint64_t ns = 1ull << 31;
  const uint64_t nfill = 740000000ull;
  ClaimEntry* t;
  unsigned long long* d;
  CK(hipMalloc(&t, ns * sizeof(ClaimEntry)));
  CK(hipMalloc(&d, 128 * 8));
  CK(hipMemset(t, 0, ns * sizeof(ClaimEntry)));
  CK(hipMemset(d, 0, 128 * 8));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a));
  hipLaunchKernelGGL(k_fill, dim3((unsigned)((nfill + 255) / 256)), dim3(256), 0, 0, t, ns, nfill, d);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  printf("fill %llu fps (CL_NEW path) in %.1f ms: %.2f G claims/s\n", (unsigned long long)nfill, ms, nfill / ms / 1e6);
  const uint64_t nq = 1ull << 28;
  for (int r = 0; r < 3; ++r) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(k_get, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, 0, t, ns, nq, 77ull + r, d);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    printf("claimset_get x %llu: %.1f ms  %.2f G lookups/s\n", (unsigned long long)nq, ms, nq / ms / 1e6);
  }
  {
    const uint64_t nr = 1ull << 28;
    unsigned long long* rec;
    unsigned int* out;
    CK(hipMalloc(&rec, nr * 8));
    const uint64_t min_per = 64;               // out holds 256 entries per workgroup
    CK(hipMalloc(&out, nr / min_per * 256 * 4));
    hipLaunchKernelGGL(k_mkrec, dim3((unsigned)(nr / 256)), dim3(256), 0, 0, rec, nr, nfill);
    const uint64_t pers[] = {64, 320, 1280, 5120};
    for (uint64_t per : pers) {
      const unsigned nt = (unsigned)(nr / per);
      CK(hipEventRecord(a));
      hipLaunchKernelGGL(k_tile, dim3(nt), dim3(256), 0, 0, t, ns, rec, per, out);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms, a, b));
      printf("tile kernel, %4llu records per 256-thread WG: %.1f ms  %.2f G lookups/s\n",
             (unsigned long long)per, ms, nr / ms / 1e6);
    }
  }
  CK(hipMemset(d, 0, 128 * 8));
  hipLaunchKernelGGL(k_len, dim3((unsigned)((nfill + 255) / 256)), dim3(256), 0, 0, t, ns, nfill, d);
  unsigned long long h[64];
  CK(hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost));
  double tot = 0, s = 0;
  for (int k = 1; k < 64; ++k) { tot += h[k]; s += (double)k * h[k]; }
  printf("probe length: mean %.3f  1:%llu 2:%llu 3:%llu 4:%llu >=5:%llu\n", s / tot, h[1], h[2], h[3], h[4],
         (unsigned long long)(tot - h[1] - h[2] - h[3] - h[4]));
  return 0;
}
