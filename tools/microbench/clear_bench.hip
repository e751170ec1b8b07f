// clear_bench.hip — ways to zero the compact NP=2 ClaimSet (32 GiB) on
// MI355X (diagnostic only): hipMemsetAsync, and grid-stride kernels of 16-B
// non-temporal or plain stores over different grids / unrolls.
//   hipcc -O3 --offload-arch=gfx950 clear_bench.hip -o clear_bench && ./clear_bench [GiB = 32]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      return 1;                                                                \
    }                                                                          \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int NT, int U>
__global__ void __launch_bounds__(256) k_clear(u32x4* __restrict__ p, uint64_t n16) {
  const u32x4 z = {0u, 0u, 0u, 0u};
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride * U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t k = i + (uint64_t)u * stride;
      if (k < n16) {
        if (NT)
          __builtin_nontemporal_store(z, &p[k]);
        else
          p[k] = z;
      }
    }
  }
}

int main(int argc, char** argv) {
  const uint64_t gib = argc > 1 ? strtoull(argv[1], nullptr, 10) : 32;
  const uint64_t bytes = gib << 30, n16 = bytes / 16;
  u32x4* p = nullptr;
  CK(hipMalloc(&p, bytes));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto run = [&](const char* name, auto launch) -> int {
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(a));
      launch();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      printf("{\"clear\": \"%s\", \"rep\": %d, \"GiB\": %llu, \"ms\": %.3f, \"TB_per_s\": %.3f}\n", name, rep,
             (unsigned long long)gib, ms, bytes / (ms * 1e-3) / 1e12);
      fflush(stdout);
    }
    return 0;
  };
  run("hipMemsetAsync", [&] { (void)hipMemsetAsync(p, 0, bytes, 0); });
  run("nt_g8192_u1", [&] { hipLaunchKernelGGL((k_clear<1, 1>), dim3(8192), dim3(256), 0, 0, p, n16); });
  run("nt_g16384_u1", [&] { hipLaunchKernelGGL((k_clear<1, 1>), dim3(16384), dim3(256), 0, 0, p, n16); });
  run("nt_g4096_u4", [&] { hipLaunchKernelGGL((k_clear<1, 4>), dim3(4096), dim3(256), 0, 0, p, n16); });
  run("nt_g2048_u1", [&] { hipLaunchKernelGGL((k_clear<1, 1>), dim3(2048), dim3(256), 0, 0, p, n16); });
  run("plain_g8192_u1", [&] { hipLaunchKernelGGL((k_clear<0, 1>), dim3(8192), dim3(256), 0, 0, p, n16); });
  run("plain_g16384_u4", [&] { hipLaunchKernelGGL((k_clear<0, 4>), dim3(16384), dim3(256), 0, 0, p, n16); });
  CK(hipFree(p));
  return 0;
}
