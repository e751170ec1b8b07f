// engine_util.h — small host helpers shared by the single-GPU engine and the
// sharded (multi-GPU) stages.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/kubecheck.h"
#include "kc_common.h"
#include "kubeapi_spec.h"

namespace kc {

// Grow a device buffer to >= need elements (doubling); keep contents if asked.
template <class T>
int grow_buffer(T*& p, uint64_t& cap, uint64_t need, bool keep, hipStream_t st) {
  if (need <= cap) return 0;
  uint64_t nc = cap ? cap : 1024;
  while (nc < need) nc *= 2;
  T* np = nullptr;
  KC_HIP_TRY(hipMalloc(&np, nc * sizeof(T)));
  if (keep && p && cap) KC_HIP_TRY(hipMemcpyAsync(np, p, cap * sizeof(T), hipMemcpyDeviceToDevice, st));
  if (p) {
    KC_HIP_TRY(hipStreamSynchronize(st));
    KC_HIP_TRY(hipFree(p));
  }
  p = np;
  cap = nc;
  return 0;
}

// The same without doubling: capacity need + 1/8 (buffers sized by a
// level's bound, where doubling would waste up to half of a large one)
template <class T>
int grow_buffer_tight(T*& p, uint64_t& cap, uint64_t need, hipStream_t st) {
  if (need <= cap) return 0;
  const uint64_t nc = need + need / 8 + 1024;
  T* np = nullptr;
  if (p) {
    KC_HIP_TRY(hipStreamSynchronize(st));
    KC_HIP_TRY(hipFree(p));
    p = nullptr;
    cap = 0;
  }
  KC_HIP_TRY(hipMalloc(&np, nc * sizeof(T)));
  p = np;
  cap = nc;
  return 0;
}

// The same for pinned host memory that kernels write directly (the trace
// file with kc_model_config.trace_host); contents always kept.
template <class T>
int grow_host_buffer(T*& p, uint64_t& cap, uint64_t need, hipStream_t st) {
  if (need <= cap) return 0;
  uint64_t nc = cap ? cap : 1024;
  while (nc < need) nc *= 2;
  T* np = nullptr;
  KC_HIP_TRY(hipHostMalloc(&np, nc * sizeof(T)));
  KC_HIP_TRY(hipStreamSynchronize(st));          // kernels may still write the old buffer
  if (p) {
    memcpy(np, p, cap * sizeof(T));
    KC_HIP_TRY(hipHostFree(p));
  }
  p = np;
  cap = nc;
  return 0;
}

// Run-time switches of a model config (constants, seeded variant,
// invariants to check: 0 = none, as TLC with no INVARIANT in the .cfg).
inline Flags flags_of(const kc_model_config& c) {
  Flags f{c.can_fail, c.can_timeout, c.variant};
  f.inv_mask = c.invariants & 7;
  return f;
}

}  // namespace kc
