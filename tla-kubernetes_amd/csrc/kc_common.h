// kc_common.h — error plumbing shared by the kubecheck C-ABI.
// No exception or abort crosses the ABI: every entry point returns 0 or a
// negative errno-style code and records a message for kc_last_error().
#pragma once
#include <errno.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <hip/hip_runtime.h>

namespace kc {

void set_error(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
const char* last_error();

}  // namespace kc

#define KC_HIP_TRY(expr)                                                              \
  do {                                                                                \
    hipError_t kc_e_ = (expr);                                                        \
    if (kc_e_ != hipSuccess) {                                                        \
      kc::set_error("%s:%d: %s failed: %s", __FILE__, __LINE__, #expr,                \
                    hipGetErrorString(kc_e_));                                        \
      return kc_e_ == hipErrorOutOfMemory ? -ENOMEM : -EIO;                           \
    }                                                                                 \
  } while (0)

#define KC_TRY(expr)                      \
  do {                                    \
    int kc_r_ = (expr);                   \
    if (kc_r_ < 0) return kc_r_;          \
  } while (0)
