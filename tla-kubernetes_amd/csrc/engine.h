// engine.h — type-erased engine interface behind the kc_engine_* C-ABI.
#pragma once
#include <stdint.h>

#include <memory>
#include <string>

#include "../../include/kubecheck.h"

namespace kc {

// Kernel kinds timed by the engine (kc_engine_kernel_times order).
enum KernelKind { KK_EXPAND = 0, KK_RESOLVE = 1, KK_SCAN = 2, KK_EMIT = 3, KK_COUNT = 4 };
// diagnostic-only ablation timings (KC_ABLATE=1 in the environment): extra
// launches of cut-down k_claim / k_emit variants on scratch buffers, printed to stderr
enum AblateKind { KA_LDS = KK_COUNT, KA_COMPUTE = KK_COUNT + 1, KA_PLAN = KK_COUNT + 2,
                  KA_E1 = KK_COUNT + 3, KA_E2 = KK_COUNT + 4, KA_E3 = KK_COUNT + 5,
                  KA_FPCHEAP = KK_COUNT + 6, KA_NOAPPLY = KK_COUNT + 7, KA_TOTAL = KK_COUNT + 8 };
// the narrow-level kernel (engine_narrow.h): levels it ran, launches, time
constexpr int KK_NARROW = KA_TOTAL;
constexpr int KK_ALL = KA_TOTAL + 1;

class EngineBase {
 public:
  // the config is kept by value; its one string is copied too
  explicit EngineBase(const kc_model_config& cfg) : cfg_(cfg), spill_dir_(cfg.spill_dir ? cfg.spill_dir : "") {
    cfg_.spill_dir = cfg.spill_dir ? spill_dir_.c_str() : nullptr;
  }
  virtual ~EngineBase() = default;
  virtual int setup() = 0;
  virtual int run(kc_result* res) = 0;
  virtual size_t trace_text(char* buf, size_t cap) const = 0;
  virtual int trace_tuple(int i, uint64_t* out) const = 0;
  virtual int64_t level_tuples(int level, uint64_t* out, uint64_t cap) = 0;
  virtual int state_words() const = 0;
  virtual int tuple_words() const = 0;
  virtual int check_fps(uint64_t* min_gap, double* prob) = 0;
  void set_capture(int level) { capture_level_ = level; }
  void set_timing(bool on) { timing_ = on ? 1 : 0; }
  void kernel_times(double* ms, uint64_t* launches) const {
    for (int k = 0; k < KK_COUNT; ++k) {
      if (ms) ms[k] = ktime_ms_[k];
      if (launches) launches[k] = klaunch_[k];
    }
  }
  void narrow_times(double* ms, uint64_t* launches, uint64_t* levels) const {
    *ms = ktime_ms_[KK_NARROW];
    *launches = klaunch_[KK_NARROW];
    *levels = narrow_levels_;
  }

 protected:
  kc_model_config cfg_;
  std::string spill_dir_;
  int capture_level_ = 0;
  int timing_ = 0;   // 1: HIP events on every kernel; 2: on k_claim only
  double ktime_ms_[KK_ALL] = {};
  uint64_t klaunch_[KK_ALL] = {};
  uint64_t narrow_levels_ = 0;
  bool ablate_ = false;
};

std::unique_ptr<EngineBase> make_engine(const kc_model_config& cfg);
const char* action_name(int a);
// TLA+-style rendering of a canonical tuple (spec_abi.cpp)
std::string format_tuple(const uint64_t* tuple, int nc, int np, int ns, bool ghost = false);

}  // namespace kc
