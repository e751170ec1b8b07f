// shard.hip — fingerprint-owner-sharded BFS stages (multi-GPU).  Filled in
// below the single-GPU engine; until then every entry point reports ENOSYS.
#include <hip/hip_runtime.h>

#include "../../include/kubecheck.h"
#include "kc_common.h"

using namespace kc;

extern "C" {

int kc_shard_create(const kc_model_config*, int, int, kc_engine** out) {
  if (out) *out = nullptr;
  set_error("kc_shard_create: not built yet");
  return -ENOSYS;
}
int kc_shard_init(kc_engine*, uint64_t*) { set_error("not built"); return -ENOSYS; }
int kc_shard_expand(kc_engine*, uint64_t*) { set_error("not built"); return -ENOSYS; }
int kc_shard_send_buffer(kc_engine*, void**, uint64_t*) { set_error("not built"); return -ENOSYS; }
int kc_shard_recv_buffer(kc_engine*, uint64_t, void**) { set_error("not built"); return -ENOSYS; }
int kc_shard_insert(kc_engine*, uint64_t, uint64_t*, uint64_t*) { set_error("not built"); return -ENOSYS; }
int kc_shard_result(kc_engine*, kc_result*) { set_error("not built"); return -ENOSYS; }

}  // extern "C"
