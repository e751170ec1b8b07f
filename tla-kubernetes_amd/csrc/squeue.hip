// squeue.hip — HBM StateQueue (kc_squeue_*): the C-ABI face of the engine's
// frontier buffers, for callers that drive their own BFS (e.g. a TLC
// StateQueue plugin over packed states; MC.out:5 "DiskStateQueue").
// A FIFO of fixed-width packed states in one device ring buffer.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>

#include "../../include/kubecheck.h"
#include "kc_common.h"

using namespace kc;

struct kc_squeue {
  int device = 0;
  int words = 0;
  uint64_t cap = 0;       // states
  uint64_t head = 0;      // index of the oldest state (mod cap)
  uint64_t size = 0;
  uint64_t* ring = nullptr;
  std::mutex mu;
};

extern "C" {

int kc_squeue_create(int state_words, uint64_t capacity_states, int device, kc_squeue** out) {
  if (!out || state_words <= 0 || capacity_states == 0) {
    set_error("kc_squeue_create: bad argument");
    return -EINVAL;
  }
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    set_error("kc_squeue_create: no HIP device");
    return -ENODEV;
  }
  KC_HIP_TRY(hipSetDevice(device));
  auto* q = new kc_squeue();
  q->device = device;
  q->words = state_words;
  q->cap = capacity_states;
  if (hipMalloc(&q->ring, capacity_states * state_words * 8) != hipSuccess) {
    delete q;
    set_error("kc_squeue_create: out of device memory");
    return -ENOMEM;
  }
  *out = q;
  return 0;
}

void kc_squeue_destroy(kc_squeue* q) {
  if (!q) return;
  (void)hipSetDevice(q->device);
  if (q->ring) (void)hipFree(q->ring);
  delete q;
}

int kc_squeue_enqueue(kc_squeue* q, const uint64_t* states, size_t n) {
  if (!q || (n && !states)) { set_error("kc_squeue_enqueue: bad argument"); return -EINVAL; }
  std::lock_guard<std::mutex> g(q->mu);
  if (q->size + n > q->cap) { set_error("kc_squeue_enqueue: queue full"); return -ENOMEM; }
  KC_HIP_TRY(hipSetDevice(q->device));
  uint64_t done = 0;
  while (done < n) {
    const uint64_t tail = (q->head + q->size) % q->cap;
    const uint64_t m = std::min<uint64_t>(n - done, q->cap - tail);
    KC_HIP_TRY(hipMemcpy(q->ring + tail * q->words, states + done * q->words, m * q->words * 8,
                         hipMemcpyHostToDevice));
    q->size += m;
    done += m;
  }
  return 0;
}

int kc_squeue_dequeue(kc_squeue* q, uint64_t* out, size_t max_n, size_t* n_out) {
  if (!q || !n_out || (max_n && !out)) { set_error("kc_squeue_dequeue: bad argument"); return -EINVAL; }
  std::lock_guard<std::mutex> g(q->mu);
  KC_HIP_TRY(hipSetDevice(q->device));
  const uint64_t n = std::min<uint64_t>(max_n, q->size);
  uint64_t done = 0;
  while (done < n) {
    const uint64_t m = std::min<uint64_t>(n - done, q->cap - q->head);
    KC_HIP_TRY(hipMemcpy(out + done * q->words, q->ring + q->head * q->words, m * q->words * 8,
                         hipMemcpyDeviceToHost));
    q->head = (q->head + m) % q->cap;
    q->size -= m;
    done += m;
  }
  *n_out = n;
  return 0;
}

uint64_t kc_squeue_size(const kc_squeue* q) { return q ? q->size : 0; }

}  // extern "C"
