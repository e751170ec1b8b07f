// shard_driver.hip — the native level loop of the fingerprint-owner-sharded
// BFS (kc_group_*): the per-level protocol of kubecheck/distributed.py's
// ShardedModelChecker, in C++ and over RCCL directly, so a level costs the
// kernels, one all-gather, one all-to-all and three host synchronisations
// (expand's counts, the all-gather, insert's new-state count), without a
// Python interpreter in the loop.
//
// Replaces TLC's single-host worker pool for this spec (TLC's own
// distributed mode, RMI TLCServer/TLCWorker, is off in Model_1:
// KubeAPI___Model_1.launch:4-7).  Per BFS level, on every rank:
//
//   expand (claim own successors, count the rest per owner)
//   all-gather of [counts per owner | new states and error key of the level
//                  finished last]            -> error? done? widths, a2a sizes
//   pack records per owner -> all-to-all (grouped ncclSend/ncclRecv, in
//   pieces of <= 256 MiB) -> insert (dedup by min key, emit)  -> advance
//
// The collectives sit behind a small Comm interface with two
// implementations: RcclComm (one shard per process, one process per GPU;
// RCCL resolved at run time with dlopen, so the library loads on hosts
// without it) and LocalComm (R shards of ONE process on one GPU, the
// collectives done by device copies).  The level loop is the same code for
// both, so the multi-rank protocol is exercised on one GPU with R = 2..15
// emulated ranks, and RCCL itself at world 1.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <memory>
#include <string>
#include <vector>

#include "../../include/kubecheck.h"
#include "engine.h"
#include "engine_util.h"
#include "kc_common.h"
#include "shard.h"
#include "shard_narrow.h"

namespace kc {

namespace {

constexpr uint64_t NONE = ~0ull;
constexpr uint64_t KEY44 = (1ull << 44) - 1;
// largest single send/recv of the exchange; also the size of each half of a
// rank's failure sink (Group::run: a rank that cannot grow its exchange
// buffers still takes part in the all-to-all, through the sink)
constexpr uint64_t PIECE_BYTES = 64ull << 20;

// Largest single transfer of the exchange in bytes: PIECE_BYTES, or
// KC_PIECE_BYTES from the environment (tests shrink it so a small model runs
// the multi-piece path).
uint64_t piece_bytes() {
  const char* e = getenv("KC_PIECE_BYTES");
  const long long v = e ? atoll(e) : 0;
  return v > 0 ? (uint64_t)v : PIECE_BYTES;
}

// ---------------------------------------------------------------- RCCL
// Resolved at run time: torch ships its own librccl.so.1; when it is loaded
// already, dlopen returns that copy (one RCCL per process).
struct RcclApi {
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclBroadcast) broadcast = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  bool ok = false;
};

const RcclApi* rccl() {
  static RcclApi api;
  static bool tried = false;
  if (tried) return api.ok ? &api : nullptr;
  tried = true;
  void* h = nullptr;
  for (const char* name : {"librccl.so.1", "librccl.so"}) {
    h = dlopen(name, RTLD_NOW | RTLD_NOLOAD);
    if (h) break;
  }
  for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
    if (h) break;
    h = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
  }
  if (!h) return nullptr;
#define KC_SYM(field, sym) api.field = (decltype(api.field))dlsym(h, #sym); if (!api.field) return nullptr;
  KC_SYM(get_unique_id, ncclGetUniqueId)
  KC_SYM(comm_init_rank, ncclCommInitRank)
  KC_SYM(comm_destroy, ncclCommDestroy)
  KC_SYM(all_gather, ncclAllGather)
  KC_SYM(all_reduce, ncclAllReduce)
  KC_SYM(broadcast, ncclBroadcast)
  KC_SYM(send, ncclSend)
  KC_SYM(recv, ncclRecv)
  KC_SYM(group_start, ncclGroupStart)
  KC_SYM(group_end, ncclGroupEnd)
  KC_SYM(error_string, ncclGetErrorString)
#undef KC_SYM
  api.ok = true;
  return &api;
}

#define KC_NCCL_TRY(expr)                                                                 \
  do {                                                                                    \
    const ncclResult_t kc_n_ = (expr);                                                    \
    if (kc_n_ != ncclSuccess) {                                                           \
      set_error("%s:%d: %s failed: %s", __FILE__, __LINE__, #expr, rccl()->error_string(kc_n_)); \
      return -EIO;                                                                        \
    }                                                                                     \
  } while (0)

}  // namespace

// ---------------------------------------------------------------- exchange plan
// The all-to-all of one rank `me` as the transfers RCCL is given, in order:
// for each peer, its send pieces, then its receive pieces; each piece at most
// `piece` records.  Offsets are in records: into the send buffer grouped by
// destination rank and the receive buffer grouped by source rank.  RCCL pairs
// the k-th send from s to d with the k-th receive at d from s, so both sides
// must cut a pair (s, d) into the same pieces: both cut Mx[s][d] here.
// RcclComm issues this plan; LocalComm executes the same plan with device
// copies, pairing pieces exactly as RCCL does (so emulated ranks test it).
std::vector<Xfer> exchange_plan(const std::vector<std::vector<uint64_t>>& Mx, int me, uint64_t piece) {
  std::vector<Xfer> out;
  const int R = (int)Mx.size();
  if (piece == 0) piece = 1;
  uint64_t soff = 0, roff = 0;
  for (int peer = 0; peer < R; ++peer) {
    const uint64_t ns = Mx[me][peer], nr = Mx[peer][me];
    for (uint64_t k = 0; k < ns; k += piece) out.push_back({peer, 1, soff + k, std::min(piece, ns - k)});
    for (uint64_t k = 0; k < nr; k += piece) out.push_back({peer, 0, roff + k, std::min(piece, nr - k)});
    soff += ns;
    roff += nr;
  }
  return out;
}

namespace {

// ---------------------------------------------------------------- Comm
// Collectives over the ranks; every call is made by the driver on behalf of
// all the shards this process holds (LocalComm: every rank; RcclComm: one).
class Comm {
 public:
  virtual ~Comm() = default;
  // rows[i] = the row of local shard i (all rows the same length L);
  // out = rank-major rows of every rank (world * L)
  virtual int all_gather(const std::vector<std::vector<uint64_t>>& rows, std::vector<uint64_t>& out) = 0;
  // per local shard: send buffer grouped by destination; Mx[src][dst] record
  // counts of every rank; recv buffers grouped by source.  sunk[i]: local
  // shard i failed without buffers for this exchange; it still takes part
  // (its peers are waiting for it), sending zeroed records from the comm's
  // sink and receiving into it, every piece at the sink's start.
  virtual int all_to_all(const std::vector<void*>& send, const std::vector<std::vector<uint64_t>>& Mx,
                         uint64_t rec_bytes, const std::vector<void*>& recv, const std::vector<char>& sunk) = 0;
  // *v: in on the local shard of rank `root` (if any), out everywhere
  virtual int broadcast(int root, uint64_t* v) = 0;
  // v[i] = the vector of local shard i; out = the element-wise sum over ranks
  virtual int all_reduce_sum(const std::vector<std::vector<uint64_t>>& v, std::vector<uint64_t>& out) = 0;
  // Device-row all-gather: row_buffer(i, L) is where local shard i's kernels
  // write its row of L words; all_gather_dev gathers every local shard's row
  // (on their streams), syncs, and returns the rank-major rows.  nullptr:
  // not supported, use all_gather.
  virtual uint64_t* row_buffer(size_t i, size_t L) {
    (void)i;
    (void)L;
    return nullptr;
  }
  virtual int all_gather_dev(size_t L, std::vector<uint64_t>& out) {
    (void)L;
    (void)out;
    set_error("all_gather_dev: not supported by this communicator");
    return -EINVAL;
  }
  // The narrow levels' fixed exchange (shard_narrow.h): slot p of local
  // shard i's send buffer goes to rank p's receive buffer, at slot (rank
  // of i); every slot is slot_bytes.  The same transfers every level,
  // whatever the ranks' device state, so they always match.
  virtual int sn_exchange(const std::vector<void*>& send, const std::vector<void*>& recv, uint64_t slot_bytes) = 0;
  // TLC order (ShardBase::tlc_masks): buf[i] = local shard i's n device words
  // (nullptr: a failed shard, which adds zeroes); every buffer becomes the
  // element-wise sum over the ranks, stream-ordered on its shard's stream
  virtual int all_reduce_dev_u32(const std::vector<uint32_t*>& buf, uint64_t n) = 0;
  // one rank in one process and every collective the identity: the level
  // loop needs no gather (Group::run's solo levels)
  virtual bool trivial() const { return false; }
};

// The emulated exchange's copies in one launch (LocalComm): a transfer list
// of (src, dst, 16-B units) — src == nullptr writes zeroes — cut into 64 KiB
// chunks; block b finds its transfer in the chunk prefix (at most a few
// hundred transfers: R^2 pieces).  One launch per exchange instead of one
// copy per piece (R = 8: 64+ copy launches per level, 47 ms of an emulated
// NP=2 check spent in ~13K copies, profiles/r05a_attr_R8.json).
struct CopyXfer {
  const ulonglong2* src;
  ulonglong2* dst;
  uint64_t units;        // 16-B units
  uint64_t chunk0;       // first chunk of this transfer (prefix over transfers)
};
constexpr uint64_t COPY_CHUNK = 4096;   // 16-B units per chunk (64 KiB)
__global__ void __launch_bounds__(256) k_multi_copy(const CopyXfer* __restrict__ x, int nx) {
  __shared__ int sh_x;
  if (threadIdx.x == 0) {
    int lo = 0, hi = nx - 1;        // last transfer with chunk0 <= blockIdx.x
    while (lo < hi) {
      const int mid = (lo + hi + 1) / 2;
      if (x[mid].chunk0 <= blockIdx.x) lo = mid; else hi = mid - 1;
    }
    sh_x = lo;
  }
  __syncthreads();
  const CopyXfer t = x[sh_x];
  const uint64_t u0 = (blockIdx.x - t.chunk0) * COPY_CHUNK;
  const uint64_t u1 = u0 + COPY_CHUNK < t.units ? u0 + COPY_CHUNK : t.units;
  for (uint64_t u = u0 + threadIdx.x; u < u1; u += blockDim.x)
    t.dst[u] = t.src ? t.src[u] : make_ulonglong2(0ull, 0ull);
}

// LocalComm's all_reduce_dev_u32: every emulated rank's words summed into all
// of them (nullptr: a failed rank, zeroes)
struct SumBufs {
  uint32_t* p[16];
  int n;
};
__global__ void __launch_bounds__(256) k_sum_u32(SumBufs b, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t v = 0;
    for (int r = 0; r < b.n; ++r)
      if (b.p[r]) v += b.p[r][i];
    for (int r = 0; r < b.n; ++r)
      if (b.p[r]) b.p[r][i] = v;
  }
}

class LocalComm final : public Comm {
 public:
  explicit LocalComm(std::vector<ShardBase*> shards) : s_(std::move(shards)) {}
  ~LocalComm() override {
    if (rows_) (void)hipFree(rows_);
    if (hrows_) (void)hipHostFree(hrows_);
    if (xd_) (void)hipFree(xd_);
    if (xh_) (void)hipHostFree(xh_);
  }
  int all_gather(const std::vector<std::vector<uint64_t>>& rows, std::vector<uint64_t>& out) override {
    out.clear();
    for (const auto& r : rows) out.insert(out.end(), r.begin(), r.end());
    return 0;
  }
  // one device row per emulated rank, gathered by copies (the rows the
  // kernels write in the RCCL path, k_owner_totals, are exercised here)
  uint64_t* row_buffer(size_t i, size_t L) override {
    const size_t need = s_.size() * L;
    if (need > rows_cap_) {
      if (rows_) (void)hipFree(rows_);
      if (hrows_) (void)hipHostFree(hrows_);
      rows_ = nullptr;
      hrows_ = nullptr;
      rows_cap_ = 0;
      if (hipMalloc(&rows_, need * 8) != hipSuccess || hipHostMalloc(&hrows_, need * 8) != hipSuccess) return nullptr;
      rows_cap_ = need;
    }
    return rows_ + i * L;
  }
  int all_gather_dev(size_t L, std::vector<uint64_t>& out) override {
    for (size_t i = 0; i < s_.size(); ++i)
      KC_HIP_TRY(hipMemcpyAsync(hrows_ + i * L, rows_ + i * L, L * 8, hipMemcpyDeviceToHost, s_[i]->stream()));
    for (auto* s : s_) KC_HIP_TRY(hipStreamSynchronize(s->stream()));
    out.assign(hrows_, hrows_ + s_.size() * L);
    return 0;
  }
  // every rank's exchange plan, its pieces paired as RCCL pairs them: the
  // k-th send from src to dst with the k-th receive at dst from src
  int all_to_all(const std::vector<void*>& send, const std::vector<std::vector<uint64_t>>& Mx,
                 uint64_t rb, const std::vector<void*>& recv, const std::vector<char>& sunk) override {
    const int R = (int)s_.size();
    const uint64_t piece = std::max<uint64_t>(1, piece_bytes() / rb);
    for (auto* s : s_) KC_HIP_TRY(hipStreamSynchronize(s->stream()));   // every pack is done
    std::vector<std::vector<Xfer>> plan(R);
    for (int r = 0; r < R; ++r) plan[r] = exchange_plan(Mx, r, piece);
    xfers_.clear();
    for (int dst = 0; dst < R; ++dst) {
      for (int src = 0; src < R; ++src) {
        std::vector<const Xfer*> sends, recvs;
        for (const auto& x : plan[src])
          if (x.send && x.peer == dst) sends.push_back(&x);
        for (const auto& x : plan[dst])
          if (!x.send && x.peer == src) recvs.push_back(&x);
        if (sends.size() != recvs.size()) {
          set_error("exchange plan: %zu sends from rank %d to %d but %zu receives", sends.size(), src, dst,
                    recvs.size());
          return -EIO;
        }
        for (size_t k = 0; k < sends.size(); ++k) {
          if (sends[k]->n != recvs[k]->n) {
            set_error("exchange plan: piece %zu of %d->%d: %llu sent, %llu received", k, src, dst,
                      (unsigned long long)sends[k]->n, (unsigned long long)recvs[k]->n);
            return -EIO;
          }
          if (sunk[dst]) continue;                  // (the failed rank's sink takes it)
          char* to = (char*)recv[dst] + recvs[k]->off * rb;
          // a failed sender's records are zeroes
          const char* from = sunk[src] ? nullptr : (const char*)send[src] + sends[k]->off * rb;
          add_xfer(from, to, sends[k]->n * rb);
        }
      }
    }
    return run_xfers();
  }
  int sn_exchange(const std::vector<void*>& send, const std::vector<void*>& recv, uint64_t slot) override {
    const int R = (int)s_.size();
    if (R == 1) return 0;
    for (auto* s : s_) KC_HIP_TRY(hipStreamSynchronize(s->stream()));   // every rank's slots are written
    xfers_.clear();
    for (int d = 0; d < R; ++d)
      for (int src = 0; src < R; ++src)
        if (src != d) add_xfer((const char*)send[src] + d * slot, (char*)recv[d] + src * slot, slot);
    return run_xfers();    // (synchronised: before any rank's next pack)
  }
  int all_reduce_dev_u32(const std::vector<uint32_t*>& buf, uint64_t n) override {
    if (s_.size() == 1 || n == 0) return 0;
    for (auto* s : s_) KC_HIP_TRY(hipStreamSynchronize(s->stream()));
    SumBufs b{};
    b.n = (int)s_.size();
    for (size_t i = 0; i < s_.size(); ++i) b.p[i] = buf[i];
    hipStream_t st = s_[0]->stream();
    hipLaunchKernelGGL(k_sum_u32, dim3((unsigned)std::min<uint64_t>((n + 255) / 256, 65536)), dim3(256), 0, st, b, n);
    KC_HIP_TRY(hipGetLastError());
    KC_HIP_TRY(hipStreamSynchronize(st));
    return 0;
  }
  int broadcast(int, uint64_t*) override { return 0; }   // the driver read it from the local root
  bool trivial() const override { return s_.size() == 1; }
  int all_reduce_sum(const std::vector<std::vector<uint64_t>>& v, std::vector<uint64_t>& out) override {
    out.assign(v[0].size(), 0);
    for (const auto& x : v)
      for (size_t k = 0; k < x.size(); ++k) out[k] += x[k];
    return 0;
  }

 private:
  void add_xfer(const void* src, void* dst, uint64_t bytes) {
    if (!bytes) return;
    xfers_.push_back(CopyXfer{(const ulonglong2*)src, (ulonglong2*)dst, bytes / 16, 0});
  }
  // the list in one launch on rank 0's stream (every stream is idle: the
  // callers synchronised them), then that stream's sync
  int run_xfers() {
    if (xfers_.empty()) return 0;
    uint64_t chunks = 0;
    for (auto& x : xfers_) {
      x.chunk0 = chunks;
      chunks += (x.units + COPY_CHUNK - 1) / COPY_CHUNK;
    }
    if (chunks >= (1ull << 31)) {
      set_error("emulated exchange: %llu chunks in one launch", (unsigned long long)chunks);
      return -EIO;
    }
    if (xfers_.size() > xcap_) {
      if (xd_) KC_HIP_TRY(hipFree(xd_));
      if (xh_) KC_HIP_TRY(hipHostFree(xh_));
      xd_ = nullptr;
      xh_ = nullptr;
      xcap_ = std::max<size_t>(2 * xfers_.size(), 256);
      KC_HIP_TRY(hipMalloc(&xd_, xcap_ * sizeof(CopyXfer)));
      KC_HIP_TRY(hipHostMalloc(&xh_, xcap_ * sizeof(CopyXfer)));
    }
    memcpy(xh_, xfers_.data(), xfers_.size() * sizeof(CopyXfer));
    hipStream_t st = s_[0]->stream();
    KC_HIP_TRY(hipMemcpyAsync(xd_, xh_, xfers_.size() * sizeof(CopyXfer), hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_multi_copy, dim3((unsigned)chunks), dim3(256), 0, st, xd_, (int)xfers_.size());
    KC_HIP_TRY(hipGetLastError());
    KC_HIP_TRY(hipStreamSynchronize(st));
    return 0;
  }
  std::vector<ShardBase*> s_;
  uint64_t* rows_ = nullptr;
  uint64_t* hrows_ = nullptr;
  size_t rows_cap_ = 0;
  std::vector<CopyXfer> xfers_;
  CopyXfer* xd_ = nullptr;
  CopyXfer* xh_ = nullptr;
  size_t xcap_ = 0;
};

class RcclComm final : public Comm {
 public:
  // At world 1 every collective is the identity, done on the host; with
  // KC_RCCL_FORCE=1 they still go through RCCL (tests of the RCCL path).
  RcclComm(ShardBase* s, ncclComm_t c) : s_(s), comm_(c) {
    const char* f = getenv("KC_RCCL_FORCE");
    trivial_ = s->world() == 1 && !(f && f[0] == '1');
  }
  ~RcclComm() override {
    if (sink_) (void)hipFree(sink_);
    if (buf_) (void)hipFree(buf_);
    if (hbuf_) (void)hipHostFree(hbuf_);
    if (comm_ && rccl()) (void)rccl()->comm_destroy(comm_);
  }
  int all_gather(const std::vector<std::vector<uint64_t>>& rows, std::vector<uint64_t>& out) override {
    if (trivial_) {
      out = rows[0];
      return 0;
    }
    const size_t L = rows[0].size(), R = (size_t)s_->world();
    KC_TRY(scratch(L * (R + 1)));
    hipStream_t st = s_->stream();
    memcpy(hbuf_, rows[0].data(), L * 8);
    KC_HIP_TRY(hipMemcpyAsync(buf_, hbuf_, L * 8, hipMemcpyHostToDevice, st));
    KC_NCCL_TRY(rccl()->all_gather(buf_, buf_ + L, L, ncclUint64, comm_, st));
    KC_HIP_TRY(hipMemcpyAsync(hbuf_ + L, buf_ + L, L * R * 8, hipMemcpyDeviceToHost, st));
    KC_HIP_TRY(hipStreamSynchronize(st));
    out.assign(hbuf_ + L, hbuf_ + L + L * R);
    return 0;
  }
  uint64_t* row_buffer(size_t i, size_t L) override {
    if (i != 0 || trivial_ || scratch(L * ((size_t)s_->world() + 1))) return nullptr;
    return buf_;
  }
  int all_gather_dev(size_t L, std::vector<uint64_t>& out) override {
    const size_t R = (size_t)s_->world();
    hipStream_t st = s_->stream();
    KC_NCCL_TRY(rccl()->all_gather(buf_, buf_ + L, L, ncclUint64, comm_, st));
    KC_HIP_TRY(hipMemcpyAsync(hbuf_ + L, buf_ + L, L * R * 8, hipMemcpyDeviceToHost, st));
    KC_HIP_TRY(hipStreamSynchronize(st));
    out.assign(hbuf_ + L, hbuf_ + L + L * R);
    return 0;
  }
  // The failure sink: allocated with the communicator (a rank that failed
  // for want of memory could not allocate it then), two halves of one piece.
  int make_sink() {
    if (trivial_ || sink_) return 0;
    KC_HIP_TRY(hipMalloc(&sink_, 2 * piece_bytes()));
    return 0;
  }
  int all_to_all(const std::vector<void*>& send, const std::vector<std::vector<uint64_t>>& Mx, uint64_t rb,
                 const std::vector<void*>& recv, const std::vector<char>& sunk) override {
    const uint64_t rw = rb / 8;                       // records are whole 8-byte words
    const uint64_t piece = std::max<uint64_t>(1, piece_bytes() / rb);   // records per piece
    hipStream_t st = s_->stream();
    const std::vector<Xfer> plan = exchange_plan(Mx, s_->rank(), piece);
    const bool sk = sunk[0] != 0;
    if (sk && !sink_) {
      set_error("kc_group_run: rank %d failed without a failure sink", s_->rank());
      return -EIO;
    }
    if (sk) KC_HIP_TRY(hipMemsetAsync(sink_, 0, piece * rb, st));
    KC_NCCL_TRY(rccl()->group_start());
    for (const auto& x : plan) {
      if (x.send)
        KC_NCCL_TRY(rccl()->send(sk ? (const uint64_t*)sink_ : (const uint64_t*)send[0] + x.off * rw, x.n * rw,
                                 ncclUint64, x.peer, comm_, st));
      else
        KC_NCCL_TRY(rccl()->recv(sk ? (uint64_t*)sink_ + piece * rw : (uint64_t*)recv[0] + x.off * rw, x.n * rw,
                                 ncclUint64, x.peer, comm_, st));
    }
    KC_NCCL_TRY(rccl()->group_end());
    return 0;                                          // stream-ordered before insert
  }
  // enqueued on the shard's stream between its pack and its receive kernels:
  // no host synchronisation
  int sn_exchange(const std::vector<void*>& send, const std::vector<void*>& recv, uint64_t slot) override {
    const int R = s_->world(), me = s_->rank();
    if (R == 1) return 0;
    const uint64_t w = slot / 8;
    hipStream_t st = s_->stream();
    KC_NCCL_TRY(rccl()->group_start());
    for (int p = 0; p < R; ++p) {
      if (p == me) continue;
      KC_NCCL_TRY(rccl()->send((const uint64_t*)send[0] + p * w, w, ncclUint64, p, comm_, st));
      KC_NCCL_TRY(rccl()->recv((uint64_t*)recv[0] + p * w, w, ncclUint64, p, comm_, st));
    }
    KC_NCCL_TRY(rccl()->group_end());
    return 0;
  }
  bool trivial() const override { return trivial_; }
  int all_reduce_dev_u32(const std::vector<uint32_t*>& buf, uint64_t n) override {
    if (trivial_ || n == 0) return 0;
    hipStream_t st = s_->stream();
    uint32_t* p = buf[0];
    if (!p) {                      // a failed rank: zeroes, through the scratch
      KC_TRY(scratch((n + 1) / 2));
      p = reinterpret_cast<uint32_t*>(buf_);
      KC_HIP_TRY(hipMemsetAsync(p, 0, n * 4, st));
    }
    KC_NCCL_TRY(rccl()->all_reduce(p, p, n, ncclUint32, ncclSum, comm_, st));
    return 0;
  }
  int broadcast(int root, uint64_t* v) override {
    if (trivial_) return 0;
    KC_TRY(scratch(1));
    hipStream_t st = s_->stream();
    hbuf_[0] = *v;
    KC_HIP_TRY(hipMemcpyAsync(buf_, hbuf_, 8, hipMemcpyHostToDevice, st));
    KC_NCCL_TRY(rccl()->broadcast(buf_, buf_, 1, ncclUint64, root, comm_, st));
    KC_HIP_TRY(hipMemcpyAsync(hbuf_, buf_, 8, hipMemcpyDeviceToHost, st));
    KC_HIP_TRY(hipStreamSynchronize(st));
    *v = hbuf_[0];
    return 0;
  }
  int all_reduce_sum(const std::vector<std::vector<uint64_t>>& v, std::vector<uint64_t>& out) override {
    if (trivial_) {
      out = v[0];
      return 0;
    }
    const size_t L = v[0].size();
    KC_TRY(scratch(L));
    hipStream_t st = s_->stream();
    memcpy(hbuf_, v[0].data(), L * 8);
    KC_HIP_TRY(hipMemcpyAsync(buf_, hbuf_, L * 8, hipMemcpyHostToDevice, st));
    KC_NCCL_TRY(rccl()->all_reduce(buf_, buf_, L, ncclUint64, ncclSum, comm_, st));
    KC_HIP_TRY(hipMemcpyAsync(hbuf_, buf_, L * 8, hipMemcpyDeviceToHost, st));
    KC_HIP_TRY(hipStreamSynchronize(st));
    out.assign(hbuf_, hbuf_ + L);
    return 0;
  }

 private:
  // device scratch for the small collectives and a pinned host mirror, so
  // their host <-> device copies are asynchronous DMA (no pageable staging)
  int scratch(size_t words) {
    if (words <= cap_) return 0;
    if (buf_) KC_HIP_TRY(hipFree(buf_));
    if (hbuf_) KC_HIP_TRY(hipHostFree(hbuf_));
    buf_ = nullptr;
    hbuf_ = nullptr;
    cap_ = std::max<size_t>(words, 256);
    KC_HIP_TRY(hipMalloc(&buf_, cap_ * 8));
    KC_HIP_TRY(hipHostMalloc(&hbuf_, cap_ * 8));
    return 0;
  }
  ShardBase* s_;
  bool trivial_ = false;
  ncclComm_t comm_ = nullptr;
  uint64_t* sink_ = nullptr;
  uint64_t* buf_ = nullptr;
  uint64_t* hbuf_ = nullptr;
  size_t cap_ = 0;
};

// One shard per process; the collectives are the caller's (kc_host_comm:
// MPI, gloo, sockets), on host buffers.  Structured like RcclComm: the
// kernels write the all-gather row in device memory (k_owner_totals), and the
// all-to-all is the same exchange plan, handed over whole (byte offsets into
// pinned staging copies of the send and receive buffers).  Besides serving
// hosts without RCCL, it runs the one-shard-per-process loop at world > 1 on
// a single GPU, which RCCL refuses ("duplicate GPU"): tests/test_gpu_hostcomm.py.
class HostComm final : public Comm {
 public:
  HostComm(ShardBase* s, const kc_host_comm& ops) : s_(s), ops_(ops) {}
  ~HostComm() override {
    if (drow_) (void)hipFree(drow_);
    if (hrow_) (void)hipHostFree(hrow_);
    if (hsend_) (void)hipHostFree(hsend_);
    if (hrecv_) (void)hipHostFree(hrecv_);
  }
  int all_gather(const std::vector<std::vector<uint64_t>>& rows, std::vector<uint64_t>& out) override {
    const size_t L = rows[0].size();
    out.assign(L * (size_t)s_->world(), 0);
    return call(ops_.all_gather(ops_.ctx, rows[0].data(), L, out.data()), "all_gather");
  }
  uint64_t* row_buffer(size_t i, size_t L) override {
    if (i != 0) return nullptr;
    if (L > row_cap_) {
      if (drow_) (void)hipFree(drow_);
      if (hrow_) (void)hipHostFree(hrow_);
      drow_ = nullptr;
      hrow_ = nullptr;
      row_cap_ = 0;
      if (hipMalloc(&drow_, L * 8) != hipSuccess || hipHostMalloc(&hrow_, L * 8) != hipSuccess) return nullptr;
      row_cap_ = L;
    }
    return drow_;
  }
  int all_gather_dev(size_t L, std::vector<uint64_t>& out) override {
    KC_HIP_TRY(hipMemcpyAsync(hrow_, drow_, L * 8, hipMemcpyDeviceToHost, s_->stream()));
    KC_HIP_TRY(hipStreamSynchronize(s_->stream()));
    out.assign(L * (size_t)s_->world(), 0);
    return call(ops_.all_gather(ops_.ctx, hrow_, L, out.data()), "all_gather");
  }
  int all_to_all(const std::vector<void*>& send, const std::vector<std::vector<uint64_t>>& Mx, uint64_t rb,
                 const std::vector<void*>& recv, const std::vector<char>& sunk) override {
    const int me = s_->rank(), R = s_->world();
    if (sunk[0]) return sunk_exchange(Mx, rb);
    uint64_t ns = 0, nr = 0;
    for (int p = 0; p < R; ++p) {
      ns += Mx[me][p];
      nr += Mx[p][me];
    }
    KC_TRY(pinned(hsend_, hsend_cap_, ns * rb));
    KC_TRY(pinned(hrecv_, hrecv_cap_, nr * rb));
    hipStream_t st = s_->stream();
    if (ns) KC_HIP_TRY(hipMemcpyAsync(hsend_, send[0], ns * rb, hipMemcpyDeviceToHost, st));
    KC_HIP_TRY(hipStreamSynchronize(st));            // every record packed and staged
    const std::vector<Xfer> plan = exchange_plan(Mx, me, std::max<uint64_t>(1, piece_bytes() / rb));
    std::vector<uint64_t> xf(4 * plan.size());
    for (size_t k = 0; k < plan.size(); ++k) {
      xf[4 * k] = (uint64_t)plan[k].peer;
      xf[4 * k + 1] = (uint64_t)plan[k].send;
      xf[4 * k + 2] = plan[k].off * rb;
      xf[4 * k + 3] = plan[k].n * rb;
    }
    KC_TRY(call(ops_.exchange(ops_.ctx, xf.data(), (int)plan.size(), hsend_, hrecv_), "exchange"));
    if (nr) KC_HIP_TRY(hipMemcpyAsync(recv[0], hrecv_, nr * rb, hipMemcpyHostToDevice, st));
    return 0;                                        // stream-ordered before insert
  }
  // synchronous: the caller's transport works on host buffers
  int sn_exchange(const std::vector<void*>& send, const std::vector<void*>& recv, uint64_t slot) override {
    const int R = s_->world(), me = s_->rank();
    if (R == 1) return 0;
    KC_TRY(pinned(hsend_, hsend_cap_, R * slot));
    KC_TRY(pinned(hrecv_, hrecv_cap_, R * slot));
    hipStream_t st = s_->stream();
    KC_HIP_TRY(hipMemcpyAsync(hsend_, send[0], R * slot, hipMemcpyDeviceToHost, st));
    KC_HIP_TRY(hipStreamSynchronize(st));
    std::vector<uint64_t> xf;
    for (int p = 0; p < R; ++p) {
      if (p == me) continue;
      for (uint64_t dir : {1ull, 0ull}) {
        xf.push_back((uint64_t)p);
        xf.push_back(dir);
        xf.push_back(p * slot);
        xf.push_back(slot);
      }
    }
    KC_TRY(call(ops_.exchange(ops_.ctx, xf.data(), (int)(xf.size() / 4), hsend_, hrecv_), "exchange"));
    KC_HIP_TRY(hipMemcpyAsync(recv[0], hrecv_, R * slot, hipMemcpyHostToDevice, st));
    return 0;
  }
  int broadcast(int root, uint64_t* v) override { return call(ops_.broadcast(ops_.ctx, root, v), "broadcast"); }
  // (the caller's all_reduce_sum works on 64-bit host words: two u32 words
  // travel in each.  The only caller is tlc_order's mask words, whose bits
  // are disjoint across ranks — each new state has one winner — so a word's
  // sum is its OR, never above 2^32 - 1, and the low half cannot carry into
  // the high one)
  int all_reduce_dev_u32(const std::vector<uint32_t*>& buf, uint64_t n) override {
    if (n == 0) return 0;
    hipStream_t st = s_->stream();
    std::vector<uint64_t> w((n + 1) / 2, 0);
    if (buf[0]) {
      KC_HIP_TRY(hipMemcpyAsync(w.data(), buf[0], n * 4, hipMemcpyDeviceToHost, st));
      KC_HIP_TRY(hipStreamSynchronize(st));
    }
    KC_TRY(call(ops_.all_reduce_sum(ops_.ctx, w.data(), w.size()), "all_reduce_sum"));
    if (!buf[0]) return 0;
    KC_HIP_TRY(hipMemcpyAsync(buf[0], w.data(), n * 4, hipMemcpyHostToDevice, st));
    KC_HIP_TRY(hipStreamSynchronize(st));
    return 0;
  }
  int all_reduce_sum(const std::vector<std::vector<uint64_t>>& v, std::vector<uint64_t>& out) override {
    out = v[0];
    return call(ops_.all_reduce_sum(ops_.ctx, out.data(), out.size()), "all_reduce_sum");
  }

 private:
  // A failed rank's part of the exchange: zeroes out, every piece in and out
  // at the start of a host sink (plain memory: its pinned staging is what it
  // may have failed to grow).
  int sunk_exchange(const std::vector<std::vector<uint64_t>>& Mx, uint64_t rb) {
    const uint64_t piece = std::max<uint64_t>(1, piece_bytes() / rb);
    const std::vector<Xfer> plan = exchange_plan(Mx, s_->rank(), piece);
    std::vector<uint64_t> xf(4 * plan.size());
    for (size_t k = 0; k < plan.size(); ++k) {
      xf[4 * k] = (uint64_t)plan[k].peer;
      xf[4 * k + 1] = (uint64_t)plan[k].send;
      xf[4 * k + 2] = 0;
      xf[4 * k + 3] = plan[k].n * rb;
    }
    std::vector<uint8_t> out(piece * rb, 0), in(piece * rb);
    return call(ops_.exchange(ops_.ctx, xf.data(), (int)plan.size(), out.data(), in.data()), "exchange");
  }
  static int call(int rc, const char* what) {
    if (rc < 0) {
      set_error("kc_host_comm %s failed (%d)", what, rc);
      return -EIO;
    }
    return 0;
  }
  // pinned staging, grown (the previous contents are not kept); the stream
  // is idle here: every use follows a synchronisation of it
  int pinned(uint8_t*& p, uint64_t& cap, uint64_t bytes) {
    if (bytes <= cap) return 0;
    KC_HIP_TRY(hipStreamSynchronize(s_->stream()));
    if (p) KC_HIP_TRY(hipHostFree(p));
    p = nullptr;
    cap = std::max<uint64_t>(bytes, 2 * cap);
    KC_HIP_TRY(hipHostMalloc(&p, cap));
    return 0;
  }
  ShardBase* s_;
  kc_host_comm ops_;
  uint64_t* drow_ = nullptr;
  uint64_t* hrow_ = nullptr;
  size_t row_cap_ = 0;
  uint8_t* hsend_ = nullptr;
  uint8_t* hrecv_ = nullptr;
  uint64_t hsend_cap_ = 0, hrecv_cap_ = 0;
};

}  // namespace

// ---------------------------------------------------------------- driver
class Group {
 public:
  Group(std::vector<ShardBase*> local, std::unique_ptr<Comm> comm, const kc_model_config& cfg)
      : local_(std::move(local)), comm_(std::move(comm)), cfg_(cfg) {
    const char* dr = getenv("KC_DEVROW");     // KC_DEVROW=0: host rows + expand's own sync (A/B)
    dev_row_off_ = dr && dr[0] == '0';
    // fault injection for the failure-path tests: KC_FAULT=rank:level:stage
    // (stage 0 expand, 1 pack, 2 insert, 3 after the all-gather as if the
    // exchange buffers could not be grown) fails that rank's stage with -EIO
    const char* fl = getenv("KC_FAULT");
    if (fl && sscanf(fl, "%d:%d:%d", &fault_rank_, &fault_level_, &fault_stage_) != 3) fault_rank_ = -1;
    world_ = local_[0]->world();
    cfg_.spill_dir = nullptr;
    for (auto* s : local_) s->set_async_pack(true);
    send_.assign(local_.size(), nullptr);
    recv_.assign(local_.size(), nullptr);
    send_cap_.assign(local_.size(), 0);
    recv_cap_.assign(local_.size(), 0);
    // device-driven narrow levels (shard_narrow.h); KC_SNARROW=0: every level
    // on the counted path; KC_SN_SLOT: records per peer slot
    const char* sn = getenv("KC_SNARROW");
    sn_on_ = !(sn && sn[0] == '0');
    const char* sc = getenv("KC_SN_SLOT");
    sn_cap_ = sc && atoi(sc) > 0 ? (uint32_t)atoi(sc) : SN_SLOT_DEFAULT;
    // KC_SOLO=0: a world-1 group runs the gather path too (A/B)
    const char* so = getenv("KC_SOLO");
    solo_off_ = so && so[0] == '0';
    // KC_SERIAL=1 (diagnostic): each local shard's stage is synchronised
    // before the next shard's launches, so emulated ranks' kernels never
    // overlap and a kernel trace attributes time per rank (Stream_Id)
    const char* se = getenv("KC_SERIAL");
    serial_ = se && se[0] == '1';
    // the deferred frontier on the counted levels (round 5); KC_SDEFER=0:
    // every insert materialises its new states (A/B)
    const char* sd = getenv("KC_SDEFER");
    defer_on_ = !(sd && sd[0] == '0');
  }
  // The narrow levels' buffers, allocated with the group (a failure here is
  // the caller's before any collective of a run).
  int setup() {
    // (a seen-set that spills takes the counted path at every level: its
    // cold check runs between the settle passes and the emit.  Every rank
    // runs with the same configuration, so they all decide alike.)
    if (cfg_.seen_hbm_bytes) sn_on_ = false;
    // TLC order: counted levels only, on the deferred frontier (ShardBase::tlc)
    tlc_ = local_[0]->tlc();
    if (tlc_) {
      sn_on_ = false;
      defer_on_ = true;
    }
    for (auto* s : local_) s->set_deferred(defer_on_ && !cfg_.seen_hbm_bytes);
    if (!sn_on_) return 0;
    for (auto* s : local_) KC_TRY(s->sn_setup(sn_cap_));
    return 0;
  }
  ~Group() {
    if (h_fail_) (void)hipHostFree(h_fail_);
    for (size_t i = 0; i < local_.size(); ++i) {
      (void)hipSetDevice(local_[i]->device());
      if (send_[i]) (void)hipFree(send_[i]);
      if (recv_[i]) (void)hipFree(recv_[i]);
    }
  }
  int run(kc_result* res);
  const std::vector<std::vector<uint64_t>>& trace() const { return trace_; }
  uint64_t records_sent() const { return sent_; }

 private:
  ShardBase* owner_local(int rank) {
    for (auto* s : local_)
      if (s->rank() == rank) return s;
    return nullptr;
  }
  // every rank takes part in the broadcast; a failed lookup on the owner
  // travels as NONE, so all ranks fail together
  int query_parent(int rank, int level, uint64_t idx, uint64_t* key) {
    uint64_t v = 0;
    std::string why;
    if (ShardBase* s = owner_local(rank)) {
      if (s->parent_key(level, idx, &v) < 0) {
        why = last_error();
        v = NONE;
      }
    }
    KC_TRY(comm_->broadcast(rank, &v));
    if (v == NONE) {
      set_error("kc_group_run: trace walk failed on rank %d at level %d index %llu%s%s", rank, level,
                (unsigned long long)idx, why.empty() ? "" : ": ", why.c_str());
      return -EIO;
    }
    *key = v;
    return 0;
  }
  int buffer(std::vector<uint64_t*>& bufs, std::vector<uint64_t>& caps, size_t i, uint64_t bytes) {
    if (bytes <= caps[i]) return 0;
    KC_HIP_TRY(hipSetDevice(local_[i]->device()));
    KC_HIP_TRY(hipStreamSynchronize(local_[i]->stream()));
    if (bufs[i]) KC_HIP_TRY(hipFree(bufs[i]));
    bufs[i] = nullptr;
    const uint64_t nb = std::max<uint64_t>(bytes, 2 * caps[i]);
    KC_HIP_TRY(hipMalloc(&bufs[i], nb));
    caps[i] = nb;
    return 0;
  }
  // TLC order: the rank and local index of the state at position G of
  // `level` (every rank searches its sorted G values; one all-reduce)
  int tlc_locate(int level, uint64_t G, int* rank, uint64_t* idx) {
    std::vector<std::vector<uint64_t>> mine(local_.size(), std::vector<uint64_t>(1, 0));
    std::string why;
    for (size_t i = 0; i < local_.size(); ++i) {
      uint64_t k = 0;
      bool found = false;
      if (local_[i]->tlc_locate(level, G, &k, &found) < 0)
        why = last_error();
      else if (found)
        mine[i][0] = ((uint64_t)(local_[i]->rank() + 1) << 48) | k;
    }
    std::vector<uint64_t> tot;
    KC_TRY(comm_->all_reduce_sum(mine, tot));
    if (tot[0] == 0 || (tot[0] >> 48) > (uint64_t)world_) {
      set_error("kc_group_run: trace walk: no state at position %llu of level %d%s%s", (unsigned long long)G, level,
                why.empty() ? "" : ": ", why.c_str());
      return -EIO;
    }
    *rank = (int)(tot[0] >> 48) - 1;
    *idx = tot[0] & ((1ull << 48) - 1);
    return 0;
  }
  int error_trace(uint64_t err, int level, kc_result* res);
  int group_failed(int rank, uint64_t word, const std::vector<int>& fail, const std::string& msg);

  std::vector<ShardBase*> local_;
  std::unique_ptr<Comm> comm_;
  kc_model_config cfg_;
  int world_ = 1;
  std::vector<uint64_t*> send_, recv_;
  std::vector<uint64_t> send_cap_, recv_cap_;
  std::vector<std::vector<uint64_t>> trace_;
  std::vector<uint64_t> sent_local_;   // records each local shard sent to other ranks
  uint64_t sent_ = 0;                  // all ranks (after run)
  uint64_t sn_levels_ = 0;             // levels run narrow (this run)
  bool dev_row_off_ = false;
  uint64_t* h_fail_ = nullptr;         // pinned: failure words copied into device rows
  int fault_rank_ = -1, fault_level_ = 0, fault_stage_ = 0;
  bool sn_on_ = true;
  bool solo_off_ = false;
  bool serial_ = false;
  bool defer_on_ = true;
  bool tlc_ = false;                   // TLC order (cfg.tlc_order at world > 1)
  uint32_t sn_cap_ = SN_SLOT_DEFAULT;
  // KC_SERIAL: wait for local shard i's stream (errors surface at its next call)
  void ser(size_t i) {
    if (serial_) (void)hipStreamSynchronize(local_[i]->stream());
  }
};

// Failure handling: no rank may leave the loop alone, or its peers would
// wait in a collective for it forever (RCCL driven directly has no
// watchdog).  A rank that fails records the code and keeps taking part in
// the collectives; the failure travels in the all-gather row (word R + 2;
// claims that overflow set it on the device) and every rank stops at the
// next gather with an error.  A failure after the gather (the end of
// expand, growing the exchange buffers, pack, insert) sends zeroed records
// for the rest of the level — from the communicator's failure sink when the
// buffers could not be grown — so no peer waits in the all-to-all and none
// receives stale bytes; the error walk and the final reduction carry a
// failure flag the same way.
int Group::run(kc_result* res) {
  memset(res, 0, sizeof *res);
  res->err_action = res->err_self = res->err_invariant = -1;
  res->claim_mode = cfg_.first_claim ? 1 : (cfg_.tlc_order && world_ > 1) ? 2 : 0;
  trace_.clear();
  sent_ = 0;
  sn_levels_ = 0;
  sent_local_.assign(local_.size(), 0);
  const auto t0 = std::chrono::steady_clock::now();
  const size_t nl = local_.size();
  const int R = world_;
  const size_t L = (size_t)R + 3;            // row: owner counts | new states | error key | failure
  std::vector<int> fail(nl, 0);
  std::string fail_msg;
  auto note = [&](size_t i, int rc) {
    if (rc < 0 && !fail[i]) {
      fail[i] = rc;
      if (fail_msg.empty()) fail_msg = last_error();
    }
  };
  auto inject = [&](size_t i, int level, int stage) {
    if (local_[i]->rank() == fault_rank_ && level == fault_level_ && stage == fault_stage_ && !fail[i]) {
      set_error("kc_group_run: injected fault (KC_FAULT) on rank %d at level %d, stage %d", fault_rank_, level, stage);
      note(i, -EIO);
    }
  };
  auto fail_word = [&](size_t i) -> uint64_t { return fail[i] ? (1ull << 32) | (uint64_t)(uint32_t)(-fail[i]) : 0ull; };
  std::vector<uint64_t> status_new(nl), status_err(nl, NONE), e1(nl, NONE);
  for (size_t i = 0; i < nl; ++i) {
    note(i, hipSetDevice(local_[i]->device()) == hipSuccess ? 0 : -EIO);
    if (!fail[i]) note(i, local_[i]->init(&status_new[i]));
    // an Init state's invariant violation is level 1's error even when level
    // 1 is not expanded (max_levels = 1)
    if (!fail[i]) status_err[i] = local_[i]->init_error();
  }
  if (!h_fail_) KC_HIP_TRY(hipHostMalloc(&h_fail_, 16 * 8));
  std::vector<uint64_t> widths;
  int level = 1;
  uint64_t err = NONE;
  std::vector<std::vector<uint64_t>> counts(nl, std::vector<uint64_t>(R, 0)), rows(nl);
  std::vector<uint64_t> all;
  std::vector<std::vector<uint64_t>> Mx(R, std::vector<uint64_t>(R, 0));
  // narrow batches: run while they complete; after one stopped at a level
  // too wide (SN_STOP) the counted path takes over until the frontier
  // shrinks again.  Batches grow 8 -> 32 levels while they complete (a
  // batch's levels past the one that stopped it still exchange their slots).
  bool sn_blocked = false;
  int sn_batch = 8;
  uint64_t prev_total = ~0ull;
  std::vector<ShardBase::SNOut> so(nl);
  const bool solo = R == 1 && nl == 1 && comm_->trivial() && !solo_off_;
  for (;;) {
    const bool last = cfg_.max_levels && level >= cfg_.max_levels;
    if (sn_on_ && !last && !sn_blocked) {
      const uint64_t slot = local_[0]->sn_slot_bytes();
      // a deferred frontier is built first (the narrow kernels read states);
      // an invariant violation among its states is the level before's error
      for (size_t i = 0; i < nl; ++i) {
        uint64_t d = NONE;
        if (!fail[i]) note(i, local_[i]->materialize(&d));
        status_err[i] = std::min(status_err[i], d);
      }
      for (size_t i = 0; i < nl; ++i) {
        so[i] = ShardBase::SNOut{};
        if (!fail[i]) note(i, hipSetDevice(local_[i]->device()) == hipSuccess ? 0 : -EIO);
        // (a failed begin still leaves a control block that stops the batch)
        note(i, local_[i]->sn_begin(status_new[i], status_err[i], sn_batch));
      }
      std::vector<void*> ss(nl), rr(nl);
      for (size_t i = 0; i < nl; ++i) {
        ss[i] = local_[i]->sn_send();
        rr[i] = local_[i]->sn_recv();
      }
      for (int k = 0; k < sn_batch; ++k) {
        for (size_t i = 0; i < nl; ++i) {
          // a failed rank marks its control block (at every level: a failure
          // noted during the batch too): the level stops every rank
          bool f = fail[i] != 0;
          if (!fail[i] && local_[i]->rank() == fault_rank_ && level + k == fault_level_) {
            set_error("kc_group_run: injected fault (KC_FAULT) on rank %d at level %d, narrow", fault_rank_,
                      level + k);
            note(i, -EIO);
            f = true;
          }
          note(i, local_[i]->sn_pre((uint32_t)k, f));
          ser(i);
        }
        KC_TRY(comm_->sn_exchange(ss, rr, slot));
        for (size_t i = 0; i < nl; ++i) {
          note(i, local_[i]->sn_post((uint32_t)k));
          ser(i);
        }
      }
      const ShardBase::SNOut* g = nullptr;
      const ShardBase::SNOut* gf = nullptr;    // a shard's that failed in sn_end after filling it
      for (size_t i = 0; i < nl; ++i) {
        const bool pre = fail[i] != 0;
        note(i, local_[i]->sn_end(&so[i]));
        // fault injection: a failure found at the end of a batch that ran
        // level fault_level (KC_FAULT=rank:level:4)
        if (!pre && !fail[i] && local_[i]->rank() == fault_rank_ && fault_stage_ == 4 && so[i].levels > 0 &&
            fault_level_ >= level && fault_level_ < level + so[i].levels) {
          set_error("kc_group_run: injected fault (KC_FAULT) on rank %d at level %d, narrow batch end", fault_rank_,
                    fault_level_);
          note(i, -EIO);
        }
        if (!pre && fail[i] && so[i].filled && !gf) gf = &so[i];
        if (!pre && !fail[i]) {
          if (g && (g->levels != so[i].levels || g->reason != so[i].reason)) {
            set_error("kc_group_run: narrow levels disagree between ranks (%d vs %d)", g->levels, so[i].levels);
            return -EIO;
          }
          g = &so[i];
          sent_local_[i] += so[i].sent;
          status_new[i] = so[i].status_new;
          status_err[i] = so[i].status_err;
        }
      }
      // A process whose only shard failed at the end of the batch still
      // follows the batch its peers saw (sn_end filled the outcome before it
      // failed): if it ran to the end, every rank starts the next batch, whose
      // first level this rank's control block stops for all of them, and they
      // reach the counted path's gather (and its failure word) together.
      // Leaving for the gather alone would hang every peer in its next
      // narrow exchange.
      if (!g) g = gf;
      if (g) {
        for (uint64_t w : g->widths) {
          if ((int)widths.size() >= KC_MAX_LEVELS) {
            set_error("kc_group_run: more than %d levels", KC_MAX_LEVELS);
            return -ENOMEM;
          }
          widths.push_back(w);
        }
        level += g->levels;
        sn_levels_ += (uint64_t)g->levels;
        if (g->reason == SN_RUN) {
          sn_batch = std::min(2 * sn_batch, SN_BATCH);
          continue;                   // the next batch (which a failed rank's control block stops)
        }
        if (g->reason == SN_STOP) sn_blocked = true;
      }
      sn_batch = 8;
      // SN_STOP, SN_ERROR, SN_DONE or a failure: this level runs on the
      // counted path, whose all-gather reports the error, the end or the
      // failure as it always does
    }
    if (solo) {
      // One rank and nothing to gather or exchange: one host sync per level
      // (insert's).  Expand's flags, error key and timing are read after it
      // (its own pinned head, h_exp_); its error belongs to the next level's
      // status as on the gather path.  An Init violation is already this
      // level's status (init_error), so the level-1 shortcut is not needed.
      if (fail[0]) return group_failed(local_[0]->rank(), fail_word(0), fail, fail_msg);
      err = status_err[0];
      const uint64_t total = status_new[0];
      if (err != NONE || total == 0) {
        --level;
        break;
      }
      widths.push_back(total);
      if (sn_blocked && total * 4 <= (uint64_t)SN_MAX && total < prev_total) sn_blocked = false;
      prev_total = total;
      if (last) {
        // a deferred frontier's invariants (its states are built here)
        uint64_t d = NONE;
        note(0, local_[0]->materialize(&d));
        if (fail[0]) return group_failed(local_[0]->rank(), fail_word(0), fail, fail_msg);
        if (d != NONE) {
          widths.pop_back();
          err = d;
          --level;
        }
        break;
      }
      uint64_t n_new = 0, e2 = NONE, c0 = 0;
      e1[0] = NONE;
      inject(0, level, 0);
      if (!fail[0]) note(0, local_[0]->expand_dev(status_new[0], status_err[0], level == 1, nullptr));
      inject(0, level, 2);
      if (!fail[0]) note(0, local_[0]->insert(nullptr, 0, &n_new, &e2));
      if (!fail[0]) note(0, local_[0]->expand_done(&c0, &e1[0]));
      const uint64_t d = fail[0] ? NONE : local_[0]->defer_error();
      if (d != NONE) {
        // an invariant violation among this level's states, found as expand
        // rebuilt them: the level before's error (its emit would have found
        // it), so this level's width and the level insert just added go
        local_[0]->drop_last_insert();
        note(0, local_[0]->drop_last_expand());
        if (fail[0]) return group_failed(local_[0]->rank(), fail_word(0), fail, fail_msg);
        widths.pop_back();
        err = d;
        --level;
        break;
      }
      if (!fail[0]) note(0, local_[0]->advance());
      status_new[0] = fail[0] ? 0 : n_new;
      status_err[0] = fail[0] ? NONE : std::min(e1[0], e2);
      ++level;
      if ((int)widths.size() >= KC_MAX_LEVELS) {
        set_error("kc_group_run: more than %d levels", KC_MAX_LEVELS);
        return -ENOMEM;
      }
      continue;
    }
    // device rows (every local shard's kernels write its all-gather row, so
    // the gather's sync is the level's first: expand has none of its own)
    std::vector<uint64_t*> d_rows(nl, nullptr);
    bool dev = !last && !dev_row_off_;
    for (size_t i = 0; i < nl && dev; ++i) {
      d_rows[i] = comm_->row_buffer(i, L);
      dev = d_rows[i] != nullptr;
    }
    if (dev) {
      for (size_t i = 0; i < nl; ++i) {
        std::fill(counts[i].begin(), counts[i].end(), 0);
        e1[i] = NONE;
        if (!fail[i]) note(i, hipSetDevice(local_[i]->device()) == hipSuccess ? 0 : -EIO);
        inject(i, level, 0);
        if (!fail[i]) note(i, local_[i]->expand_dev(status_new[i], status_err[i], level == 1, d_rows[i]));
        ser(i);
        if (fail[i]) {          // the row says so, whatever else it holds
          h_fail_[i % 16] = fail_word(i);
          KC_HIP_TRY(hipMemcpyAsync(d_rows[i] + R + 2, &h_fail_[i % 16], 8, hipMemcpyHostToDevice,
                                    local_[i]->stream()));
        }
      }
      KC_TRY(comm_->all_gather_dev(L, all));
      for (size_t i = 0; i < nl; ++i) {
        if (fail[i]) continue;
        note(i, local_[i]->expand_done(counts[i].data(), &e1[i]));
        if (level == 1 && e1[i] != NONE && (e1[i] & 0xFF) == 0x12) {
          status_err[i] = e1[i];       // (k_owner_totals put it in the row already)
          e1[i] = NONE;
        }
      }
    } else {
      for (size_t i = 0; i < nl; ++i) {
        std::fill(counts[i].begin(), counts[i].end(), 0);
        e1[i] = NONE;
        if (!last) inject(i, level, 0);
        if (!last && !fail[i]) note(i, hipSetDevice(local_[i]->device()) == hipSuccess ? 0 : -EIO);
        if (!last && !fail[i]) {
          note(i, local_[i]->expand(counts[i].data(), &e1[i]));
          if (level == 1 && e1[i] != NONE && (e1[i] & 0xFF) == 0x12) {
            // an Init state violates an invariant: level 1's error, ahead of
            // any level-2 error (distributed.py does the same)
            status_err[i] = e1[i];
            e1[i] = NONE;
          }
        }
        // a deferred frontier's invariant key (expand rebuilt it; at the
        // max_levels stop it is built here)
        uint64_t d = NONE;
        if (last && !fail[i])
          note(i, local_[i]->materialize(&d));
        else if (!fail[i])
          d = local_[i]->defer_error();
        rows[i] = counts[i];
        rows[i].push_back(status_new[i]);
        rows[i].push_back(std::min(status_err[i], d));
        rows[i].push_back(fail_word(i));
      }
      KC_TRY(comm_->all_gather(rows, all));
    }
    for (int r = 0; r < R; ++r) {
      const uint64_t w = all[(size_t)r * L + R + 2];
      if (w) return group_failed(r, w, fail, fail_msg);
    }
    uint64_t total = 0;
    err = NONE;
    for (int r = 0; r < R; ++r) {
      const uint64_t* row = all.data() + (size_t)r * L;
      for (int d = 0; d < R; ++d) Mx[r][d] = row[d];
      total += row[R];
      err = std::min(err, row[R + 1]);
    }
    if (err != NONE || total == 0) {
      --level;
      break;
    }
    widths.push_back(total);
    // back to the narrow levels once the frontier shrinks well below their limit
    if (sn_blocked && total * 4 <= (uint64_t)R * SN_MAX && total < prev_total) sn_blocked = false;
    prev_total = total;
    if (last) break;
    std::vector<char> sunk(nl, 0);
    for (size_t i = 0; i < nl; ++i) {
      const int me = local_[i]->rank();
      uint64_t ns = 0, nr = 0;
      for (int d = 0; d < R; ++d) {
        ns += Mx[me][d];
        nr += Mx[d][me];
      }
      sent_local_[i] += ns - Mx[me][me];
      const uint64_t rb = local_[i]->record_bytes();
      // a rank that failed here (expand_done above, or growing its buffers)
      // still takes part in the exchange: zeroed records, through the sink
      // if it has no buffers of the size
      if (!fail[i]) note(i, buffer(send_, send_cap_, i, std::max<uint64_t>(ns, 1) * rb));
      if (!fail[i]) note(i, buffer(recv_, recv_cap_, i, std::max<uint64_t>(nr, 1) * rb));
      const bool grow_fault = !fail[i] && local_[i]->rank() == fault_rank_ && level == fault_level_ && fault_stage_ == 3;
      inject(i, level, 3);
      if (fail[i] && (grow_fault || send_cap_[i] < std::max<uint64_t>(ns, 1) * rb ||
                      recv_cap_[i] < std::max<uint64_t>(nr, 1) * rb))
        sunk[i] = 1;
      if (!fail[i]) note(i, hipSetDevice(local_[i]->device()) == hipSuccess ? 0 : -EIO);
      bool packed = false;
      if (!fail[i]) {
        note(i, local_[i]->pack(send_[i]));
        packed = !fail[i];
      }
      if (!packed && !sunk[i] && ns) note(i, hipMemsetAsync(send_[i], 0, ns * rb, local_[i]->stream()) == hipSuccess ? 0 : -EIO);
      ser(i);
      inject(i, level, 1);      // (a failure found after a complete pack)
    }
    std::vector<void*> sv(send_.begin(), send_.end()), rv(recv_.begin(), recv_.end());
    KC_TRY(comm_->all_to_all(sv, Mx, local_[0]->record_bytes(), rv, sunk));
    for (size_t i = 0; i < nl; ++i) {
      const int me = local_[i]->rank();
      uint64_t nr = 0;
      for (int s = 0; s < R; ++s) nr += Mx[s][me];
      uint64_t n_new = 0, e2 = NONE;
      if (!fail[i]) note(i, hipSetDevice(local_[i]->device()) == hipSuccess ? 0 : -EIO);
      inject(i, level, 2);
      if (!fail[i]) note(i, local_[i]->insert(recv_[i], nr, &n_new, &e2));
      status_new[i] = fail[i] ? 0 : n_new;
      status_err[i] = fail[i] ? NONE : std::min(e1[i], e2);
    }
    if (tlc_) {
      // the new states' G: per-parent winner masks summed over the ranks
      // (a failed rank adds zeroes and fails at the next gather)
      if (total >= (1ull << 31)) {
        set_error("kc_group_run: tlc_order: a level of %llu states (2^31 at most)", (unsigned long long)total);
        return -ENOMEM;
      }
      std::vector<uint32_t*> masks(nl, nullptr);
      for (size_t i = 0; i < nl; ++i)
        if (!fail[i]) note(i, local_[i]->tlc_masks(total, &masks[i]));
      KC_TRY(comm_->all_reduce_dev_u32(masks, total));
      for (size_t i = 0; i < nl; ++i) {
        if (!fail[i]) note(i, local_[i]->tlc_order(total));
        if (fail[i]) status_new[i] = 0;
      }
    }
    for (size_t i = 0; i < nl; ++i)
      if (!fail[i]) note(i, local_[i]->advance());
    ++level;
    if ((int)widths.size() >= KC_MAX_LEVELS) {
      set_error("kc_group_run: more than %d levels", KC_MAX_LEVELS);
      return -ENOMEM;
    }
  }
  // global totals (the same on every rank), with a failure count
  std::vector<std::vector<uint64_t>> mine(nl);
  for (size_t i = 0; i < nl; ++i) {
    kc_result r;
    memset(&r, 0, sizeof r);
    if (!fail[i]) note(i, local_[i]->result(&r));
    for (int a = 0; a < KC_NACTIONS; ++a) mine[i].push_back(r.act_gen[a]);
    for (int a = 0; a < KC_NACTIONS; ++a) mine[i].push_back(r.act_dist[a]);
    mine[i].push_back(r.init);
    mine[i].push_back(r.generated);
    mine[i].push_back(r.distinct);
    mine[i].push_back(sent_local_[i]);
    mine[i].push_back(fail[i] ? 1 : 0);
    // seen-set spill (summed over the ranks)
    for (uint64_t v : {r.seen_flushes, r.seen_cold_fps, r.seen_cold_runs, r.seen_cold_queries, r.seen_cold_hits,
                       r.seen_merges, r.seen_disk_bytes})
      mine[i].push_back(v);
  }
  std::vector<uint64_t> tot;
  KC_TRY(comm_->all_reduce_sum(mine, tot));
  if (tot[2 * KC_NACTIONS + 4]) return group_failed(-1, 0, fail, fail_msg);
  {
    const uint64_t* sp = tot.data() + 2 * KC_NACTIONS + 5;
    res->seen_flushes = sp[0];
    res->seen_cold_fps = sp[1];
    res->seen_cold_runs = sp[2];
    res->seen_cold_queries = sp[3];
    res->seen_cold_hits = sp[4];
    res->seen_merges = sp[5];
    res->seen_disk_bytes = sp[6];
  }
  for (int a = 0; a < KC_NACTIONS; ++a) {
    res->act_gen[a] = tot[a];
    res->act_dist[a] = tot[KC_NACTIONS + a];
  }
  res->init = tot[2 * KC_NACTIONS];
  res->generated = tot[2 * KC_NACTIONS] + tot[2 * KC_NACTIONS + 1];
  res->distinct = tot[2 * KC_NACTIONS + 2];
  sent_ = tot[2 * KC_NACTIONS + 3];
  res->nlevels = (int)widths.size();
  res->depth = res->nlevels;
  res->narrow_levels = sn_levels_;
  for (size_t k = 0; k < widths.size(); ++k) res->level_width[k] = widths[k];
  res->complete = err == NONE && !(cfg_.max_levels && level >= cfg_.max_levels);
  if (err != NONE) KC_TRY(error_trace(err, level, res));
  const double d = (double)res->distinct, g = (double)res->generated;
  res->collision_optimistic = d * (g - d) / 18446744073709551616.0;
  res->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return 0;
}

// Every rank leaves with an error: its own message where one of its shards
// failed, otherwise the failing rank and what its failure word says.
int Group::group_failed(int rank, uint64_t word, const std::vector<int>& fail, const std::string& msg) {
  for (size_t i = 0; i < fail.size(); ++i) {
    if (fail[i]) {
      set_error("%s", msg.c_str());
      return fail[i];
    }
  }
  if (rank < 0) {
    set_error("kc_group_run: a peer rank failed");
    return -EIO;
  }
  if (word >> 32) {
    set_error("kc_group_run: rank %d failed (errno %d)", rank, (int)(word & 0xffffffffu));
    return -(int)(word & 0xffffffffu);
  }
  set_error("kc_group_run: rank %d: successor overflow or full table", rank);
  return -ENOMEM;
}

// Walk the parent keys back across ranks (TLC's trace file), then replay
// the path on the host: the same protocol as distributed.py's _error.
int Group::error_trace(uint64_t err, int level, kc_result* res) {
  const int kind = (int)(err & 0xFF);
  const int pos = (int)((err >> 8) & 0xFF);
  std::vector<int> path;
  int r = (int)(err >> 60), lvl = level;
  uint64_t idx = (err >> 16) & KEY44;
  if (kind == 0x12) {          // an Init state: its index in TLC's order is in the key
    int act = -1, self = -1, inv = -1;
    KC_TRY(local_[0]->replay((int)idx, path, kind, pos, trace_, &act, &self, &inv));
    res->err_kind = E_INVARIANT;
    res->err_invariant = inv;
    res->err_level = 1;
    res->trace_len = (int)trace_.size();
    return 0;
  }
  // (TLC order: keys carry G, located by a search on every rank)
  if (tlc_) KC_TRY(tlc_locate(lvl, idx, &r, &idx));
  while (lvl > 1) {
    uint64_t key = 0;
    KC_TRY(query_parent(r, lvl, idx, &key));
    path.push_back((int)((key >> 8) & 0xFF));
    r = (int)(key >> 60);
    idx = (key >> 16) & KEY44;
    --lvl;
    if (tlc_) KC_TRY(tlc_locate(lvl, idx, &r, &idx));
  }
  uint64_t init_key = 0;
  KC_TRY(query_parent(r, 1, idx, &init_key));
  std::reverse(path.begin(), path.end());
  int act = -1, self = -1, inv = -1;
  KC_TRY(local_[0]->replay((int)(init_key & 0xFFFF), path, kind, pos, trace_, &act, &self, &inv));
  res->err_kind = kind == 0x12 ? E_INVARIANT : kind;
  res->err_action = act;
  res->err_self = self;
  res->err_invariant = inv;
  res->err_level = kind == E_INVARIANT ? level + 1 : (kind == 0x12 ? 1 : level);
  res->trace_len = (int)trace_.size();
  return 0;
}

}  // namespace kc

using namespace kc;

struct kc_group {
  std::unique_ptr<Group> impl;
};

extern "C" {

int kc_rccl_unique_id(uint8_t* id_out) {
  if (!id_out) { set_error("kc_rccl_unique_id: NULL"); return -EINVAL; }
  const RcclApi* api = rccl();
  if (!api) { set_error("kc_rccl_unique_id: RCCL (librccl.so.1) not loadable"); return -ENODEV; }
  ncclUniqueId id;
  KC_NCCL_TRY(api->get_unique_id(&id));
  static_assert(sizeof(ncclUniqueId) == KC_RCCL_ID_BYTES, "ncclUniqueId size");
  memcpy(id_out, &id, sizeof id);
  return 0;
}

int kc_group_create_rccl(kc_shard* s, const uint8_t* id, kc_group** out) {
  if (!s || !id || !out) { set_error("kc_group_create_rccl: NULL"); return -EINVAL; }
  *out = nullptr;
  const RcclApi* api = rccl();
  if (!api) { set_error("kc_group_create_rccl: RCCL (librccl.so.1) not loadable"); return -ENODEV; }
  ShardBase* sh = s->impl.get();
  KC_HIP_TRY(hipSetDevice(sh->device()));
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof uid);
  ncclComm_t comm = nullptr;
  KC_NCCL_TRY(api->comm_init_rank(&comm, sh->world(), uid, sh->rank()));
  std::unique_ptr<RcclComm> rc(new RcclComm(sh, comm));
  KC_TRY(rc->make_sink());
  std::unique_ptr<Group> g(new Group({sh}, std::move(rc), sh->config()));
  KC_TRY(g->setup());
  *out = new kc_group{std::move(g)};
  return 0;
}

int kc_group_create_host(kc_shard* s, const kc_host_comm* comm, kc_group** out) {
  if (!s || !comm || !out) { set_error("kc_group_create_host: NULL"); return -EINVAL; }
  *out = nullptr;
  if (!comm->all_gather || !comm->exchange || !comm->broadcast || !comm->all_reduce_sum) {
    set_error("kc_group_create_host: every kc_host_comm callback is required");
    return -EINVAL;
  }
  ShardBase* sh = s->impl.get();
  KC_HIP_TRY(hipSetDevice(sh->device()));
  std::unique_ptr<Group> g(new Group({sh}, std::unique_ptr<Comm>(new HostComm(sh, *comm)), sh->config()));
  KC_TRY(g->setup());
  *out = new kc_group{std::move(g)};
  return 0;
}

int kc_group_create_local(kc_shard** shards, int nshards, kc_group** out) {
  if (!shards || nshards < 1 || !out) { set_error("kc_group_create_local: bad argument"); return -EINVAL; }
  *out = nullptr;
  std::vector<ShardBase*> v;
  for (int i = 0; i < nshards; ++i) {
    if (!shards[i]) { set_error("kc_group_create_local: NULL shard"); return -EINVAL; }
    ShardBase* sh = shards[i]->impl.get();
    if (sh->world() != nshards || sh->rank() != i || sh->device() != shards[0]->impl->device()) {
      set_error("kc_group_create_local: shard %d must be rank %d of %d on one device", i, i, nshards);
      return -EINVAL;
    }
    v.push_back(sh);
  }
  std::unique_ptr<Group> g(new Group(v, std::unique_ptr<Comm>(new LocalComm(v)), v[0]->config()));
  KC_TRY(g->setup());
  *out = new kc_group{std::move(g)};
  return 0;
}

void kc_group_destroy(kc_group* g) { delete g; }

int kc_group_run(kc_group* g, kc_result* res) {
  if (!g || !res) { set_error("kc_group_run: NULL"); return -EINVAL; }
  return g->impl->run(res);
}

int kc_group_trace_tuple(kc_group* g, int i, uint64_t* out) {
  if (!g || !out) { set_error("kc_group_trace_tuple: NULL"); return -EINVAL; }
  const auto& t = g->impl->trace();
  if (i < 0 || i >= (int)t.size()) { set_error("kc_group_trace_tuple: index"); return -EINVAL; }
  std::copy(t[i].begin(), t[i].end(), out);
  return (int)t[i].size();
}

uint64_t kc_group_records_sent(const kc_group* g) { return g ? g->impl->records_sent() : 0; }

int kc_exchange_plan(int world, int me, const uint64_t* Mx, uint64_t piece_records, uint64_t* out, int cap) {
  if (world < 1 || me < 0 || me >= world || !Mx || cap < 0 || (cap > 0 && !out)) {
    set_error("kc_exchange_plan: bad argument");
    return -EINVAL;
  }
  std::vector<std::vector<uint64_t>> M(world, std::vector<uint64_t>(world));
  for (int s = 0; s < world; ++s)
    for (int d = 0; d < world; ++d) M[s][d] = Mx[(size_t)s * world + d];
  const std::vector<Xfer> plan = exchange_plan(M, me, piece_records);
  for (size_t k = 0; k < plan.size() && (int)k < cap; ++k) {
    out[4 * k] = (uint64_t)plan[k].peer;
    out[4 * k + 1] = (uint64_t)plan[k].send;
    out[4 * k + 2] = plan[k].off;
    out[4 * k + 3] = plan[k].n;
  }
  return (int)plan.size();
}

}  // extern "C"
