// engine.hip — single-GPU level-synchronous BFS model checker for KubeAPI.tla
// (replaces TLC's BFS ModelChecker + workers, FPSet and StateQueue for this
// spec; MC.out:5).  Host loop + C-ABI kc_engine_*.
//
// Per level (all on one HIP stream, one host sync per level):
//   for each chunk of <= chunk_states parents:
//     k_claim (LDS tile dedup + ClaimSet claims); k_settle_rec<0>, <1> (winners);
//     hipcub exclusive scan; k_emit; k_advance
//   read {next width, next candidates, error key} back.
// The frontier buffers are the StateQueue: double-buffered packed states
// in HBM, FIFO order = (parent order, TLC successor order), identical to a
// sequential TLC -workers 1 BFS.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <memory>
#include <string>
#include <vector>

#include "../../include/kubecheck.h"
#include "coldset.h"
#include "engine.h"
#include "engine_kernels.h"
#include "engine_narrow.h"
#include "engine_spill.h"
#include "engine_util.h"
#include "fpset_host.h"
#include "kc_common.h"
#include "squeue.h"

namespace kc {

namespace {

const char* kActionNames[A_COUNT] = {
    "DoRequest", "DoReply", "DoListRequest", "DoListReply", "CStart", "C1", "C10", "C11",
    "c12", "C13", "C2", "C3", "C8", "C6", "C7", "C4", "C5", "PVCStart", "PVCListedPVCs",
    "PVCHavePVCs", "PVCDone", "APIStart"};

}  // namespace

// chunk_base += the chunk's new states (last exclusive offset + last count,
// or the tile scan's total tile_off[tiles]); cand_total = sum of the
// next_cand stripes (one 64-lane wave, one stripe per lane).  host != nullptr
// (the level's last chunk): the level's head goes straight into pinned host
// memory and the device head is reset for the next level (no copy launch,
// no separate reset launch).
// (K_ADVANCE_THREADS lanes: the 64-KiB snapshot copy is 16 loads per lane,
// all in flight at once; round 5's 64 lanes ran it as 8 dependent batches)
constexpr int K_ADVANCE_THREADS = 256;
__global__ void __launch_bounds__(K_ADVANCE_THREADS)
k_advance(const uint32_t* __restrict__ offsets, const uint32_t* __restrict__ newmask, uint64_t n,
          Counters* __restrict__ C, const uint32_t* __restrict__ tile_off, uint64_t tiles,
          unsigned long long* __restrict__ host, unsigned long long* __restrict__ ovf_count = nullptr,
          CtrStripe* __restrict__ snap = nullptr) {
  static_assert(CTR_STRIPES == 64, "one lane per stripe");
  constexpr int UNITS = (int)(CTR_STRIPES * sizeof(CtrStripe) / 16), PER = UNITS / K_ADVANCE_THREADS;
  static_assert(UNITS % K_ADVANCE_THREADS == 0, "whole 16-B units per lane");
  if (ovf_count && threadIdx.x == 0) *ovf_count = 0;   // the next chunk's candidate overflow list starts empty
  // the level's last chunk: the counters as the level leaves them, kept for
  // a deferred-frontier redo from the next level
  if (snap) {
    const ulonglong2* src = reinterpret_cast<const ulonglong2*>(C->s);
    ulonglong2* dst = reinterpret_cast<ulonglong2*>(snap);
    ulonglong2 v[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) v[k] = src[k * K_ADVANCE_THREADS + threadIdx.x];
#pragma unroll
    for (int k = 0; k < PER; ++k) dst[k * K_ADVANCE_THREADS + threadIdx.x] = v[k];
  }
  if (threadIdx.x >= 64) return;
  unsigned long long v = C->s[threadIdx.x].next_cand;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  if (threadIdx.x == 0) {
    C->cand_total = v;
    if (tile_off)
      C->chunk_base += tile_off[tiles];
    else if (n > 0)
      C->chunk_base += (unsigned long long)offsets[n - 1] + NewCount()(newmask[n - 1]);
    if (host) {
      host[0] = C->err_key;
      host[1] = C->chunk_base;
      host[2] = C->overflow;
      host[3] = C->batch_used;
      host[4] = C->cand_total;
      host[5] = C->level_new;
      host[7] = C->defer_flags;
      host[8] = C->defer_inv_n;        // (Counters::defer_inv_n of the pinned copy)
      C->err_key = ~0ull;
      C->chunk_base = 0;
      C->overflow = 0;
      C->batch_used = 0;
      C->defer_flags = 0;
      C->defer_inv_n = 0;
    }
  }
}

// Per-level counter head reset (err_key = ~0; chunk_base, overflow,
// batch_used = 0), enqueued behind the previous level's head read-back so
// it runs while the host waits, not after it.
__global__ void k_level_reset(Counters* __restrict__ C) {
  if (threadIdx.x == 0) {
    C->err_key = ~0ull;
    C->chunk_base = 0;
    C->overflow = 0;
    C->batch_used = 0;
    C->defer_flags = 0;
    C->defer_inv_n = 0;
  }
}

const char* action_name(int a) { return (a >= 0 && a < A_COUNT) ? kActionNames[a] : "?"; }

// Deferred-frontier redo from level X: every fingerprint claimed at a
// successor level above X (inserted by level X or later) leaves the
// ClaimSet.  Linear probing never moves an entry, so with no rehash since
// level X began the table is then exactly what level X found.
__global__ void k_claimset_drop(ClaimEntry* __restrict__ t, uint64_t nslots, uint32_t level) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nslots; i += (uint64_t)gridDim.x * blockDim.x) {
    const ulonglong2 e = *reinterpret_cast<const ulonglong2*>(t + i);
    if (e.x && ((~e.y) >> CLAIM_KEY_BITS) >= level)
      *reinterpret_cast<ulonglong2*>(t + i) = make_ulonglong2(0ull, 0ull);
  }
}

// The counters as a redo from level X needs them: every stripe as level
// X - 1 left it (prev), except the per-action distinct counts, taken from
// level X's snapshot (cur): on the deferred frontier a level's own states
// are counted when its k_claim rebuilds them, which the exact path (it
// counts them in the previous level's emit) will not do again.
__global__ void __launch_bounds__(64)
k_counters_restore(Counters* __restrict__ C, const CtrStripe* __restrict__ prev, const CtrStripe* __restrict__ cur) {
  CtrStripe& d = C->s[threadIdx.x];
  d = prev[threadIdx.x];
#pragma unroll
  for (int a = 0; a < A_COUNT; ++a) d.act_dist[a] = cur[threadIdx.x].act_dist[a];
}

// fingerprints of a ClaimSet into a dense array (order irrelevant: sorted next)
// (csh: slot i's fp word is word i << csh, DevClaimSet::word_shift)
__global__ void k_claimset_fps(const unsigned long long* __restrict__ w, uint64_t nslots, uint32_t csh,
                               unsigned long long* __restrict__ out, uint64_t cap,
                               unsigned long long* __restrict__ n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nslots; i += (uint64_t)gridDim.x * blockDim.x) {
    const unsigned long long fp = w[i << csh];
    if (fp) {
      const unsigned long long k = atomicAdd(n, 1ull);
      if (k < cap) out[k] = fp;
    }
  }
}
__global__ void k_adjacent_min_gap(const unsigned long long* __restrict__ s, uint64_t n,
                                   unsigned long long* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i + 1 < n) atomicMin(out, s[i + 1] - s[i]);
}

constexpr uint64_t kMaxChunk = (1ull << 27) - 256;

template <class M>
class EngineT final : public EngineBase {
  using State = typename M::State;

 public:
  explicit EngineT(const kc_model_config& cfg) : EngineBase(cfg) {
    flags_ = flags_of(cfg);
    timing_ = cfg.timing == 2 ? 2 : (cfg.timing != 0 ? 1 : 0);
    const char* ab = getenv("KC_ABLATE");
    ablate_ = ab && ab[0] == '1';
    if (ablate_) timing_ = 1;
    // the narrow-level kernel: on by default; off when the caller asks for
    // explicit chunks (the chunked wide path is what they exercise) or with
    // KC_NARROW=0
    const char* nw = getenv("KC_NARROW");
    narrow_on_ = cfg.chunk_states == 0 && !(nw && nw[0] == '0') && !ablate_;
    // frontiers in the StateQueue (spill mode): the chunked wide path only
    queued_ = cfg.frontier_hbm_bytes > 0;
    if (queued_) narrow_on_ = false;
    // seen-set spill: a fixed-size hot ClaimSet + the cold tier (coldset.h);
    // the chunked wide path with tile offsets only
    spill_ = cfg.seen_hbm_bytes > 0;
    if (spill_) narrow_on_ = false;
    const char* ts = getenv("KC_TSCAN");
    tscan_ = spill_ || !(ts && ts[0] == '0');
    const char* nb = getenv("KC_NARROW_BATCH");   // narrow levels enqueued per host sync (A/B)
    if (nb && atoi(nb) > 0) narrow_batch_ = atoi(nb);
    const char* tr = getenv("KC_TSCAN_REG");
    tscan_reg_ = !(tr && tr[0] == '0');
    const char* hc = getenv("KC_HEADCOPY");
    headcopy_ = hc && hc[0] == '1';
    // deferred frontier (engine_kernels.h DeferArgs): the default wide path
    // (KC_DEFER=0: every level's k_emit builds and stores its new states)
    const char* df = getenv("KC_DEFER");
    defer_ = !(df && df[0] == '0') && !spill_ && !queued_ && !ablate_;
    // KC_DEFER_SLACK: the capacity estimate's factor over the measured
    // successors per state (tests shrink it to force the exact-path redo)
    const char* dr = getenv("KC_DEFER_REDO");      // KC_DEFER_REDO=0: an anomaly redoes the run from Init
    redo_on_ = !(dr && dr[0] == '0');
    const char* dd = getenv("KC_DEFER_DIRECT");    // KC_DEFER_DIRECT=0: invariant anomalies are redone too (A/B)
    defer_direct_ = !(dd && dd[0] == '0');
    const char* ds = getenv("KC_DEFER_SLACK");
    if (ds && atof(ds) > 0) defer_slack_ = atof(ds);
    if (defer_) tscan_ = true;    // the link emit takes the tile offsets
    // KC_FIRST_CLAIM=1: first-claim mode (k_claim FIRST) on the in-HBM wide
    // path: the first inserter of a fingerprint wins, no settle passes (decided
    // after the tile scan is, which it needs; kc_result.claim_mode reports it)
    const char* fc = getenv("KC_FIRST_CLAIM");
    first_claim_ = (cfg.first_claim || (fc && fc[0] == '1')) && tscan_ && !spill_ && !queued_;
    // (first-claim mode writes no claim words, so no level's inserts can be
    // dropped: a deferred-frontier capacity anomaly redoes the run from Init;
    // an Assert or deadlock key is reported directly, as on the exact path)
    if (first_claim_) redo_on_ = false;
    // its ClaimSet holds fp words only (8-B slots: half the table to clear);
    // KC_CLAIM_COMPACT=0 keeps 16-B slots (A/B)
    const char* cc = getenv("KC_CLAIM_COMPACT");
    cs_.compact = first_claim_ && !(cc && cc[0] == '0');
    const char* ck = getenv("KC_CHUNK_SCAN");
    chunk_scan_ = !(ck && ck[0] == '0');
  }
  ~EngineT() override { release(); }

  int state_words() const override { return M::W; }
  int tuple_words() const override { return M::TUPLE_WORDS; }

  int setup() override {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
      set_error("kubecheck: no HIP device visible (the engine has no CPU fallback)");
      return -ENODEV;
    }
    if (cfg_.device < 0 || cfg_.device >= ndev) {
      set_error("kubecheck: bad device %d", cfg_.device);
      return -EINVAL;
    }
    KC_HIP_TRY(hipSetDevice(cfg_.device));
    KC_HIP_TRY(hipStreamCreateWithFlags(&st_, hipStreamNonBlocking));
    KC_HIP_TRY(hipMalloc(&d_ctr_, sizeof(Counters)));
    KC_HIP_TRY(hipHostMalloc(&h_ctr_, sizeof(Counters)));
    KC_HIP_TRY(hipMalloc(&d_ns_, sizeof(NarrowCtl)));
    KC_HIP_TRY(hipHostMalloc(&h_ns_, sizeof(NarrowCtl)));
    if (narrow_on_) {
      KC_HIP_TRY(hipMalloc(&d_nsc_, sizeof(NarrowScratch)));
    }
    return 0;
  }

  // A deferred level that meets anything but a clean level (an error of any
  // kind, a capacity estimate too small) is redone on the exact,
  // materialising path from the level the anomaly belongs to (redo_from:
  // the ClaimSet, the counters and the host state are put back as that
  // level found them), so error reports and every count come from the path
  // that checks each new state where it is emitted.  When that cannot be
  // done exactly (a rehash since, KC_DEFER_REDO=0) the whole run is redone
  // from Init on the exact path.
  int run(kc_result* res) override {
    defer_now_ = defer_;
    int rc = run_once(res);
    if (rc == kDeferRetry) {
      ++defer_fallbacks_;
      defer_now_ = false;
      rc = run_once(res);
      res->defer_fallback = 1;
      res->defer_redo_level = 1;
    }
    return rc;
  }

  int run_once(kc_result* res) {
    KC_HIP_TRY(hipSetDevice(cfg_.device));
    memset(res, 0, sizeof *res);
    res->err_action = res->err_self = res->err_invariant = -1;
    res->claim_mode = first_claim_ ? 1 : 0;
    trace_.clear();
    narrow_probes_ = 0;
    for (auto& t : ktime_ms_) t = 0;
    ev_kind_.clear();
    ev_used_ = 0;
    for (auto& c : klaunch_) c = 0;
    narrow_levels_ = 0;
    exact_until_ = 0;
    for (auto& v : snap_lv_) v = -1;
    for (auto& h : hs_) h.level = -1;
    for (auto& v : succ_lv_) v = -1;
    const auto t0 = std::chrono::steady_clock::now();

    // ---- Init (KubeAPI.tla:455-469), on the host: 2^NC states
    const int ni = M::num_init();
    std::vector<State> init(ni);
    std::vector<uint64_t> fps(ni);
    uint64_t cand = 0;
    for (int k = 0; k < ni; ++k) {
      M::init_state(k, init[k], cfg_.variant);
      fps[k] = M::fingerprint(init[k]);
      cand += (uint64_t)M::plan(init[k], flags_).total;
    }
    // the seen-set allocation is kept across runs (cleared each run), like a
    // TLC FPSet pre-sized with -fpmem; it grows by rehash when needed
    const uint64_t fp_slots = cfg_.fpset_slots ? cfg_.fpset_slots : (1ull << 20);
    if (spill_) {
      KC_TRY(spill_setup());
    } else if (cs_.t && cs_.capacity() >= fp_slots) {
      KC_TRY(cs_.clear(st_));
    } else {
      KC_TRY(cs_.init(fp_slots, st_));
    }
    KC_TRY(grow_buffer(cur_, cur_cap_, (uint64_t)ni, false, st_));
    KC_TRY(grow_trace((uint64_t)ni + cand, false));
    KC_HIP_TRY(hipMemcpyAsync(cur_, init.data(), ni * sizeof(State), hipMemcpyHostToDevice, st_));
    // (the Init fingerprints' device buffers are kept across runs: a
    // hipMalloc / hipFree pair per run cost a device-wide sync)
    KC_TRY(grow_buffer(init_fps_, init_fps_cap_, (uint64_t)ni, false, st_));
    KC_TRY(grow_buffer(init_res_, init_res_cap_, (uint64_t)ni, false, st_));
    uint64_t* const d_fps = init_fps_;
    int* const d_res = init_res_;
    KC_HIP_TRY(hipMemcpyAsync(d_fps, fps.data(), ni * 8, hipMemcpyHostToDevice, st_));
    launch_claimset_insert_list(d_fps, (uint64_t)ni, cs_, 1u, d_res, st_);
    std::vector<int> ires(ni);
    KC_HIP_TRY(hipMemcpyAsync(ires.data(), d_res, ni * sizeof(int), hipMemcpyDeviceToHost, st_));
    std::vector<unsigned long long> ipar(ni, ~0ull);
    std::vector<uint8_t> iord(ni);
    for (int k = 0; k < ni; ++k) iord[k] = (uint8_t)k;
    if (cfg_.trace_host) {
      KC_HIP_TRY(hipStreamSynchronize(st_));
      memcpy(parent_, ipar.data(), ni * 8);
      memcpy(ord_, iord.data(), ni);
    } else {
      KC_HIP_TRY(hipMemcpyAsync(parent_, ipar.data(), ni * 8, hipMemcpyHostToDevice, st_));
      KC_HIP_TRY(hipMemcpyAsync(ord_, iord.data(), ni, hipMemcpyHostToDevice, st_));
    }
    KC_HIP_TRY(hipStreamSynchronize(st_));
    for (int k = 0; k < ni; ++k) {
      if (ires[k] != CL_NEW) {
        set_error("kubecheck: init states not distinct");
        return -EIO;
      }
    }
    cs_.count = ni;
    hot_count_ = ni;
    KC_HIP_TRY(hipMemsetAsync(d_ctr_, 0, sizeof(Counters), st_));
    if (d_ovf_cnt_) KC_HIP_TRY(hipMemsetAsync(d_ovf_cnt_, 0, 8, st_));
    if (defer_now_) KC_TRY(counter_snap(0));
    res->init = ni;
    res->generated = ni;
    res->distinct = ni;
    init_states_ = init;

    uint64_t n = ni, level_gidx = 0, cand_total = 0;
    int level = 1;
    res->level_width[0] = n;
    res->nlevels = 1;
    // invariants of the initial states
    for (int k = 0; k < ni; ++k) {
      const int inv = M::check(init[k], flags_.inv_mask);
      if (inv >= 0) {
        res->err_kind = E_INVARIANT;
        res->err_invariant = inv;
        res->err_level = 1;
        trace_.push_back(init[k]);
        res->trace_len = 1;
        finish(res, t0, n);
        return 0;
      }
    }

    if (queued_) return run_queued(res, t0, n, cand, init);

    // default: one chunk per level; chunk_states bounds the per-chunk
    // buffers.  Claims are level-global (keys grow with the parent index),
    // so a chunk's winners are final once its own claim pass is done.
    // per-level counter fields: err_key = ~0, the rest 0 (act_* are cumulative)
    hipLaunchKernelGGL(k_level_reset, dim3(1), dim3(64), 0, st_, d_ctr_);
    // <= 2^27 parents per chunk: the chunk's scan runs on int counts and its
    // offsets are u32 (at most 32 new states per parent: < 2^32 per chunk)
    const uint64_t chunk =
        (std::min<uint64_t>(cfg_.chunk_states ? cfg_.chunk_states : kMaxChunk, kMaxChunk) + 255) / 256 * 256;
    // Deferred frontier (defer_now_): `mat` = cur_ holds this level's states.
    // Otherwise the level's k_claim rebuilds them from the previous frontier
    // (next_, which starts at global index prev_gidx) and the links the
    // previous level's emit wrote; `cand` is then unknown and the level's
    // buffers are sized from `ratio`, the last measured successors per state.
    bool mat = true;
    uint64_t prev_gidx = 0;
    double ratio = n ? (double)cand / (double)n : 1.0;
    pc_valid_ = false;                 // pc_prev_ holds the previous frontier's plans
    while (n > 0) {
      if (cfg_.max_levels && level >= cfg_.max_levels) break;
      if (narrow_on_ && n <= (uint64_t)NARROW_MAX &&
          (mat || (double)n * ratio <= 1.25 * (double)NARROW_CAND_MAX)) {
        // ---- narrow levels: one single-workgroup launch runs as many
        // levels as fit (engine_narrow.h); the host takes over at the first
        // level it cannot run.  It needs the states and their exact
        // successor count: a deferred frontier is materialised first.
        if (!mat) {
          KC_TRY(materialize(n, level_gidx, prev_gidx, cand, cand_total));
          mat = true;
          KC_TRY(counter_snap(level - 1));     // (k_materialize counted the states' actions)
        }
        pc_valid_ = false;
        int stop = cfg_.max_levels;
        if (capture_level_ >= level + 1 && (stop == 0 || capture_level_ - 1 < stop)) stop = capture_level_ - 1;
        NarrowRun nr;
        KC_TRY(run_narrow(n, level, level_gidx, cand, stop, nr));
        res->distinct += nr.new_total;
        for (int L = level; L < nr.level; ++L) {
          if (L >= KC_MAX_LEVELS) {
            set_error("kubecheck: more than %d levels", KC_MAX_LEVELS);
            return -ENOMEM;
          }
          res->level_width[L] = h_ns_->widths[L];
        }
        if (nr.levels) res->peak_frontier = std::max<uint64_t>(res->peak_frontier, std::max(n, nr.peak));
        level = nr.level;
        level_gidx = nr.level_gidx;
        n = nr.n;
        cand = nr.cand;
        if (nr.levels) res->nlevels = n ? level : level - 1;
        if (defer_now_ && nr.levels && nr.reason != NX_ERROR) KC_TRY(counter_snap(level - 1));
        if (nr.reason == NX_ERROR) {
          KC_TRY(report_error(res, h_ns_->err_key, level, level_gidx, n));
          finish(res, t0, 0);
          return 0;
        }
        if (nr.levels > 0 || n == 0) continue;
        // not even one level fitted (buffer room): this level goes wide
      }
      if (n >= (1ull << 32)) {
        set_error("kubecheck: level wider than 2^32 states");
        return -ENOMEM;
      }
      // capacity for this level's output: cand is exact (next_cand of the
      // previous level) when the states are materialised; a deferred level's
      // is estimated, and a level past the estimate (DF_CAPACITY, a full
      // candidate list or table) is redone on the exact path
      const bool dfr = defer_now_ && level > exact_until_;
      if (mat && n) ratio = std::max(1.0, (double)cand / (double)n);
      const uint64_t bound = mat ? cand
                                 : std::min<uint64_t>((uint64_t)((double)n * ratio * defer_slack_) + 4096,
                                                      (uint64_t)M::MAXSUCC * n);
      const bool use_link = !cfg_.keep_trace || cfg_.trace_host;   // links in HBM (the trace may be host memory)
      if (dfr) {
        if (!mat) KC_TRY(grow_buffer(cur_, cur_cap_, n, false, st_));   // (free: the previous frontier is in next_)
        KC_TRY(grow_buffer(pc_cur_, pc_cur_cap_, n, false, st_));
        if (use_link) KC_TRY(grow_buffer(link_next_, link_next_cap_, std::max<uint64_t>(bound, 1), false, st_));
      } else {
        KC_TRY(grow_buffer(next_, next_cap_, cand ? cand : 1, false, st_));
      }
      const uint64_t next_gidx = level_gidx + n;
      if (cfg_.keep_trace) KC_TRY(grow_trace(next_gidx + bound + 1, true));
      // (a deferred level reserves for 16 new states per parent at least:
      // (count + 16 n) * 2 <= capacity keeps even MAXSUCC = 32 per parent
      // from filling the table, whatever the estimate)
      if (!spill_) KC_TRY(cs_.reserve(mat ? bound : std::max<uint64_t>(bound, 16 * n), st_));
      {
        const uint64_t tiles = (std::min(n, chunk) + CLAIM_TILE - 1) / CLAIM_TILE;
        KC_TRY(grow_buffer(rcount_, rcount_cap_, tiles, false, st_));
        if (tscan_) {
          KC_TRY(grow_buffer(ttot_, ttot_cap_, tiles + 4, false, st_));
          KC_TRY(grow_buffer(toff_, toff_cap_, tiles + 4, false, st_));
          if (first_claim_ && chunk_scan_) {
            const uint64_t old = csum_cap_;
            KC_TRY(grow_buffer(csum_, csum_cap_, tiles / CSUM_TILES + 4, false, st_));
            if (csum_cap_ != old) KC_HIP_TRY(hipMemsetAsync(csum_, 0, csum_cap_ * sizeof(uint32_t), st_));
          }
        }
        KC_TRY(grow_buffer(rec_fp_, rec_fp_cap_, tiles * CLAIM_RCAP, false, st_));
        KC_TRY(grow_buffer(rec_lk_, rec_lk_cap_, tiles * CLAIM_RCAP, false, st_));
        KC_TRY(cand_overflow(bound, level, n));
      }
      KC_TRY(grow_buffer(newmask_, mask_cap_, std::min(n, chunk), false, st_));
      DeferArgs df = mat ? DeferArgs{} : defer_args(level_gidx, prev_gidx);
      if (dfr) df.counts_out = pc_cur_;   // this level's plans, for the next level's rebuild
      if (!mat) res->deferred_states += n;
      uint64_t link_cap = ~0ull;
      if (dfr) {
        if (use_link) link_cap = link_next_cap_;
        if (cfg_.keep_trace) link_cap = std::min<uint64_t>(link_cap, std::min(par_cap_, ord_cap_) - next_gidx);
      }
      KC_TRY(grow_buffer(offsets_, off_cap_, std::min(n, chunk), false, st_));
      if (defer_now_)      // (after this level's ClaimSet growth: a rehash later rules out a redo from here)
        hs_[level % 3] = HostSnap{level, n, level_gidx, cand, prev_gidx, cs_.count, res->distinct,
                                  res->peak_frontier, cand_total, cs_.nslots, res->nlevels, mat, ratio};
      const uint32_t succ_level = (uint32_t)level + 1;   // BFS level of the successors
      for (uint64_t start = 0, cn = 0; start < n; start += cn) {
        cn = std::min(chunk, n - start);
        // seen-set spill: a chunk whose insertions fit the hot table (may flush it)
        if (spill_) KC_TRY(spill_cut(cur_ + start, cn, &cn));
        ++res->levels_chunks;
        const unsigned grid = (unsigned)((cn + 255) / 256);
        const unsigned tiles = (unsigned)((cn + CLAIM_TILE - 1) / CLAIM_TILE);
        // first-claim levels with the link emit: tile counts summed per chunk
        // of CSUM_TILES tiles by k_claim, k_chunk_scan over the chunks
        // (KC_CHUNK_SCAN=0: k_tile_scan over every tile)
        const bool cscan = first_claim_ && chunk_scan_ && tscan_ && dfr;
        const unsigned nchunk = (tiles + CSUM_TILES - 1) / CSUM_TILES;
        timed(KK_EXPAND, [&] {
          if (first_claim_) {
            ShardArgs fa = claim_args_;
            fa.ttot = ttot_;
            if (cscan) fa.csum = csum_;
            if (cs_.compact)
              hipLaunchKernelGGL((k_claim<M, 0, false, 0, false, true, true>), dim3(tiles), dim3(CLAIM_TILE), 0, st_,
                                 cur_ + start, cn, start, flags_, cfg_.check_deadlock, cs_.t, cs_.nslots, succ_level,
                                 abl_mask_, rcount_, rec_fp_, rec_lk_, newmask_, d_ctr_, fa, df);
            else
              hipLaunchKernelGGL((k_claim<M, 0, false, 0, false, true>), dim3(tiles), dim3(CLAIM_TILE), 0, st_,
                                 cur_ + start, cn, start, flags_, cfg_.check_deadlock, cs_.t, cs_.nslots, succ_level,
                                 abl_mask_, rcount_, rec_fp_, rec_lk_, newmask_, d_ctr_, fa, df);
          } else {
            hipLaunchKernelGGL(k_claim<M>, dim3(tiles), dim3(CLAIM_TILE), 0, st_, cur_ + start, cn,
                               start, flags_, cfg_.check_deadlock, cs_.t, cs_.nslots, succ_level,
                               abl_mask_, rcount_, rec_fp_, rec_lk_, newmask_, d_ctr_, claim_args_, df);
          }
        });
        if (ablate_) {
          KC_TRY(grow_buffer(abl_mask_, abl_cap_, cn, false, st_));
          timed(KA_LDS, [&] {
            hipLaunchKernelGGL((k_claim<M, 1>), dim3(tiles), dim3(CLAIM_TILE), 0, st_, cur_ + start,
                               cn, start, flags_, cfg_.check_deadlock, cs_.t, cs_.nslots,
                               succ_level, abl_mask_, rcount_, rec_fp_, rec_lk_, newmask_, d_ctr_, claim_args_);
          });
          timed(KA_COMPUTE, [&] {
            hipLaunchKernelGGL((k_claim<M, 2>), dim3(tiles), dim3(CLAIM_TILE), 0, st_, cur_ + start,
                               cn, start, flags_, cfg_.check_deadlock, cs_.t, cs_.nslots,
                               succ_level, abl_mask_, rcount_, rec_fp_, rec_lk_, newmask_, d_ctr_, claim_args_);
          });
          timed(KA_PLAN, [&] {
            hipLaunchKernelGGL((k_claim<M, 3>), dim3(tiles), dim3(CLAIM_TILE), 0, st_, cur_ + start,
                               cn, start, flags_, cfg_.check_deadlock, cs_.t, cs_.nslots,
                               succ_level, abl_mask_, rcount_, rec_fp_, rec_lk_, newmask_, d_ctr_, claim_args_);
          });
          timed(KA_FPCHEAP, [&] {
            hipLaunchKernelGGL((k_claim<M, 4>), dim3(tiles), dim3(CLAIM_TILE), 0, st_, cur_ + start,
                               cn, start, flags_, cfg_.check_deadlock, cs_.t, cs_.nslots,
                               succ_level, abl_mask_, rcount_, rec_fp_, rec_lk_, newmask_, d_ctr_, claim_args_);
          });
          timed(KA_NOAPPLY, [&] {
            hipLaunchKernelGGL((k_claim<M, 5>), dim3(tiles), dim3(CLAIM_TILE), 0, st_, cur_ + start,
                               cn, start, flags_, cfg_.check_deadlock, cs_.t, cs_.nslots,
                               succ_level, abl_mask_, rcount_, rec_fp_, rec_lk_, newmask_, d_ctr_, claim_args_);
          });
        }
        // (a small chunk: the overflow list's pass B inside the tile scan's launch)
        const bool fuse = tscan_ && cn <= FUSE_OVF_SCAN_MAX && !first_claim_;
        if (!first_claim_)
          timed(KK_RESOLVE,
                [&] { launch_settle(cn, start, tiles, succ_level, tscan_ ? ttot_ : (uint32_t*)nullptr, fuse); });
        if (cscan) {
          timed(KK_SCAN, [&] {
            hipLaunchKernelGGL(k_chunk_scan, dim3(1), dim3(TSCAN_THREADS), 0, st_, csum_, nchunk, toff_, tscan_reg_);
          });
        } else if (tscan_) {
          timed(KK_SCAN, [&] {
            if (fuse)
              hipLaunchKernelGGL(k_ovf_tile_scan, dim3(1), dim3(TSCAN_THREADS), 0, st_, claim_args_.ovf, cn, start,
                                 cs_.t, cs_.nslots, succ_level, newmask_, d_ctr_, ClaimKeys(0u), ttot_, tiles, toff_,
                                 tscan_reg_);
            else
              hipLaunchKernelGGL(k_tile_scan, dim3(1), dim3(TSCAN_THREADS), 0, st_, ttot_, tiles, toff_, tscan_reg_);
          });
        } else {
        size_t tmp_bytes = 0;
        const hipcub::TransformInputIterator<uint32_t, NewCount, const uint32_t*> newcnt(newmask_, NewCount());
        KC_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, newcnt, offsets_, (int)cn, st_));
        KC_TRY(grow_buffer(scan_tmp_, scan_cap_, tmp_bytes + 16, false, st_));
        hipError_t scan_err = hipSuccess;
        timed(KK_SCAN, [&] {
          scan_err = hipcub::DeviceScan::ExclusiveSum(scan_tmp_, tmp_bytes, newcnt, offsets_, (int)cn, st_);
        });
        KC_HIP_TRY(scan_err);
        }
        if (spill_) KC_TRY(spill_check(cur_ + start, cn, tiles));
        const uint32_t* toff = tscan_ ? toff_ : nullptr;
        if (ablate_) {
          // cut-down k_emit variants on scratch counters, before the real
          // launch (which rewrites whatever they stored)
          if (!d_ctr_abl_) KC_HIP_TRY(hipMalloc(&d_ctr_abl_, sizeof(Counters)));
          KC_HIP_TRY(hipMemsetAsync(d_ctr_abl_, 0, sizeof(Counters), st_));
          timed(KA_E1, [&] {
            hipLaunchKernelGGL((k_emit<M, 1>), dim3(grid), dim3(256), 0, st_, cur_ + start, cn, start,
                               flags_, newmask_, offsets_, next_, 0ull, level_gidx, next_gidx, parent_, ord_,
                               cfg_.keep_trace, d_ctr_abl_, toff);
          });
          timed(KA_E2, [&] {
            hipLaunchKernelGGL((k_emit<M, 2>), dim3(grid), dim3(256), 0, st_, cur_ + start, cn, start,
                               flags_, newmask_, offsets_, next_, 0ull, level_gidx, next_gidx, parent_, ord_,
                               cfg_.keep_trace, d_ctr_abl_, toff);
          });
          timed(KA_E3, [&] {
            hipLaunchKernelGGL((k_emit<M, 3>), dim3(grid), dim3(256), 0, st_, cur_ + start, cn, start,
                               flags_, newmask_, offsets_, next_, 0ull, level_gidx, next_gidx, parent_, ord_,
                               cfg_.keep_trace, d_ctr_abl_, toff);
          });
        }
        timed(KK_EMIT, [&] {
          if (dfr)
            hipLaunchKernelGGL(k_emit_links, dim3((tiles + EMIT_TPB - 1) / EMIT_TPB), dim3(256), 0, st_, cn, start,
                               newmask_, toff_, level_gidx,
                               next_gidx, cfg_.keep_trace ? parent_ : nullptr, cfg_.keep_trace ? ord_ : nullptr,
                               use_link ? link_next_ : nullptr, link_cap, d_ctr_,
                               cscan ? ttot_ : (const uint32_t*)nullptr);
          else
            hipLaunchKernelGGL(k_emit<M>, dim3(grid), dim3(256), 0, st_, cur_ + start, cn, start,
                               flags_, newmask_, offsets_, next_, 0ull, level_gidx, next_gidx, parent_, ord_,
                               cfg_.keep_trace, d_ctr_, toff);
        });
        const bool last = start + cn >= n;
        hipLaunchKernelGGL(k_advance, dim3(1), dim3(K_ADVANCE_THREADS), 0, st_, offsets_, newmask_, cn, d_ctr_,
                           tscan_ ? toff_ : (const uint32_t*)nullptr, (uint64_t)(cscan ? nchunk : tiles),
                           last && !headcopy_ ? reinterpret_cast<unsigned long long*>(h_ctr_) : nullptr,
                           claim_args_.ovf.count,
                           last && defer_now_ && !headcopy_ ? d_snap_[level % 3].s : (CtrStripe*)nullptr);
      }
      KC_HIP_TRY(hipGetLastError());
      if (headcopy_) {
        KC_HIP_TRY(hipMemcpyAsync(h_ctr_, d_ctr_, kCtrHead, hipMemcpyDeviceToHost, st_));
        hipLaunchKernelGGL(k_level_reset, dim3(1), dim3(64), 0, st_, d_ctr_);   // next level's head
      }
      KC_HIP_TRY(hipStreamSynchronize(st_));
      collect_times();
      const Counters& c = *h_ctr_;
      // a deferred level with anything to report: redo exactly, from the level
      // the anomaly belongs to
      // (first-claim mode: an Assert or deadlock key alone is reported below,
      // from the states this k_claim rebuilt into cur_, exactly as the
      // materialising path's k_claim of this level reports it — no redo)
      const bool key_only = first_claim_ && !c.overflow && !c.batch_used && !c.defer_flags;
      if (dfr && !key_only && (c.overflow || c.batch_used || c.err_key != ~0ull || c.defer_flags)) {
        // an invariant violation among the states this level rebuilt is
        // the previous level's error (its emit would have found it); the
        // rest (Assert / deadlock keys of this level's parents, a capacity
        // estimate too small) are this level's
        if (c.defer_flags == DF_INVARIANT && !c.overflow && !c.batch_used && defer_direct_) {
          // an invariant violation among this level's rebuilt states and
          // nothing else: reported as the previous level's emit would have
          // (no redo), unless the snapshots it needs are missing
          const int rc = report_deferred_invariant(res, level, level_gidx, n);
          if (rc < 0) return rc;
          if (rc == 0) {
            finish(res, t0, 0);
            return 0;
          }
        }
        const int X = (c.defer_flags & DF_INVARIANT) ? level - 1 : level;
        const uint64_t dc_here = c.cand_total - cand_total;
        if (!redo_from(X, level, mat, dc_here, res, n, level_gidx, cand, prev_gidx, cand_total, ratio)) return kDeferRetry;
        level = X;
        mat = true;
        pc_valid_ = false;
        continue;
      }
      if (c.overflow || c.batch_used) {
        set_error("kubecheck: state with more than %d successors or full table", M::MAXSUCC);
        return -ENOMEM;
      }
      const uint64_t n_new = c.chunk_base;
      cs_.count = spill_ ? hot_count_ : cs_.count + n_new;
      res->peak_frontier = std::max<uint64_t>(res->peak_frontier, n);
      if (c.err_key != ~0ull) {
        KC_TRY(report_error(res, c.err_key, level, level_gidx, n));
        res->distinct += n_new;
        finish(res, t0, 0);
        return 0;
      }
      res->distinct += n_new;
      if (cfg_.verbose)
        fprintf(stderr, "kubecheck: level %d width %llu -> %llu new, %llu distinct\n",
                level, (unsigned long long)n, (unsigned long long)n_new,
                (unsigned long long)res->distinct);
      if (!dfr && capture_level_ == level + 1 && n_new) {
        captured_.resize(n_new);
        KC_HIP_TRY(hipMemcpy(captured_.data(), next_, n_new * sizeof(State), hipMemcpyDeviceToHost));
      }
      // successors counted this level: the new states' (materialising emit),
      // or this level's own (a deferred k_claim)
      const uint64_t dc = c.cand_total - cand_total;
      cand_total = c.cand_total;
      if (defer_now_) {              // this level's counters (k_advance) and successor count, for a redo
        if (!headcopy_) snap_lv_[level % 3] = level;
        succ_[level % 3] = mat ? cand : dc;
        succ_lv_[level % 3] = level;
      }
      if (dfr) {
        if (!mat && n) ratio = std::max(1.0, (double)dc / (double)n);
        cand = 0;
        prev_gidx = level_gidx;
        mat = false;
        if (use_link) {
          std::swap(link_cur_, link_next_);
          std::swap(link_cur_cap_, link_next_cap_);
        }
        std::swap(pc_cur_, pc_prev_);
        std::swap(pc_cur_cap_, pc_prev_cap_);
        pc_valid_ = true;
      } else {
        cand = dc;
      }
      level_gidx = next_gidx;
      std::swap(cur_, next_);
      std::swap(cur_cap_, next_cap_);
      n = n_new;
      ++level;
      if (dfr && capture_level_ == level && n) {
        KC_TRY(materialize(n, level_gidx, prev_gidx, cand, cand_total));
        mat = true;
        KC_TRY(counter_snap(level - 1));
        captured_.resize(n);
        KC_HIP_TRY(hipMemcpy(captured_.data(), cur_, n * sizeof(State), hipMemcpyDeviceToHost));
      }
      if (n) {
        if (level > KC_MAX_LEVELS) {
          set_error("kubecheck: more than %d levels", KC_MAX_LEVELS);
          return -ENOMEM;
        }
        res->level_width[level - 1] = n;
        res->nlevels = level;
      }
    }
    // the last, unexpanded level (max_levels): its states' invariants
    if (!mat && n) KC_TRY(materialize(n, level_gidx, prev_gidx, cand, cand_total));
    last_level_ = res->nlevels;
    last_n_ = n;
    finish(res, t0, n);
    if (ablate_) {
      fprintf(stderr, "kubecheck ablate: claim %.2f ms | successors+LDS %.2f ms | successors only %.2f ms | plan only %.2f ms | settle %.2f | emit %.2f ms"
              " | emit-no-plan %.2f | emit-no-plan-no-check %.2f | emit-parent-only %.2f"
              " | successors, XOR fingerprint %.2f | fingerprints, no apply %.2f\n",
              ktime_ms_[KK_EXPAND], ktime_ms_[KA_LDS], ktime_ms_[KA_COMPUTE], ktime_ms_[KA_PLAN], ktime_ms_[KK_RESOLVE],
              ktime_ms_[KK_EMIT], ktime_ms_[KA_E1], ktime_ms_[KA_E2], ktime_ms_[KA_E3], ktime_ms_[KA_FPCHEAP],
              ktime_ms_[KA_NOAPPLY]);
      KC_HIP_TRY(hipMemcpy(h_ctr_, d_ctr_, sizeof(Counters), hipMemcpyDeviceToHost));
      fprintf(stderr, "kubecheck claim outcomes (KC_DIAG builds): old %llu lost %llu cur %llu new %llu\n",
              h_ctr_->claim_out(0), h_ctr_->claim_out(1), h_ctr_->claim_out(2), h_ctr_->claim_out(3));
      fprintf(stderr, "kubecheck old-state level distance (KC_DIAG): 1:%llu 2:%llu 3:%llu 4:%llu 5-8:%llu 9-16:%llu 17+:%llu\n",
              h_ctr_->old_dist(0), h_ctr_->old_dist(1), h_ctr_->old_dist(2), h_ctr_->old_dist(3), h_ctr_->old_dist(4),
              h_ctr_->old_dist(5), h_ctr_->old_dist(6));
      fprintf(stderr, "kubecheck k_claim successor loop (KC_DIAG): wave trips %llu x 64 lanes, lane trips %llu (%.3f busy);"
              " dealt by successor count: wave trips %llu (%.3f busy)\n",
              h_ctr_->loop_max(), h_ctr_->loop_sum(),
              h_ctr_->loop_max() ? (double)h_ctr_->loop_sum() / (64.0 * h_ctr_->loop_max()) : 0.0,
              h_ctr_->loop_sorted(),
              h_ctr_->loop_sorted() ? (double)h_ctr_->loop_sum() / (64.0 * h_ctr_->loop_sorted()) : 0.0);
    }
    return 0;
  }

  size_t trace_text(char* buf, size_t cap) const override;

  // TLC checkFPs over the ClaimSet's fingerprints: compact, radix-sort,
  // minimum adjacent gap (MC.out:42 "based on the actual fingerprints").
  int check_fps(uint64_t* min_gap, double* prob) override {
    KC_HIP_TRY(hipSetDevice(cfg_.device));
    if (spill_) return check_fps_spill(min_gap, prob);
    const uint64_t cnt = std::max<uint64_t>(cs_.count, 2);
    unsigned long long *a = nullptr, *b = nullptr, *d_n = nullptr;
    void* tmp = nullptr;
    int rc = 0;
    unsigned long long n = 0, gap = ~0ull;
    if (hipMalloc(&a, cnt * 8) != hipSuccess || hipMalloc(&b, cnt * 8) != hipSuccess ||
        hipMalloc(&d_n, 16) != hipSuccess) {
      set_error("kc_engine_check_fps: out of device memory");
      rc = -ENOMEM;
    }
    if (!rc) {
      (void)hipMemsetAsync(d_n, 0, 8, st_);
      (void)hipMemcpyAsync(d_n + 1, &gap, 8, hipMemcpyHostToDevice, st_);
      hipLaunchKernelGGL(k_claimset_fps, dim3(table_grid(cs_.nslots)), dim3(256), 0, st_,
                         cs_.words(), cs_.nslots, cs_.word_shift(), a, cnt, d_n);
      (void)hipMemcpyAsync(&n, d_n, 8, hipMemcpyDeviceToHost, st_);
      if (hipStreamSynchronize(st_) != hipSuccess || n > cnt) {
        set_error("kc_engine_check_fps: fingerprint count %llu > %llu", n, (unsigned long long)cnt);
        rc = -EIO;
      }
    }
    if (!rc && n > 1) {
      size_t tb = 0;
      if (hipcub::DeviceRadixSort::SortKeys(nullptr, tb, a, b, (int)n, 0, 64, st_) != hipSuccess ||
          hipMalloc(&tmp, tb) != hipSuccess) {
        set_error("kc_engine_check_fps: sort setup");
        rc = -EIO;
      } else {
        (void)hipcub::DeviceRadixSort::SortKeys(tmp, tb, a, b, (int)n, 0, 64, st_);
        hipLaunchKernelGGL(k_adjacent_min_gap, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st_, b, n,
                           d_n + 1);
        (void)hipMemcpyAsync(&gap, d_n + 1, 8, hipMemcpyDeviceToHost, st_);
        if (hipStreamSynchronize(st_) != hipSuccess) {
          set_error("kc_engine_check_fps: HIP failure");
          rc = -EIO;
        }
      }
    }
    for (void* p : {(void*)a, (void*)b, (void*)d_n, tmp})
      if (p) (void)hipFree(p);
    if (rc) return rc;
    *min_gap = gap;
    *prob = (n > 1 && gap && gap != ~0ull) ? 1.0 / (double)gap : 0.0;
    return 0;
  }
  // the same over hot + cold tiers, on the host (cold keys are mixed
  // fingerprints: unmixed, merged with the hot table's, sorted)
  int check_fps_spill(uint64_t* min_gap, double* prob) {
    std::vector<uint64_t> keys;
    KC_TRY(cold_.all_keys(keys));
    uint64_t* hk = reinterpret_cast<uint64_t*>(sp_arena_);
    KC_HIP_TRY(hipMemsetAsync(d_spctr_ + 1, 0, 8, st_));
    hipLaunchKernelGGL(k_claimset_keys, dim3(table_grid(cs_.nslots)), dim3(256), 0, st_, cs_.t,
                       cs_.nslots, hk, hot_limit_, d_spctr_ + 1);
    KC_HIP_TRY(hipMemcpyAsync(h_spctr_, d_spctr_, 16, hipMemcpyDeviceToHost, st_));
    KC_HIP_TRY(hipStreamSynchronize(st_));
    const uint64_t c = std::min<uint64_t>(h_spctr_[1], hot_limit_);
    const size_t at = keys.size();
    keys.resize(at + c);
    if (c) KC_HIP_TRY(hipMemcpy(keys.data() + at, hk, c * 8, hipMemcpyDeviceToHost));
    for (auto& k : keys) k = cold_unkey(k);
    std::sort(keys.begin(), keys.end());
    uint64_t gap = ~0ull;
    for (size_t i = 1; i < keys.size(); ++i) gap = std::min<uint64_t>(gap, keys[i] - keys[i - 1]);
    *min_gap = gap;
    *prob = (keys.size() > 1 && gap && gap != ~0ull) ? 1.0 / (double)gap : 0.0;
    return 0;
  }
  int trace_tuple(int i, uint64_t* out) const override {
    if (i < 0 || i >= (int)trace_.size()) {
      set_error("trace index out of range");
      return -EINVAL;
    }
    M::to_tuple(trace_[i], out);
    return M::TUPLE_WORDS;
  }
  int64_t level_tuples(int level, uint64_t* out, uint64_t cap) override {
    if (level == capture_level_ && !captured_.empty()) {
      for (uint64_t i = 0; i < captured_.size() && i < cap; ++i)
        M::to_tuple(captured_[i], out + i * M::TUPLE_WORDS);
      return (int64_t)captured_.size();
    }
    if (level == 1) {
      for (uint64_t i = 0; i < init_states_.size() && i < cap; ++i)
        M::to_tuple(init_states_[i], out + i * M::TUPLE_WORDS);
      return (int64_t)init_states_.size();
    }
    set_error("level %d not captured", level);
    return -EINVAL;
  }

 private:
  template <class F>
  void timed(int k, F&& f) {
    // (timing 2: events bracket the roofline kernel only; ten events per
    // level cost the NP=2 check 6 ms and Model_1 4 ms of host/queue time)
    if (timing_ == 1 || (timing_ == 2 && (k == KK_EXPAND || k == KK_NARROW))) {
      if (ev_used_ + 2 > ev_pool_.size()) {
        hipEvent_t a, b;
        (void)hipEventCreate(&a);
        (void)hipEventCreate(&b);
        ev_pool_.push_back(a);
        ev_pool_.push_back(b);
      }
      hipEvent_t a = ev_pool_[ev_used_], b = ev_pool_[ev_used_ + 1];
      (void)hipEventRecord(a, st_);
      f();
      (void)hipEventRecord(b, st_);
      ev_kind_.push_back(k);
      ev_used_ += 2;
    } else {
      f();
    }
    ++klaunch_[k];
  }
  // after the level's sync: accumulate every timed launch
  void collect_times() {
    for (size_t q = 0; q < ev_kind_.size(); ++q) {
      float ms = 0;
      if (hipEventElapsedTime(&ms, ev_pool_[2 * q], ev_pool_[2 * q + 1]) == hipSuccess)
        ktime_ms_[ev_kind_[q]] += ms;
    }
    ev_kind_.clear();
    ev_used_ = 0;
  }

  // parent_host: the parent state when the caller already holds it (the
  // queued path); otherwise it is read from the frontier (cur_)
  int report_error(kc_result* res, uint64_t key, int level, uint64_t level_gidx, uint64_t n,
                   const State* parent_host = nullptr) {
    const int kind = (int)(key & 0xff);
    const int pos = (int)((key >> 8) & 0xff);
    const uint64_t pidx = key >> 16;
    if (pidx >= n) {
      set_error("kubecheck: bad error key");
      return -EIO;
    }
    res->err_kind = kind;
    // path to the parent through the parent pointers (TLC's trace file);
    // without them only the parent itself, still in the current frontier
    std::vector<State> path;
    if (cfg_.keep_trace) {
      KC_TRY(path_to(level_gidx + pidx, path));
    } else if (parent_host) {
      path.assign(1, *parent_host);
    } else {
      path.resize(1);
      KC_HIP_TRY(hipMemcpy(&path[0], cur_ + pidx, sizeof(State), hipMemcpyDeviceToHost));
    }
    const State& s = path.back();
    const typename M::Plan pl = M::plan(s, flags_);
    if (kind == E_ASSERT) {
      res->err_action = M::slot_action(s, pl.fail_slot);
      res->err_self = pl.fail_slot < M::A ? pl.fail_slot
                      : pl.fail_slot < 2 * M::A ? pl.fail_slot - M::A
                                               : M::A + (pl.fail_slot - 2 * M::A);
      res->err_level = level;
    } else if (kind == E_INVARIANT) {
      int slot, j;
      M::locate(pl, pos, slot, j);
      State x;
      M::apply(s, slot, j, flags_, x);
      res->err_invariant = M::check(x, flags_.inv_mask);
      path.push_back(x);
      res->err_level = level + 1;
    } else {
      res->err_level = level;
    }
    if (cfg_.keep_trace) {
      trace_ = path;
      res->trace_len = (int)path.size();
    }
    return 0;
  }

  // Rebuild the states on the path to global state index g by walking the
  // parent pointers (TLC's trace file) and replaying successors on the host.
  int path_to(uint64_t g, std::vector<State>& out) {
    if (!cfg_.keep_trace) {
      set_error("kubecheck: trace requested but keep_trace=0");
      return -EINVAL;
    }
    std::vector<std::pair<uint64_t, uint8_t>> chain;
    if (cfg_.trace_host) {
      KC_HIP_TRY(hipStreamSynchronize(st_));
      for (;;) {
        const unsigned long long p = parent_[g];
        chain.push_back({g, ord_[g]});
        if (p == ~0ull) break;
        g = p;
        if (chain.size() > KC_MAX_LEVELS + 2) {
          set_error("kubecheck: corrupt parent chain");
          return -EIO;
        }
      }
    } else {
      // one lane walks the chain in HBM, one readback (instead of two
      // synchronous 8-B copies per level: the time to a counterexample)
      constexpr uint32_t cap = KC_MAX_LEVELS + 3;
      if (!h_chain_) KC_HIP_TRY(hipHostMalloc(&h_chain_, (cap + 1) * 8));
      hipLaunchKernelGGL(k_parent_chain, dim3(1), dim3(64), 0, st_, parent_, ord_, (uint64_t)g, h_chain_ + 1, cap,
                         h_chain_);
      KC_HIP_TRY(hipGetLastError());
      KC_HIP_TRY(hipStreamSynchronize(st_));
      const uint64_t len = h_chain_[0];
      if (len == 0 || len > cap) {
        set_error("kubecheck: corrupt parent chain");
        return -EIO;
      }
      for (uint64_t k = 0; k < len; ++k) chain.push_back({h_chain_[1 + k] >> 8, (uint8_t)(h_chain_[1 + k] & 0xff)});
    }
    std::reverse(chain.begin(), chain.end());
    out.clear();
    out.push_back(init_states_.at(chain[0].second));
    for (size_t k = 1; k < chain.size(); ++k) {
      const State& s = out.back();
      const typename M::Plan pl = M::plan(s, flags_);
      int slot, j;
      M::locate(pl, chain[k].second, slot, j);
      State x;
      M::apply(s, slot, j, flags_, x);
      out.push_back(x);
    }
    return 0;
  }

  void finish(kc_result* res, std::chrono::steady_clock::time_point t0, uint64_t left) {
    // the striped totals are read once, at the end (levels read only the head)
    if (hipMemcpy(h_ctr_, d_ctr_, sizeof(Counters), hipMemcpyDeviceToHost) != hipSuccess)
      set_error("kubecheck: counter readback failed");
    uint64_t gen = 0;
    for (int a = 0; a < A_COUNT; ++a) {
      res->act_gen[a] = h_ctr_->act_gen(a);
      res->act_dist[a] = h_ctr_->act_dist(a);
      gen += res->act_gen[a];
    }
    res->generated = res->init + gen;
    res->depth = res->nlevels;
    res->queue_left = left;
    res->complete = (left == 0 && res->err_kind == 0 && !(cfg_.max_levels && res->nlevels >= cfg_.max_levels && left));
    const double d = (double)res->distinct, gg = (double)res->generated;
    res->collision_optimistic = d * (gg - d) / 18446744073709551616.0;
    res->fpset_slots = cs_.capacity();
    res->fpset_probes = h_ctr_->probes() + narrow_probes_;
    for (int b = 0; b < OUTDEG_BINS; ++b) res->outdeg_hist[b] = h_ctr_->outdeg(b);
    res->batch_inserts = h_ctr_->settles();
    res->cand_overflow_records = h_ctr_->cand_ovf();
    res->cand_buffer_peak_bytes = cand_buf_peak_;
    res->narrow_levels = narrow_levels_;
    if (spill_) {
      ColdStats cst;
      cold_.stats(&cst);
      unsigned long long hits = 0;
      if (hipMemcpy(&hits, d_spctr_, 8, hipMemcpyDeviceToHost) != hipSuccess) set_error("kubecheck: spill counter readback");
      res->seen_flushes = sp_flushes_;
      res->seen_cold_fps = cst.keys;
      res->seen_cold_queries = sp_queries_;
      res->seen_cold_hits = hits;
      res->seen_cold_runs = cst.runs;
      res->seen_disk_bytes = cst.disk_written;
      res->seen_peak_hbm_bytes = cs_.nslots * cs_.slot_bytes() + sp_arena_bytes_ + cst.peak_meta_bytes;
      res->seen_filter_tests = cst.filter_tests;
      res->seen_filter_passed = cst.filter_passed;
      res->seen_merges = cst.merges;
      res->seen_seconds = sp_seconds_;
      res->seen_flush_seconds = sp_flush_seconds_;
      res->seen_merge_seconds = cst.merge_seconds;
      res->seen_check_seconds = sp_check_seconds_;
      if (cfg_.verbose)
        fprintf(stderr, "kubecheck seen-set spill: %.3f s host (flushes %.3f: pin %.3f merge %.3f meta+copy %.3f files %.3f;"
                        " checks %.3f), %llu flushes, %llu runs (%llu with %llu keys in HBM), %llu merges, %.1f GB uploaded,"
                        " %llu streaming merge-probes\n",
                sp_seconds_, sp_flush_seconds_, cst.pin_seconds, cst.merge_seconds, cst.meta_seconds, cst.evict_seconds,
                sp_check_seconds_, (unsigned long long)sp_flushes_, (unsigned long long)cst.runs,
                (unsigned long long)cst.cached_runs, (unsigned long long)cst.cached_keys,
                (unsigned long long)cst.merges, cst.cache_uploaded / 1e9, (unsigned long long)cst.merge_probes);
    }
    if (q_) {
      kc_squeue_stats qs;
      q_->stats(&qs);
      res->frontier_spilled_bytes = qs.spilled_host_bytes + qs.spilled_disk_bytes;
      res->frontier_reloaded_bytes = qs.reloaded_bytes;
      res->frontier_peak_hbm_bytes = qs.peak_hbm_bytes;
    }
    res->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }

  void release() {
    (void)hipSetDevice(cfg_.device);
    cs_.release();
    q_.reset();
    if (cfg_.trace_host) {
      if (parent_) (void)hipHostFree(parent_);
      if (ord_) (void)hipHostFree(ord_);
      parent_ = nullptr;
      ord_ = nullptr;
    }
    for (void* p : {(void*)ovf_fp_, (void*)ovf_lk_, (void*)ovf_tile_, (void*)d_ovf_cnt_, (void*)link_cur_,
                    (void*)link_next_, (void*)pc_cur_, (void*)pc_prev_})
      if (p) (void)hipFree(p);
    if (sp_arena_) (void)hipFree(sp_arena_);
    if (sp_tsum_) (void)hipFree(sp_tsum_);
    if (d_spctr_) (void)hipFree(d_spctr_);
    if (h_tsum_) (void)hipHostFree(h_tsum_);
    if (h_spctr_) (void)hipHostFree(h_spctr_);
    for (void* p : {(void*)cur_, (void*)next_, (void*)parent_, (void*)ord_, (void*)newmask_, (void*)abl_mask_, (void*)rcount_, (void*)rec_fp_, (void*)rec_lk_,
                    (void*)offsets_, (void*)scan_tmp_, (void*)d_ctr_, (void*)d_ctr_abl_, (void*)ttot_, (void*)toff_,
                    (void*)init_fps_, (void*)init_res_, (void*)csum_})
      if (p) (void)hipFree(p);
    if (h_ctr_) (void)hipHostFree(h_ctr_);
    if (h_chain_) (void)hipHostFree(h_chain_);
    h_chain_ = nullptr;
    if (h_last_) (void)hipHostFree(h_last_);
    if (d_ns_) (void)hipFree(d_ns_);
    if (d_snap_) (void)hipFree(d_snap_);
    if (d_nsc_) (void)hipFree(d_nsc_);
    if (d_ntrace_) (void)hipFree(d_ntrace_);
    if (h_ns_) (void)hipHostFree(h_ns_);
    for (auto& e : ev_pool_) (void)hipEventDestroy(e);
    if (st_) (void)hipStreamDestroy(st_);
  }

  // One launch of k_narrow from the host loop's state; on return the
  // engine's cur_ holds the frontier of level nr.level.
  struct NarrowRun {
    uint64_t n = 0, level_gidx = 0, cand = 0, new_total = 0, peak = 0;
    int level = 0, levels = 0, reason = 0;
  };
  int run_narrow(uint64_t n, int level, uint64_t level_gidx, uint64_t cand, int stop, NarrowRun& nr) {
    constexpr uint64_t kBuf = 1ull << 16;            // frontier room (states) of a narrow run
    constexpr uint64_t kNew = 1ull << 20;            // new states one run may add
    const uint64_t bufs = std::max(cand, kBuf);
    KC_TRY(grow_buffer(cur_, cur_cap_, bufs, true, st_));
    KC_TRY(grow_buffer(next_, next_cap_, bufs, false, st_));
    const uint64_t need_par = level_gidx + n + std::max(cand, kNew) + 1;
    if (cfg_.keep_trace) KC_TRY(grow_trace(need_par, true));
    KC_TRY(cs_.reserve(std::max(cand, kNew), st_));
    NarrowCtl& h = *h_ns_;
    memset(&h, 0, offsetof(NarrowCtl, widths));
    h.n = n;
    h.level_gidx = level_gidx;
    h.cand = cand;
    h.level = (uint32_t)level;
    h.cur_is_b = 0;
    h.buf_cap = std::min(cur_cap_, next_cap_);
    h.par_cap = cfg_.keep_trace ? std::min(par_cap_, ord_cap_) : ~0ull;
    h.room = cs_.capacity() / 2 > cs_.count ? cs_.capacity() / 2 - cs_.count : 0;
    h.stop_level = (uint32_t)stop;
    h.err[0] = h.err[1] = ~0ull;
    h.epoch = ++narrow_epoch_;
    h.reason = narrow_exit_reason(h);
    h.active = h.reason == 0;
    nr = NarrowRun{};
    if (!h.active) {                             // this level cannot run narrow
      nr.n = n, nr.level_gidx = level_gidx, nr.cand = cand, nr.level = level, nr.reason = h.reason;
      return 0;
    }
    KC_HIP_TRY(hipMemcpyAsync(d_ns_, h_ns_, offsetof(NarrowCtl, widths), hipMemcpyHostToDevice, st_));
    // both level tables clear (the last level of the previous run left one dirty)
    KC_HIP_TRY(hipMemsetAsync(d_nsc_, 0, sizeof(NarrowScratch), st_));
    const char* nt = getenv("KC_NARROW_TRACE");
    if (nt && nt[0] == '1' && !d_ntrace_) KC_HIP_TRY(hipMalloc(&d_ntrace_, kNtraceBytes));
    if (d_ntrace_) KC_HIP_TRY(hipMemsetAsync(d_ntrace_, 0, kNtraceBytes, st_));
    // NARROW_BATCH levels' launches per host sync; they all read the control
    // block, so the ones after the run has ended return at once
    State *a = cur_, *b = next_;
    uint32_t lev = 0;                            // level launches enqueued in this run
    // the run's first level is expanded on its own; every k_nfinish then
    // expands the states it emits for the level after it
    hipLaunchKernelGGL(k_nexpand<M>, dim3(NARROW_WG * NARROW_SUB), dim3(NARROW_THREADS), 0, st_, a, b, flags_,
                       cfg_.check_deadlock, 0u, d_ns_, d_nsc_, d_ctr_, d_ntrace_);
    for (;;) {
      // (round 6 captured a batch's launches into a hipGraph, replayed with
      // one hipGraphLaunch: Model_1 2.79-2.82 ms against 2.80 — the cost of
      // a level is its in-kernel chain, not the launches; removed,
      // profiles/r06g_model1_narrow_graph_ab.log)
      timed(KK_NARROW, [&] {
        for (int k = 0; k < narrow_batch_; ++k, ++lev)
          hipLaunchKernelGGL(k_nfinish<M>, dim3(NARROW_FWG), dim3(NARROW_THREADS), 0, st_, a, b, flags_,
                             cfg_.check_deadlock, parent_, ord_, cfg_.keep_trace, lev, d_ns_, d_nsc_, cs_.t,
                             cs_.nslots, d_ctr_, d_ntrace_, cs_.word_shift());
      });
      KC_HIP_TRY(hipGetLastError());
      KC_HIP_TRY(hipMemcpyAsync(h_ns_, d_ns_, offsetof(NarrowCtl, close_acc), hipMemcpyDeviceToHost, st_));
      KC_HIP_TRY(hipMemcpyAsync(h_ctr_, d_ctr_, kCtrHead, hipMemcpyDeviceToHost, st_));
      KC_HIP_TRY(hipStreamSynchronize(st_));
      if (h_ctr_->overflow) {
        set_error("kubecheck: state with more than %d successors", M::MAXSUCC);
        return -ENOMEM;
      }
      if (!h.active) break;
    }
    collect_times();
    if (d_ntrace_) KC_TRY(print_ntrace(lev));
    KC_HIP_TRY(hipMemcpy(h_ns_->widths + level, d_ns_->widths + level,
                         sizeof(uint64_t) * std::min<uint64_t>(h.levels + 1, KC_MAX_LEVELS - level),
                         hipMemcpyDeviceToHost));
    nr.n = h.n;
    nr.level_gidx = h.level_gidx;
    nr.cand = h.cand;
    nr.level = (int)h.level;
    nr.levels = (int)h.levels;
    nr.reason = h.reason;
    nr.new_total = h.new_total;
    nr.peak = 0;
    for (int L = level; L < nr.level && L < KC_MAX_LEVELS; ++L) nr.peak = std::max<uint64_t>(nr.peak, h.widths[L]);
    if (nr.reason == NX_ERROR) h_ctr_->err_key = h.err_key;
    cs_.count += h.new_total;
    narrow_levels_ += h.levels;
    narrow_probes_ += h.probes;
    if (h.cur_is_b) {
      std::swap(cur_, next_);
      std::swap(cur_cap_, next_cap_);
    }
    return 0;
  }

  // Deferred frontier: the rebuild arguments of the level starting at global
  // index level_gidx, whose parents (the previous frontier, from prev_gidx)
  // are in next_; the states go to cur_.
  DeferArgs defer_args(uint64_t level_gidx, uint64_t prev_gidx) const {
    DeferArgs df;
    df.prev = next_;
    df.out = cur_;
    if (!cfg_.keep_trace || cfg_.trace_host) {
      df.link = link_cur_;
    } else {
      df.parent = parent_;
      df.ord = ord_;
      df.gidx0 = level_gidx;
      df.prev_gidx0 = prev_gidx;
    }
    if (pc_valid_) df.prev_counts = pc_prev_;
    return df;
  }
  // Materialise a deferred frontier of n states into cur_ (k_materialize):
  // invariants checked (a violation -> kDeferRetry), actions counted, and
  // the exact successor count of the level into cand.
  int materialize(uint64_t n, uint64_t level_gidx, uint64_t prev_gidx, uint64_t& cand, uint64_t& cand_total) {
    KC_TRY(grow_buffer(cur_, cur_cap_, n, false, st_));
    const DeferArgs df = defer_args(level_gidx, prev_gidx);
    hipLaunchKernelGGL(k_materialize<M>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st_, df, n, flags_, d_ctr_);
    KC_HIP_TRY(hipGetLastError());
    KC_HIP_TRY(hipMemcpyAsync(h_ctr_, d_ctr_, sizeof(Counters), hipMemcpyDeviceToHost, st_));
    KC_HIP_TRY(hipStreamSynchronize(st_));
    if (h_ctr_->defer_flags) return kDeferRetry;
    const uint64_t tot = h_ctr_->next_cand();
    cand = tot - cand_total;
    cand_total = tot;
    return 0;
  }

  // The chunk's candidate overflow list (engine_kernels.h CandOvf), sized by
  // the level's successor count `bound` (no chunk of the level has more), and
  // the peak of the candidate buffers (verbose: per level).
  int cand_overflow(uint64_t bound, int level, uint64_t n) {
    bound = std::max<uint64_t>(bound, 1);
    KC_TRY(grow_buffer_tight(ovf_fp_, ovf_fp_cap_, bound, st_));
    KC_TRY(grow_buffer_tight(ovf_lk_, ovf_lk_cap_, bound, st_));
    KC_TRY(grow_buffer_tight(ovf_tile_, ovf_tile_cap_, bound, st_));
    // empty when allocated and at every run's start (run(); a run that
    // stopped mid-level may have left entries); k_advance empties it again
    // after every chunk, so a level needs no reset launch of its own
    if (!d_ovf_cnt_) {
      KC_HIP_TRY(hipMalloc(&d_ovf_cnt_, 8));
      KC_HIP_TRY(hipMemsetAsync(d_ovf_cnt_, 0, 8, st_));
    }
    claim_args_.ovf = CandOvf{d_ovf_cnt_, ovf_fp_, ovf_lk_, ovf_tile_,
                              std::min(ovf_fp_cap_, std::min(ovf_lk_cap_, ovf_tile_cap_))};
    const uint64_t b = rcount_cap_ * 4 + rec_fp_cap_ * 8 + rec_lk_cap_ * 4 + ovf_fp_cap_ * 8 + ovf_lk_cap_ * 4 +
                       ovf_tile_cap_ * 4;
    cand_buf_peak_ = std::max(cand_buf_peak_, b);
    if (cfg_.verbose)
      fprintf(stderr, "kubecheck: level %d width %llu: candidate buffers %.1f MiB (%.1f B per parent)\n", level,
              (unsigned long long)n, b / 1048576.0, n ? (double)b / (double)n : 0.0);
    return 0;
  }
  unsigned long long* ovf_fp_ = nullptr;
  unsigned int *ovf_lk_ = nullptr, *ovf_tile_ = nullptr;
  uint64_t ovf_fp_cap_ = 0, ovf_lk_cap_ = 0, ovf_tile_cap_ = 0, cand_buf_peak_ = 0;
  unsigned long long* d_ovf_cnt_ = nullptr;
  // deferred frontier (DeferArgs): links of the level being expanded / being
  // emitted, when they are not the (device) trace
  unsigned long long* link_cur_ = nullptr;
  unsigned long long* link_next_ = nullptr;
  uint64_t link_cur_cap_ = 0, link_next_cap_ = 0;
  // plans (Plan::counts) of the frontier being expanded / of the previous one
  unsigned long long* pc_cur_ = nullptr;
  unsigned long long* pc_prev_ = nullptr;
  uint64_t pc_cur_cap_ = 0, pc_prev_cap_ = 0;
  bool pc_valid_ = false;
  static constexpr int kDeferRetry = -100000;
  bool defer_ = false, defer_now_ = false;
  double defer_slack_ = 1.25;
  uint64_t defer_fallbacks_ = 0;
  // deferred-frontier redo from a level (redo_from): per level mod 3, the
  // counters as the level left them (k_advance), the host state as it began
  // and its states' successor count
  struct HostSnap {
    int level = -1;
    uint64_t n = 0, level_gidx = 0, cand = 0, prev_gidx = 0, cs_count = 0, distinct = 0, peak = 0, cand_total = 0,
             nslots = 0;
    int nlevels = 0;
    bool mat = true;
    double ratio = 1.0;
  };
  Counters* d_snap_ = nullptr;        // [3]
  int snap_lv_[3] = {-1, -1, -1};
  HostSnap hs_[3];
  uint64_t succ_[3] = {0, 0, 0};
  int succ_lv_[3] = {-1, -1, -1};
  int exact_until_ = 0;               // levels <= this run on the exact path (after a redo)
  bool redo_on_ = true;               // KC_DEFER_REDO=0: an anomaly redoes the run from Init
  bool defer_direct_ = true;          // KC_DEFER_DIRECT=0: an invariant anomaly is redone too

  // Level L's k_claim rebuilt a state violating an invariant (and found
  // nothing else): the error TLC reports is the first such state of level L
  // in BFS order, the lowest rebuilt index (defer_inv_n).  The materialising
  // path finds it in level L - 1's emit and stops there, so the result is
  // put back as that emit left it: counters of level L - 1 (its k_advance
  // snapshot) with level L's per-action distinct counts (counted here by the
  // rebuild), level L's claims of level L + 1 dropped from the ClaimSet, L - 1
  // levels expanded; the trace is the path to the state through the parent
  // pointers.  1: not possible here (the caller redoes from L - 1).
  int report_deferred_invariant(kc_result* res, int L, uint64_t level_gidx, uint64_t n) {
    if (!cfg_.keep_trace || headcopy_ || !d_snap_ || L < 2 || snap_lv_[(L - 1) % 3] != L - 1) return 1;
    // (k_advance copied it with the level head and reset it)
    const unsigned long long inv_n = h_ctr_->defer_inv_n;
    if (!inv_n) return 1;
    const uint64_t idx = ~(uint64_t)inv_n;
    if (idx >= n) {
      set_error("kubecheck: deferred invariant index %llu past the level's %llu states", (unsigned long long)idx,
                (unsigned long long)n);
      return -EIO;
    }
    KC_TRY(counter_snap(L));
    hipLaunchKernelGGL(k_counters_restore, dim3(1), dim3(64), 0, st_, d_ctr_, d_snap_[(L - 1) % 3].s,
                       d_snap_[L % 3].s);
    // (first-claim mode writes no claim words: there is no level to drop by,
    // and a drop keyed on the empty word would clear every wide-level entry;
    // the run ends here and the next one clears the table)
    if (!first_claim_)
      hipLaunchKernelGGL(k_claimset_drop, dim3(table_grid(cs_.nslots)), dim3(256), 0, st_, cs_.t, cs_.nslots,
                         (uint32_t)L + 1);
    KC_HIP_TRY(hipGetLastError());
    KC_HIP_TRY(hipStreamSynchronize(st_));
    std::vector<State> path;
    KC_TRY(path_to(level_gidx + idx, path));
    res->err_kind = E_INVARIANT;
    res->err_invariant = M::check(path.back(), flags_.inv_mask);
    res->err_level = L;
    res->nlevels = L - 1;
    res->level_width[L - 1] = 0;
    trace_ = path;
    res->trace_len = (int)path.size();
    return 0;
  }

  // The counters after level `lv` (end of a narrow run, or the start) into
  // snapshot lv mod 3.
  int counter_snap(int lv) {
    if (!d_snap_) KC_HIP_TRY(hipMalloc(&d_snap_, 3 * sizeof(Counters)));
    KC_HIP_TRY(hipMemcpyAsync(d_snap_[lv % 3].s, d_ctr_->s, sizeof(d_ctr_->s), hipMemcpyDeviceToDevice, st_));
    snap_lv_[lv % 3] = lv;
    return 0;
  }
  // Put the run back as level X found it (L = the level that met the
  // anomaly, X = L or L - 1): ClaimSet entries of levels > X dropped,
  // counters of level X - 1 restored (k_counters_restore), the host state of X's start; X's
  // states are cur_ (X = L: k_claim rebuilt or had them) or next_ (X = L -
  // 1: the previous frontier).  Levels <= L then run exactly.  False: not
  // possible exactly (the caller redoes the run from Init).
  bool redo_from(int X, int L, bool mat, uint64_t dc_here, kc_result* res, uint64_t& n, uint64_t& level_gidx,
                 uint64_t& cand, uint64_t& prev_gidx, uint64_t& cand_total, double& ratio) {
    if (!redo_on_ || X < 1 || !d_snap_ || snap_lv_[(X - 1) % 3] != X - 1 || hs_[X % 3].level != X) return false;
    // level X's own snapshot: X = L - 1 completed; X = L's k_advance wrote it (the anomaly is seen after)
    if (X != L && snap_lv_[X % 3] != X) return false;
    if (X == L && headcopy_) return false;
    const HostSnap& h = hs_[X % 3];
    if (h.nslots != cs_.nslots) return false;      // rehashed since: dropping entries would break probe chains
    uint64_t c;
    if (X == L) {
      c = mat ? cand : dc_here;                    // k_claim rebuilt the states into cur_ and counted them
    } else {
      if (mat || succ_lv_[X % 3] != X) return false;   // (X's states are the previous frontier, next_)
      c = succ_[X % 3];
    }
    const unsigned grid = (unsigned)std::min<uint64_t>(8192, (cs_.nslots + 255) / 256);
    hipLaunchKernelGGL(k_claimset_drop, dim3(grid), dim3(256), 0, st_, cs_.t, cs_.nslots, (uint32_t)X + 1);
    hipLaunchKernelGGL(k_counters_restore, dim3(1), dim3(64), 0, st_, d_ctr_, d_snap_[(X - 1) % 3].s, d_snap_[X % 3].s);
    hipLaunchKernelGGL(k_level_reset, dim3(1), dim3(64), 0, st_, d_ctr_);
    if (hipGetLastError() != hipSuccess || hipStreamSynchronize(st_) != hipSuccess) return false;
    if (X != L) {
      std::swap(cur_, next_);
      std::swap(cur_cap_, next_cap_);
    }
    n = h.n;
    level_gidx = h.level_gidx;
    cand = c;
    prev_gidx = h.prev_gidx;
    cand_total = h.cand_total;
    ratio = h.ratio;
    cs_.count = h.cs_count;
    res->distinct = h.distinct;
    res->peak_frontier = h.peak;
    res->nlevels = h.nlevels;
    exact_until_ = L;
    res->defer_fallback = 1;
    res->defer_redo_level = (uint64_t)X;
    ++defer_fallbacks_;
    return true;
  }

  // ---- seen-set spill (cfg.seen_hbm_bytes > 0; engine_spill.h, coldset.h).
  // HBM budget B: the hot ClaimSet takes the largest power-of-two table of
  // <= B/2 bytes and holds <= 1/2 load (hot_limit_); one scratch arena serves
  // the flush (the hot keys; the sort borrows the cleared-to-be table) and
  // the per-chunk queries (keys, locations, found flags, sort space; at most
  // q_max_ per chunk); the rest is the cold runs' directories and filters.
  int spill_setup() {
    if (!cs_.t) {
      const uint64_t B = cfg_.seen_hbm_bytes;
      // the hot table's share of the budget: 1/2 (round 4 A/B: 1/4 leaves room
      // for HBM copies of the newest cold runs but doubles the flushes,
      // 6.0-6.6 s against 4.7-5.3 s on NP=2 at 4 GiB)
      uint64_t ns = 1ull << 12;
      while (ns * 2 * sizeof(ClaimEntry) <= B / 2) ns *= 2;
      KC_TRY(cs_.init(ns, st_));
      hot_limit_ = ns / 2;
      q_max_ = std::max<uint64_t>(CLAIM_TILE * 32, hot_limit_ / 3) / 256 * 256;
      size_t tmp = 0;
      {
        hipcub::DoubleBuffer<uint64_t> k(nullptr, nullptr);
        hipcub::DoubleBuffer<uint32_t> v(nullptr, nullptr);
        KC_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, k, v, (int)q_max_, 0, 64, st_));
      }
      sp_qtmp_bytes_ = tmp;
      const uint64_t qbytes = q_max_ * (8 + 8 + 4 + 4 + 1) + tmp + 1024;
      sp_arena_bytes_ = std::max<uint64_t>(hot_limit_ * 8, qbytes);
      KC_HIP_TRY(hipMalloc(&sp_arena_, sp_arena_bytes_));
      KC_HIP_TRY(hipMalloc(&d_spctr_, 64));
      KC_HIP_TRY(hipHostMalloc(&h_spctr_, 64));
      const uint64_t used = ns * sizeof(ClaimEntry) + sp_arena_bytes_;
      if (used + (1ull << 20) > B) {
        set_error("kubecheck: seen_hbm_bytes %llu too small (hot table + scratch need %llu B)",
                  (unsigned long long)B, (unsigned long long)used);
        return -EINVAL;
      }
      ColdSet::Config cc;
      cc.device = cfg_.device;
      cc.meta_hbm_bytes = B - used;
      cc.host_bytes = cfg_.seen_host_bytes;
      cc.dir = cfg_.spill_dir ? cfg_.spill_dir : "";
      const char* wk = getenv("KC_COLD_WINDOW");      // disk-run staging window (keys); tests shrink it
      if (wk && atoll(wk) > 0) cc.window_keys = (uint64_t)atoll(wk);
      const char* bb = getenv("KC_COLD_BLOOM_BITS");  // filter bits per key (0 = no filters; A/B)
      if (bb) cc.bloom_bits = atoi(bb);
      const char* ck = getenv("KC_COLD_CACHE");       // KC_COLD_CACHE=0: no HBM copies of run keys (A/B)
      cc.cache_keys = !(ck && ck[0] == '0');
      KC_TRY(cold_.init(cc));
    } else {
      KC_TRY(cs_.clear(st_));
    }
    cold_.clear();
    hot_count_ = 0;
    sp_flushes_ = sp_queries_ = 0;
    sp_seconds_ = sp_flush_seconds_ = sp_check_seconds_ = 0;
    const char* ss = getenv("KC_SPILL_SYNC");
    sp_sync_check_ = ss && ss[0] == '1';
    KC_HIP_TRY(hipMemsetAsync(d_spctr_, 0, 64, st_));
    return 0;
  }

  // Cut [cur, cur + len) to a chunk whose successors (an upper bound on its
  // hot-table insertions) fit both the table's room and q_max_; flush the
  // hot table into the cold tier first when the room alone would make the
  // chunk less than half as long as q_max_ allows.
  int spill_cut(const State* cur, uint64_t len, uint64_t* cut) {
    const auto t0 = std::chrono::steady_clock::now();
    const uint64_t plan_len = std::min<uint64_t>(len, std::max<uint64_t>(CLAIM_TILE, q_max_ / 2 / 256 * 256));
    const uint64_t tiles = (plan_len + 255) / 256;
    KC_TRY(grow_buffer(sp_tsum_, sp_tsum_cap_, tiles, false, st_));
    KC_TRY(grow_host_buffer(h_tsum_, h_tsum_cap_, tiles, st_));
    hipLaunchKernelGGL(k_tile_succ<M>, dim3((unsigned)tiles), dim3(256), 0, st_, cur, plan_len, flags_, sp_tsum_);
    KC_HIP_TRY(hipMemcpyAsync(h_tsum_, sp_tsum_, tiles * 4, hipMemcpyDeviceToHost, st_));
    KC_HIP_TRY(hipStreamSynchronize(st_));
    auto pick = [&](uint64_t cap) {
      uint64_t acc = 0, c = 0;
      for (uint64_t t = 0; t < tiles; ++t) {
        if (acc + h_tsum_[t] > cap) break;
        acc += h_tsum_[t];
        c = std::min(plan_len, (t + 1) * 256);
      }
      return c;
    };
    const uint64_t room = hot_limit_ > hot_count_ ? hot_limit_ - hot_count_ : 0;
    uint64_t c = pick(std::min(room, q_max_));
    if (c < plan_len && c < pick(q_max_) / 2 && hot_count_ > 0) {
      KC_TRY(spill_flush());
      c = pick(q_max_);
    }
    if (c == 0) {
      set_error("kubecheck: a 256-parent tile has %u successors, more than the seen-set's hot table takes per chunk "
                "(%llu); raise seen_hbm_bytes", h_tsum_[0], (unsigned long long)q_max_);
      return -ENOMEM;
    }
    *cut = c;
    sp_seconds_ += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return 0;
  }

  // Hot table -> one sorted cold run; the table starts over empty.
  int spill_flush() {
    const auto t0 = std::chrono::steady_clock::now();
    uint64_t* keys = reinterpret_cast<uint64_t*>(sp_arena_);
    KC_HIP_TRY(hipMemsetAsync(d_spctr_ + 1, 0, 8, st_));
    hipLaunchKernelGGL(k_claimset_keys, dim3(table_grid(cs_.nslots)), dim3(256), 0, st_, cs_.t,
                       cs_.nslots, keys, hot_limit_, d_spctr_ + 1);
    KC_HIP_TRY(hipMemcpyAsync(h_spctr_, d_spctr_, 16, hipMemcpyDeviceToHost, st_));
    KC_HIP_TRY(hipStreamSynchronize(st_));
    const uint64_t c = h_spctr_[1];
    if (c > hot_limit_) {
      set_error("kubecheck: hot seen-set holds %llu > %llu fingerprints", (unsigned long long)c,
                (unsigned long long)hot_limit_);
      return -EIO;
    }
    if (c) {
      // sort in place, borrowing the hot table (cleared right after) as the
      // alternate buffer and temporary storage
      uint64_t* alt = reinterpret_cast<uint64_t*>(cs_.t);
      const uint64_t tab = cs_.nslots * sizeof(ClaimEntry);
      const uint64_t off = (c * 8 + 255) / 256 * 256;
      hipcub::DoubleBuffer<uint64_t> kb(keys, alt);
      size_t tb = 0;
      KC_HIP_TRY(hipcub::DeviceRadixSort::SortKeys(nullptr, tb, kb, (int)c, 0, 64, st_));
      if (off + tb > tab) {
        set_error("kubecheck: seen-set flush sort needs %llu B > %llu", (unsigned long long)(off + tb),
                  (unsigned long long)tab);
        return -ENOMEM;
      }
      KC_HIP_TRY(hipcub::DeviceRadixSort::SortKeys(reinterpret_cast<uint8_t*>(cs_.t) + off, tb, kb, (int)c, 0, 64, st_));
      KC_TRY(cold_.add_run(kb.Current(), c, st_));
    }
    KC_TRY(cs_.clear(st_));
    hot_count_ = 0;
    ++sp_flushes_;
    sp_flush_seconds_ += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return 0;
  }

  // After the chunk's claim + settle + tile scan: its winners w.r.t. the hot
  // tier are checked against the cold tier; those found lose (k_spill_apply)
  // and the tile offsets are recomputed.
  int spill_check(const State* cur, uint64_t cn, unsigned tiles) {
    const auto t0 = std::chrono::steady_clock::now();
    uint8_t* a = sp_arena_;
    uint64_t* qk = reinterpret_cast<uint64_t*>(a);
    uint64_t* qk2 = qk + q_max_;
    uint32_t* ql = reinterpret_cast<uint32_t*>(qk2 + q_max_);
    uint32_t* ql2 = ql + q_max_;
    uint8_t* found = reinterpret_cast<uint8_t*>(ql2 + q_max_);
    uint8_t* tmp = found + (q_max_ + 255) / 256 * 256;
    hipLaunchKernelGGL(k_spill_queries<M>, dim3(tiles), dim3(256), 0, st_, cur, cn, flags_, newmask_, toff_, qk, ql);
    KC_HIP_TRY(hipMemcpyAsync(h_spctr_ + 2, toff_ + tiles, 4, hipMemcpyDeviceToHost, st_));
    KC_HIP_TRY(hipStreamSynchronize(st_));
    const uint64_t m = (uint32_t)h_spctr_[2];
    if (m > q_max_) {
      set_error("kubecheck: chunk has %llu new fingerprints > %llu", (unsigned long long)m,
                (unsigned long long)q_max_);
      return -EIO;
    }
    hot_count_ += m;
    sp_queries_ += m;
    if (m && !cold_.empty()) {
      hipcub::DoubleBuffer<uint64_t> kb(qk, qk2);
      hipcub::DoubleBuffer<uint32_t> vb(ql, ql2);
      size_t tb = sp_qtmp_bytes_;
      KC_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tb, kb, vb, (int)m, 0, 64, st_));
      KC_HIP_TRY(hipMemsetAsync(found, 0, m, st_));
      KC_TRY(cold_.probe(kb.Current(), m, found, d_spctr_, st_));
      hipLaunchKernelGGL(k_spill_apply, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, st_, kb.Current(),
                         vb.Current(), found, m, newmask_, ttot_, cs_.t, cs_.nslots, d_ctr_);
      hipLaunchKernelGGL(k_tile_scan, dim3(1), dim3(TSCAN_THREADS), 0, st_, ttot_, tiles, toff_, tscan_reg_);
      KC_HIP_TRY(hipGetLastError());
      if (sp_sync_check_) KC_HIP_TRY(hipStreamSynchronize(st_));   // (KC_SPILL_SYNC=1: time the check itself)
    }
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    sp_seconds_ += dt;
    sp_check_seconds_ += dt;
    return 0;
  }

  bool spill_ = false;
  ColdSet cold_;
  uint64_t hot_limit_ = 0, q_max_ = 0, hot_count_ = 0;
  uint8_t* sp_arena_ = nullptr;
  uint64_t sp_arena_bytes_ = 0;
  size_t sp_qtmp_bytes_ = 0;
  uint32_t *sp_tsum_ = nullptr, *h_tsum_ = nullptr;
  uint64_t sp_tsum_cap_ = 0, h_tsum_cap_ = 0;
  unsigned long long *d_spctr_ = nullptr, *h_spctr_ = nullptr;   // [0] cold hits, [1] flush count
  uint64_t sp_flushes_ = 0, sp_queries_ = 0;
  double sp_seconds_ = 0, sp_flush_seconds_ = 0, sp_check_seconds_ = 0;
  bool sp_sync_check_ = false;

  // the trace file (parent index + ordinal per state) in HBM, or in pinned
  // host RAM with cfg.trace_host (kernels store into it directly)
  int grow_trace(uint64_t need, bool keep) {
    if (cfg_.trace_host) {
      KC_TRY(grow_host_buffer(parent_, par_cap_, need, st_));
      return grow_host_buffer(ord_, ord_cap_, need, st_);
    }
    KC_TRY(grow_buffer(parent_, par_cap_, need, keep, st_));
    return grow_buffer(ord_, ord_cap_, need, keep, st_);
  }

  // ---- frontiers in the StateQueue (cfg.frontier_hbm_bytes > 0; squeue.h).
  // The queue holds level L's states followed by level L+1's as they are
  // made.  Each chunk of <= one segment of parents is read in place from the
  // head (front), expanded by the same kernels as the in-HBM path, and its
  // new states go straight into a run reserved at the tail; segments past
  // the HBM budget spill to host RAM / disk and come back when the head
  // reaches them.  A chunk's parents are popped one chunk later, after the
  // sync that would report an error found among them.  One host sync per
  // chunk: its new-state count sizes the reservation.  Same kernels, same
  // order keys: results equal the in-HBM path's.
  int run_queued(kc_result* res, std::chrono::steady_clock::time_point t0, uint64_t n, uint64_t cand,
                 const std::vector<State>& init) {
    if (!q_) {
      SegQueue::Config qc;
      qc.words = M::W;
      qc.device = cfg_.device;
      qc.seg_states = cfg_.frontier_segment_states ? cfg_.frontier_segment_states : (1ull << 22);
      qc.hbm_bytes = cfg_.frontier_hbm_bytes;
      qc.host_bytes = cfg_.frontier_host_bytes;
      qc.dir = cfg_.spill_dir ? cfg_.spill_dir : "";
      q_.reset(new SegQueue());
      KC_TRY(q_->init(qc));
    }
    if (!h_last_) KC_HIP_TRY(hipHostMalloc(&h_last_, 16));
    KC_TRY(q_->clear(st_));
    KC_TRY(q_->enqueue_host(reinterpret_cast<const uint64_t*>(init.data()), n, st_));
    const uint64_t chunk = std::min<uint64_t>(
        std::min<uint64_t>(cfg_.chunk_states ? cfg_.chunk_states : kMaxChunk, kMaxChunk), q_->seg_states());
    uint64_t level_gidx = 0, cand_total = 0;
    int level = 1;
    State err_parent{};
    hipLaunchKernelGGL(k_level_reset, dim3(1), dim3(64), 0, st_, d_ctr_);
    while (n > 0) {
      if (cfg_.max_levels && level >= cfg_.max_levels) break;
      if (n >= (1ull << 32)) {
        set_error("kubecheck: level wider than 2^32 states");
        return -ENOMEM;
      }
      const uint64_t next_gidx = level_gidx + n;
      if (cfg_.keep_trace) KC_TRY(grow_trace(next_gidx + cand + 1, true));
      if (!spill_) KC_TRY(cs_.reserve(cand, st_));
      const uint64_t cmax = std::min(n, chunk);
      {
        const uint64_t tiles = (cmax + CLAIM_TILE - 1) / CLAIM_TILE;
        KC_TRY(grow_buffer(rcount_, rcount_cap_, tiles, false, st_));
        if (tscan_) {
          KC_TRY(grow_buffer(ttot_, ttot_cap_, tiles + 4, false, st_));
          KC_TRY(grow_buffer(toff_, toff_cap_, tiles + 4, false, st_));
        }
        KC_TRY(grow_buffer(rec_fp_, rec_fp_cap_, tiles * CLAIM_RCAP, false, st_));
        KC_TRY(grow_buffer(rec_lk_, rec_lk_cap_, tiles * CLAIM_RCAP, false, st_));
        KC_TRY(cand_overflow(cand, level, n));
      }
      KC_TRY(grow_buffer(newmask_, mask_cap_, cmax, false, st_));
      KC_TRY(grow_buffer(offsets_, off_cap_, cmax, false, st_));
      const uint32_t succ_level = (uint32_t)level + 1;
      uint64_t start = 0, level_new = 0, popped = 0, pend = 0;
      unsigned long long seen_err = ~0ull;
      bool have_parent = false;
      // after a sync: overflow, and a new minimum error key, whose parent
      // (in this chunk or the one before, neither popped yet) is copied out
      auto check = [&](uint64_t hi) -> int {
        const Counters& c = *h_ctr_;
        if (c.overflow || c.batch_used) {
          set_error("kubecheck: state with more than %d successors or full table", M::MAXSUCC);
          return -ENOMEM;
        }
        if (c.err_key != seen_err) {
          seen_err = c.err_key;
          const uint64_t pidx = seen_err >> 16;
          if (pidx < popped || pidx >= hi) {
            set_error("kubecheck: bad error key");
            return -EIO;
          }
          const uint64_t* p = nullptr;
          uint64_t got = 0;
          KC_TRY(q_->front(pidx - popped, 1, &p, &got, st_));
          KC_HIP_TRY(hipMemcpyAsync(&err_parent, p, sizeof(State), hipMemcpyDeviceToHost, st_));
          KC_HIP_TRY(hipStreamSynchronize(st_));
          have_parent = true;
        }
        return 0;
      };
      while (start < n) {
        const uint64_t* p = nullptr;
        uint64_t m = 0;
        KC_TRY(q_->front(start - popped, std::min(chunk, n - start), &p, &m, st_));
        if (m == 0) {
          set_error("kubecheck: StateQueue holds fewer states than the level");
          return -EIO;
        }
        const State* cur = reinterpret_cast<const State*>(p);
        // seen-set spill: a chunk whose insertions fit the hot table (may flush it)
        if (spill_) KC_TRY(spill_cut(cur, m, &m));
        ++res->levels_chunks;
        const unsigned tiles = (unsigned)((m + CLAIM_TILE - 1) / CLAIM_TILE);
        timed(KK_EXPAND, [&] {
          hipLaunchKernelGGL(k_claim<M>, dim3(tiles), dim3(CLAIM_TILE), 0, st_, cur, m, start, flags_,
                             cfg_.check_deadlock, cs_.t, cs_.nslots, succ_level, abl_mask_, rcount_, rec_fp_,
                             rec_lk_, newmask_, d_ctr_, claim_args_);
        });
        timed(KK_RESOLVE, [&] { launch_settle(m, start, tiles, succ_level, spill_ ? ttot_ : (uint32_t*)nullptr); });
        if (spill_) {
          // the tile-count path: the cold check clears winners and recounts tiles
          timed(KK_SCAN, [&] {
            hipLaunchKernelGGL(k_tile_scan, dim3(1), dim3(TSCAN_THREADS), 0, st_, ttot_, tiles, toff_, tscan_reg_);
          });
          KC_TRY(spill_check(cur, m, tiles));
          KC_HIP_TRY(hipMemcpyAsync(h_last_, toff_ + tiles, 4, hipMemcpyDeviceToHost, st_));
          h_last_[1] = 0;
        } else {
          size_t tmp_bytes = 0;
          const hipcub::TransformInputIterator<uint32_t, NewCount, const uint32_t*> newcnt(newmask_, NewCount());
          KC_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, newcnt, offsets_, (int)m, st_));
          KC_TRY(grow_buffer(scan_tmp_, scan_cap_, tmp_bytes + 16, false, st_));
          hipError_t scan_err = hipSuccess;
          timed(KK_SCAN, [&] {
            scan_err = hipcub::DeviceScan::ExclusiveSum(scan_tmp_, tmp_bytes, newcnt, offsets_, (int)m, st_);
          });
          KC_HIP_TRY(scan_err);
          KC_HIP_TRY(hipMemcpyAsync(h_last_, offsets_ + m - 1, 4, hipMemcpyDeviceToHost, st_));
          KC_HIP_TRY(hipMemcpyAsync(h_last_ + 1, newmask_ + m - 1, 4, hipMemcpyDeviceToHost, st_));
        }
        KC_HIP_TRY(hipMemcpyAsync(h_ctr_, d_ctr_, kCtrHead, hipMemcpyDeviceToHost, st_));
        KC_HIP_TRY(hipStreamSynchronize(st_));
        collect_times();
        KC_TRY(check(start + m));
        const uint64_t nn = (uint64_t)h_last_[0] + NewCount()(h_last_[1]);
        uint64_t* dst = nullptr;
        if (nn) KC_TRY(q_->reserve(nn, &dst, st_));
        timed(KK_EMIT, [&] {
          hipLaunchKernelGGL(k_emit<M>, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, st_, cur, m, start,
                             flags_, newmask_, offsets_, reinterpret_cast<State*>(dst), level_new, level_gidx,
                             next_gidx, parent_, ord_, cfg_.keep_trace, d_ctr_,
                             spill_ ? (const uint32_t*)toff_ : (const uint32_t*)nullptr);
        });
        hipLaunchKernelGGL(k_advance, dim3(1), dim3(K_ADVANCE_THREADS), 0, st_, offsets_, newmask_, m, d_ctr_,
                           spill_ ? (const uint32_t*)toff_ : (const uint32_t*)nullptr, (uint64_t)(spill_ ? tiles : 0),
                           (unsigned long long*)nullptr, claim_args_.ovf.count);
        KC_HIP_TRY(hipGetLastError());
        if (nn) KC_TRY(q_->commit(nn, st_));
        level_new += nn;
        if (pend) KC_TRY(q_->pop(pend, st_));
        popped += pend;
        pend = m;
        start += m;
      }
      KC_HIP_TRY(hipMemcpyAsync(h_ctr_, d_ctr_, kCtrHead, hipMemcpyDeviceToHost, st_));
      KC_HIP_TRY(hipStreamSynchronize(st_));
      collect_times();
      KC_TRY(check(n));
      if (h_ctr_->chunk_base != level_new) {
        set_error("kubecheck: StateQueue level count %llu != %llu", (unsigned long long)level_new,
                  (unsigned long long)h_ctr_->chunk_base);
        return -EIO;
      }
      const uint64_t cand_now = h_ctr_->cand_total;
      hipLaunchKernelGGL(k_level_reset, dim3(1), dim3(64), 0, st_, d_ctr_);   // next level's head
      cs_.count = spill_ ? hot_count_ : cs_.count + level_new;
      res->peak_frontier = std::max<uint64_t>(res->peak_frontier, n);
      if (seen_err != ~0ull) {
        KC_TRY(report_error(res, seen_err, level, level_gidx, n, have_parent ? &err_parent : nullptr));
        res->distinct += level_new;
        finish(res, t0, 0);
        return 0;
      }
      if (pend) KC_TRY(q_->pop(pend, st_));
      res->distinct += level_new;
      if (cfg_.verbose) {
        kc_squeue_stats qs;
        q_->stats(&qs);
        fprintf(stderr, "kubecheck: level %d width %llu -> %llu new, %llu distinct; queue %llu HBM / %llu host / %llu disk segments\n",
                level, (unsigned long long)n, (unsigned long long)level_new, (unsigned long long)res->distinct,
                (unsigned long long)qs.seg_hbm, (unsigned long long)qs.seg_host, (unsigned long long)qs.seg_disk);
      }
      if (capture_level_ == level + 1 && level_new) {
        captured_.resize(level_new);
        KC_TRY(q_->peek_host(0, level_new, reinterpret_cast<uint64_t*>(captured_.data()), st_));
      }
      level_gidx = next_gidx;
      n = level_new;
      cand = cand_now - cand_total;
      cand_total = cand_now;
      ++level;
      if (n) {
        if (level > KC_MAX_LEVELS) {
          set_error("kubecheck: more than %d levels", KC_MAX_LEVELS);
          return -ENOMEM;
        }
        res->level_width[level - 1] = n;
        res->nlevels = level;
      }
    }
    last_level_ = res->nlevels;
    last_n_ = n;
    finish(res, t0, n);
    return 0;
  }

  // KC_NARROW_TRACE=1: per-phase timestamps of the narrow kernels (thread 0
  // of every workgroup), summarised on stderr after each narrow run
  static constexpr size_t kNtraceBytes = (NTRACE_FOFF + NTRACE_LEVELS * NARROW_FWG * NTRACE_PH) * 8;
  int print_ntrace(uint32_t launches) {
    std::vector<unsigned long long> t(kNtraceBytes / 8);
    KC_HIP_TRY(hipMemcpy(t.data(), d_ntrace_, kNtraceBytes, hipMemcpyDeviceToHost));
    const int FW = NARROW_FWG;
    constexpr int P = NTRACE_PH;
    double all[P] = {}, w0[P] = {}, span = 0, gap = 0, close = 0, pub_spread = 0;
    int nl = 0, ng = 0;
    unsigned long long prev_end = 0;
    for (uint32_t l = 0; l < launches && l < NTRACE_LEVELS; ++l) {
      const unsigned long long* f = &t[NTRACE_FOFF + (uint64_t)l * FW * P];
      if (!f[1]) {                                     // inactive launch
        prev_end = 0;
        continue;
      }
      unsigned long long f0 = ~0ull, f9 = 0, f10 = 0, f4min = ~0ull, f4max = 0;
      for (int w = 0; w < FW; ++w) {
        const unsigned long long* q = f + w * P;
        f0 = std::min(f0, q[0]);
        f4min = std::min(f4min, q[3]);
        f4max = std::max(f4max, q[3]);
        f9 = std::max(f9, q[9]);
        if (q[10]) f10 = q[10];
        for (int k = 1; k <= 9; ++k) all[k] += (double)(q[k] - q[k - 1]) / FW;
      }
      for (int k = 1; k <= 9; ++k) w0[k] += (double)(f[k] - f[k - 1]);   // workgroup 0 (always live)
      close += (double)(f10 - f9);
      span += (double)(f10 - f0);
      pub_spread += (double)(f4max - f4min);
      if (prev_end && f0 > prev_end) {
        gap += (double)(f0 - prev_end);
        ++ng;
      }
      prev_end = f10;
      ++nl;
    }
    if (!nl) return 0;
    const double u = 0.01 / nl;             // 100 MHz ticks -> us, per level
    static const char* names[P] = {"", "start", "successors+ClaimSet", "mask scan", "publish+wait", "emit",
                                   "task scan", "expand tasks", "clear", "counters", "", ""};
    std::string a = "kubecheck narrow trace (" + std::to_string(nl) + " levels, us per level; mean over workgroups / workgroup 0):";
    char buf[96];
    for (int k = 1; k <= 9; ++k) {
      snprintf(buf, sizeof buf, " %s %.2f/%.2f,", names[k], all[k] * u, w0[k] * u);
      a += buf;
    }
    snprintf(buf, sizeof buf, " close %.2f; span %.2f; publish spread %.2f; gap between levels %.2f\n", close * u,
             span * u, pub_spread * u, ng ? gap * 0.01 / ng : 0.0);
    a += buf;
    fputs(a.c_str(), stderr);
    return 0;
  }
  unsigned long long* d_ntrace_ = nullptr;

  Flags flags_{};
  ShardArgs claim_args_{};
  bool queued_ = false;
  std::unique_ptr<SegQueue> q_;
  uint32_t* h_last_ = nullptr;       // pinned: a chunk's last offset and mask
  hipStream_t st_ = nullptr;
  NarrowCtl *d_ns_ = nullptr, *h_ns_ = nullptr;
  NarrowScratch* d_nsc_ = nullptr;
  bool narrow_on_ = true;
  uint64_t narrow_probes_ = 0;
  uint32_t narrow_epoch_ = 0;
  DevClaimSet cs_;
  State *cur_ = nullptr, *next_ = nullptr;
  uint64_t cur_cap_ = 0, next_cap_ = 0;
  unsigned long long* parent_ = nullptr;
  uint8_t* ord_ = nullptr;
  uint64_t par_cap_ = 0, ord_cap_ = 0;
  uint32_t *newmask_ = nullptr, *offsets_ = nullptr;
  uint32_t* abl_mask_ = nullptr;
  Counters* d_ctr_abl_ = nullptr;   // KC_ABLATE: scratch counters of the k_emit variants
  // Default: settle pass B counts each tile's new states and one workgroup
  // scans the tile counts (k_tile_scan); KC_TSCAN=0: the per-parent hipcub
  // scan instead.  KC_HEADCOPY=1: the level head read back by a copy launch
  // plus a reset launch instead of k_advance's direct write.  (Same-box A/B,
  // NP=2 with events on every kernel: 165.7 ms both off, 163.9 direct head,
  // 162.5 both on; profiles/r02o_ab1.txt.)
  bool tscan_ = false, headcopy_ = false;
  int narrow_batch_ = NARROW_BATCH;
  int tscan_reg_ = 1;   // KC_TSCAN_REG=0: k_tile_scan's loop path (levels > 65,536 tiles) at any width
  // settle passes A and B of a chunk's tiles (k_settle_rec, one workgroup
  // per tile; round 5 measured 2 / 4 / 8 tiles per workgroup no faster,
  // DESIGN §7.3), then the overflow list's pass B
  void launch_settle(uint64_t cn, uint64_t start, unsigned tiles, uint32_t succ_level, uint32_t* ttot,
                     bool ovf_in_scan = false) {
    hipLaunchKernelGGL(k_settle_rec<0>, dim3(tiles + SETTLE_OVF_BLOCKS), dim3(CLAIM_TILE), 0, st_, cn, start,
                       cs_.t, cs_.nslots, succ_level, rcount_, rec_fp_, rec_lk_, newmask_, d_ctr_, 0u,
                       (uint32_t*)nullptr, tiles, claim_args_.ovf);
    hipLaunchKernelGGL(k_settle_rec<1>, dim3(tiles), dim3(CLAIM_TILE), 0, st_, cn, start, cs_.t, cs_.nslots,
                       succ_level, rcount_, rec_fp_, rec_lk_, newmask_, d_ctr_, 0u, ttot);
    if (!ovf_in_scan)   // (else k_ovf_tile_scan settles it)
      hipLaunchKernelGGL(k_settle_ovf<1>, dim3(SETTLE_OVF_GRID), dim3(256), 0, st_, claim_args_.ovf, cn, start, cs_.t,
                         cs_.nslots, succ_level, newmask_, d_ctr_, 0u, ttot);
  }
  // k_chunk_scan's chunk sums (zeroed at allocation and by each scan)
  bool chunk_scan_ = true;
  uint32_t* csum_ = nullptr;
  uint64_t csum_cap_ = 0;
  uint64_t* init_fps_ = nullptr;
  int* init_res_ = nullptr;
  uint64_t init_fps_cap_ = 0, init_res_cap_ = 0;
  bool first_claim_ = false;   // KC_FIRST_CLAIM=1: k_claim FIRST, no settle passes (multi-worker TLC semantics)
  uint32_t *ttot_ = nullptr, *toff_ = nullptr;
  uint64_t ttot_cap_ = 0, toff_cap_ = 0;
  unsigned int *rcount_ = nullptr, *rec_lk_ = nullptr;
  unsigned long long* rec_fp_ = nullptr;
  uint64_t rcount_cap_ = 0, rec_fp_cap_ = 0, rec_lk_cap_ = 0;
  uint64_t abl_cap_ = 0;
  uint64_t mask_cap_ = 0, off_cap_ = 0;
  uint8_t* scan_tmp_ = nullptr;
  uint64_t scan_cap_ = 0;
  Counters* d_ctr_ = nullptr;
  Counters* h_ctr_ = nullptr;
  uint64_t* h_chain_ = nullptr;        // pinned: [0] length, then the parent chain (k_parent_chain)
  std::vector<hipEvent_t> ev_pool_;
  std::vector<int> ev_kind_;
  size_t ev_used_ = 0;
  std::vector<State> init_states_, trace_, captured_;
  uint64_t last_n_ = 0;
  int last_level_ = 0;
};

template <class M>
size_t EngineT<M>::trace_text(char* buf, size_t cap) const {
  std::string s;
  for (size_t i = 0; i < trace_.size(); ++i) {
    s += "State " + std::to_string(i + 1) + ":\n";
    std::vector<uint64_t> t(M::TUPLE_WORDS);
    M::to_tuple(trace_[i], t.data());
    s += format_tuple(t.data(), cfg_.nc, cfg_.np, cfg_.ns, (cfg_.invariants & 4) != 0);
    s += "\n";
  }
  if (buf && cap) {
    const size_t k = std::min(cap - 1, s.size());
    memcpy(buf, s.data(), k);
    buf[k] = 0;
  }
  return s.size() + 1;
}

std::unique_ptr<EngineBase> make_engine(const kc_model_config& cfg) {
#define KC_MAKE(a, b, c)                                              \
  if (cfg.nc == a && cfg.np == b && cfg.ns == c)                      \
    return std::unique_ptr<EngineBase>(new EngineT<Model<a, b, c>>(cfg));
  KC_FOR_EACH_MODEL(KC_MAKE)
#undef KC_MAKE
  return nullptr;
}

}  // namespace kc

using namespace kc;

struct kc_engine {
  std::unique_ptr<EngineBase> impl;
};

extern "C" {

void kc_model_config_default(kc_model_config* c) {
  if (!c) return;
  memset(c, 0, sizeof *c);
  c->nc = c->np = c->ns = 1;
  c->can_fail = c->can_timeout = 1;
  c->check_deadlock = 1;
  c->keep_trace = 1;
  c->invariants = 3;
}

int kc_engine_create(const kc_model_config* cfg, kc_engine** out) {
  if (!cfg || !out) { set_error("kc_engine_create: NULL argument"); return -EINVAL; }
  *out = nullptr;
  auto impl = make_engine(*cfg);
  if (!impl) {
    set_error("kc_engine_create: unsupported model nc=%d np=%d ns=%d", cfg->nc, cfg->np, cfg->ns);
    return -EINVAL;
  }
  KC_TRY(impl->setup());
  *out = new kc_engine{std::move(impl)};
  return 0;
}

void kc_engine_destroy(kc_engine* e) { delete e; }

int kc_engine_run(kc_engine* e, kc_result* res) {
  if (!e || !res) { set_error("kc_engine_run: NULL argument"); return -EINVAL; }
  return e->impl->run(res);
}

size_t kc_engine_trace_text(kc_engine* e, char* buf, size_t cap) {
  return e ? e->impl->trace_text(buf, cap) : 0;
}

int kc_engine_trace_tuple(kc_engine* e, int i, uint64_t* out) {
  if (!e || !out) { set_error("kc_engine_trace_tuple: NULL"); return -EINVAL; }
  return e->impl->trace_tuple(i, out);
}

int64_t kc_engine_level_tuples(kc_engine* e, int level, uint64_t* out, uint64_t cap) {
  if (!e) { set_error("kc_engine_level_tuples: NULL"); return -EINVAL; }
  return e->impl->level_tuples(level, out, cap);
}

int kc_engine_capture_level(kc_engine* e, int level) {
  if (!e) { set_error("kc_engine_capture_level: NULL"); return -EINVAL; }
  e->impl->set_capture(level);
  return 0;
}

int kc_engine_narrow_times(kc_engine* e, double* ms, uint64_t* launches, uint64_t* levels) {
  if (!e || !ms || !launches || !levels) { set_error("kc_engine_narrow_times: NULL"); return -EINVAL; }
  e->impl->narrow_times(ms, launches, levels);
  return 0;
}

int kc_engine_check_fps(kc_engine* e, uint64_t* min_gap, double* prob) {
  if (!e || !min_gap || !prob) { set_error("kc_engine_check_fps: NULL"); return -EINVAL; }
  return e->impl->check_fps(min_gap, prob);
}

int kc_engine_kernel_times(kc_engine* e, double* ms4, uint64_t* launches4) {
  if (!e) { set_error("kc_engine_kernel_times: NULL"); return -EINVAL; }
  e->impl->kernel_times(ms4, launches4);
  return 0;
}

}  // extern "C"
