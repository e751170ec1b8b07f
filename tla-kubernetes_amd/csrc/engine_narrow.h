// engine_narrow.h — device-driven narrow BFS levels (gfx950).
//
// While the frontier is small (<= NARROW_MAX parents) a level is run by four
// short kernels that read the level's size and buffers from a control block
// in device memory (NarrowCtl) instead of from the host; the host enqueues
// NARROW_BATCH levels' worth of them back to back and synchronises once per
// batch.  Each kernel returns at once when the control block is inactive,
// so the launches after the level that ended the narrow run are nearly free.
//
// Why: the reference's own model (Model_1, MC.cfg) is deep and narrow: 124
// levels, at most 3,939 states wide.  On the wide-level path
// every level costs ~6 launches AND a host round trip (~70 us) whatever its
// width.  Here a level costs four dependent kernel boundaries (~1.5 us each
// on MI355X, MI355X_MICROARCH.md price table "boundary") plus the latency of
// its work.  A persistent cooperative kernel was measured slower: its grid
// barrier (cooperative_groups, software on ROCm 7.2) cost ~8 us at 64
// workgroups, four per level (6.8 ms per Model_1 check).  Enlarged models
// start and end narrow too.
//
// Per level (parents in buffer A or B, count n):
//   k_nexpand   lane i = parent i; each successor's fingerprint goes into a
//               level table in HBM (NARROW_LT 16-B entries {fp, min key},
//               L2/MALL-resident) with a CAS + atomicMin of the order key
//               (parent << 5 | t): an EXACT level-wide dedup, so the first
//               copy in sequential BFS order (the state a 1-worker TLC meets
//               first) is known without the wide path's claim protocol.
//   k_ninsert   every used entry looks its fingerprint up in the ClaimSet
//               (fpset_dev.h) and inserts it with a CAS if absent: a new
//               state.  Its claim word gets the key (later wide levels then
//               see an earlier level's state) and its parent's newmask bit is
//               set; the entry is cleared for the next level.
//   k_nemit     workgroup w publishes its popcount total of newmask (tagged
//               with the level) and adds the totals of the lower workgroups
//               as they arrive (all NARROW_WG workgroups are resident at
//               once), plus a workgroup scan; then each lane writes its
//               parent's new states in t order with parent pointer, ordinal,
//               invariant check and per-action distinct count; the successor
//               count of the next level accumulates.
//   k_nstep     one wave: level bookkeeping, and the decision for the next
//               level (stop before a level that is too wide, could overflow a
//               buffer / the level table / the ClaimSet's room, or reaches
//               stop_level; stop after a level without new states or with an
//               error).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "engine_kernels.h"
#include "fpset_dev.h"
#include "kubeapi_spec.h"

namespace kc {

constexpr int NARROW_THREADS = 256;
constexpr int NARROW_MAX = 8192;                          // parents of a narrow level
constexpr int NARROW_WG = NARROW_MAX / NARROW_THREADS;    // workgroups of the per-parent kernels
constexpr int NARROW_LT_BITS = 16;
constexpr uint64_t NARROW_LT = 1ull << NARROW_LT_BITS;   // level-table entries
constexpr uint64_t NARROW_CAND_MAX = NARROW_LT / 2;       // successors of a narrow level
constexpr int NARROW_BATCH = 16;                          // levels enqueued per host sync
static_assert((uint64_t)NARROW_MAX * 32 < (1u << 20), "a workgroup total fits PUB_TOTAL_BITS");

enum NarrowExit : int {
  NX_WIDE = 1,      // the next level is wider than NARROW_MAX
  NX_ROOM = 2,      // the next level may not fit a buffer / the level table / the ClaimSet room
  NX_STOP = 3,      // stop_level reached (max_levels, level capture)
  NX_DONE = 4,      // no new state: the check is complete
  NX_ERROR = 5,     // an assertion, deadlock or invariant error in the last level
};

// The control block (device memory; the host fills it before a run, the
// kernels keep it up to date level by level).
struct NarrowCtl {
  uint32_t active;       // 1 while the next level runs narrow
  int32_t reason;        // NarrowExit once inactive
  uint32_t level;        // BFS level about to be expanded (1 = Init)
  uint32_t cur_is_b;     // its states are in buffer B (else A)
  uint64_t n;            // its width
  uint64_t level_gidx;   // global index of its first state
  uint64_t cand;         // its successor count
  uint64_t room;         // new states the ClaimSet may still take
  uint64_t buf_cap;      // states per frontier buffer
  uint64_t par_cap;      // entries of parent[] / ord[]
  uint32_t stop_level;   // do not expand a level >= stop_level (0 = none)
  uint32_t levels;       // levels expanded in this run
  uint32_t epoch;        // this run's number (tags k_nemit's published totals)
  uint32_t pad1;
  uint64_t new_total;    // states added in this run
  uint64_t probes;       // ClaimSet lookups in this run
  uint64_t err_key;      // the error that ended the run (NX_ERROR)
  // per level (returned to 0 / ~0 by k_nstep)
  unsigned long long cand_acc;             // successors of the new states
  unsigned long long err;                  // min error key (~0 = none)
  unsigned long long wg_pub[NARROW_WG];    // k_nemit: pub_tag(epoch, level) | workgroup's new states
  uint64_t widths[KC_MAX_LEVELS];          // widths[L] = width of level L + 1
};

struct NarrowLT {
  unsigned long long fp;   // 0 = empty
  unsigned int key;        // min order key (parent << 5 | t); ~0 = none
  unsigned int pad;
};
struct NarrowScratch {
  NarrowLT lt[NARROW_LT];
  unsigned int newmask[NARROW_MAX];
};

// The rule a level is checked against before it runs narrow (the host
// before a run, k_nstep after every level).
__host__ __device__ __forceinline__ int narrow_exit_reason(const NarrowCtl& c) {
  if (c.n == 0) return NX_DONE;
  if (c.stop_level && c.level >= c.stop_level) return NX_STOP;
  if (c.n > (uint64_t)NARROW_MAX) return NX_WIDE;
  if (c.cand > c.buf_cap || c.cand > c.room || c.cand > NARROW_CAND_MAX ||
      c.level_gidx + c.n + c.cand + 1 > c.par_cap)
    return NX_ROOM;
  return 0;
}

__global__ void k_narrow_scratch_init(NarrowScratch* sc) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < NARROW_LT) {
    sc->lt[i].fp = 0;
    sc->lt[i].key = ~0u;
  }
  if (i < NARROW_MAX) sc->newmask[i] = 0;
}

// k_nemit's published workgroup totals carry (run epoch, level) above the
// total (< 2^20: at most 8192 parents x 32 successors), so a stale value of
// an earlier level or run is never mistaken for the current one.
constexpr int PUB_TOTAL_BITS = 20;
__device__ __forceinline__ unsigned long long pub_tag(uint32_t epoch, uint32_t level) {
  return (((unsigned long long)epoch << 12) | level) << PUB_TOTAL_BITS;
}

__device__ __forceinline__ uint64_t lt_slot(uint64_t fp) {
  return (fp * 0xd6e8feb86659fd93ull) >> (64 - NARROW_LT_BITS);
}

template <class M>
__global__ void __launch_bounds__(NARROW_THREADS)
k_nexpand(const typename M::State* __restrict__ bufA, const typename M::State* __restrict__ bufB, Flags f,
          int check_deadlock, NarrowCtl* __restrict__ ctl, NarrowScratch* __restrict__ sc,
          Counters* __restrict__ C) {
  using State = typename M::State;
  if (!ctl->active) return;
  __shared__ unsigned int sh_act[A_COUNT];
  if (threadIdx.x < A_COUNT) sh_act[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t n = ctl->n;
  const uint64_t i = (uint64_t)blockIdx.x * NARROW_THREADS + threadIdx.x;
  if (i < n) {
    const State* __restrict__ cur = ctl->cur_is_b ? bufB : bufA;
    const State s = load_state<M>(cur, i);
    const typename M::Plan pl = M::plan(s, f);
    if (pl.fail_pos >= 0)
      atomicMin(&ctl->err, (i << 16) | ((uint64_t)pl.fail_pos << 8) | E_ASSERT);
    else if (pl.total == 0 && check_deadlock)
      atomicMin(&ctl->err, (i << 16) | E_DEADLOCK);
#pragma unroll
    for (int slot = 0; slot < M::NSLOT; ++slot) {
      const int c = (int)((pl.counts >> (6 * slot)) & 63);
      if (c) atomicAdd(&sh_act[M::slot_action(s, slot)], (unsigned)c);
    }
    if (pl.total > M::MAXSUCC) atomicAdd(&C->overflow, 1ull);     // fails the run loudly
    const int tot = pl.total < M::MAXSUCC ? pl.total : M::MAXSUCC;
    const uint64_t fold = M::fp_fold(s);
    // successors in groups of NB: all fingerprints first, then the group's
    // CASes back to back (independent round trips in flight), then the
    // key minimums — a lane waits ~2 atomic latencies per group instead of
    // 2 per successor
    constexpr int NB = 8;
    for (int t0 = 0; t0 < tot; t0 += NB) {
      uint64_t fp[NB], h[NB];
      unsigned long long e[NB];
#pragma unroll
      for (int k = 0; k < NB; ++k) {
        fp[k] = 0;
        if (t0 + k < tot) {
          int slot, j, who;
          M::locate(pl, t0 + k, slot, j);
          State x;
          M::apply(s, slot, j, f, x, who);
          fp[k] = M::fingerprint_succ(s, fold, x, who);
        }
        h[k] = lt_slot(fp[k]);
      }
#pragma unroll
      for (int k = 0; k < NB; ++k)
        e[k] = fp[k] ? atomicCAS(&sc->lt[h[k]].fp, 0ull, (unsigned long long)fp[k]) : 0ull;
#pragma unroll
      for (int k = 0; k < NB; ++k) {
        if (!fp[k]) continue;
        // collision: probe on (rare at <= 1/2 load)
        for (uint64_t q = 0; e[k] != 0ull && e[k] != fp[k] && q < NARROW_LT; ++q) {
          h[k] = (h[k] + 1) & (NARROW_LT - 1);
          e[k] = atomicCAS(&sc->lt[h[k]].fp, 0ull, (unsigned long long)fp[k]);
        }
      }
#pragma unroll
      for (int k = 0; k < NB; ++k)
        if (fp[k]) atomicMin(&sc->lt[h[k]].key, (unsigned int)((i << 5) | (uint64_t)(t0 + k)));
    }
  }
  __syncthreads();
  if (threadIdx.x < A_COUNT && sh_act[threadIdx.x])
    atomicAdd(&stripe(C).act_gen[threadIdx.x], (unsigned long long)sh_act[threadIdx.x]);
}

__global__ void __launch_bounds__(NARROW_THREADS)
k_ninsert(NarrowCtl* __restrict__ ctl, NarrowScratch* __restrict__ sc, ClaimEntry* __restrict__ cs,
          uint64_t nslots) {
  if (!ctl->active) return;
  const uint64_t h = (uint64_t)blockIdx.x * NARROW_THREADS + threadIdx.x;
  const unsigned long long fp = sc->lt[h].fp;
  unsigned long long probes = 0;
  if (fp) {
    const unsigned int key = sc->lt[h].key;
    sc->lt[h].fp = 0ull;
    sc->lt[h].key = ~0u;
    probes = 1;
    const uint32_t succ_level = ctl->level + 1;
    uint64_t ix = bucket_of(fp, nslots);
    for (uint64_t q = 0; q < nslots; ++q) {
      const unsigned long long e = atomicCAS(&cs[ix].fp, 0ull, fp);
      if (e == 0ull) {                           // inserted: a new state of the level
        cs[ix].nclaim = ~make_claim(succ_level, ((uint64_t)(key >> 5) << 8) | (key & 31));
        atomicOr(&sc->newmask[key >> 5], 1u << (key & 31));
        break;
      }
      if (e == fp) break;                         // seen in an earlier level
      ix = (ix + 1 == nslots) ? 0 : ix + 1;
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) probes += __shfl_down(probes, off, 64);
  if ((threadIdx.x & 63) == 0 && probes) atomicAdd((unsigned long long*)&ctl->probes, probes);
}

template <class M>
__global__ void __launch_bounds__(NARROW_THREADS)
k_nemit(typename M::State* __restrict__ bufA, typename M::State* __restrict__ bufB, Flags f,
        unsigned long long* __restrict__ parent, uint8_t* __restrict__ ord, int keep_trace,
        NarrowCtl* __restrict__ ctl, NarrowScratch* __restrict__ sc, Counters* __restrict__ C) {
  using State = typename M::State;
  if (!ctl->active) return;
  __shared__ unsigned int sh_dist[A_COUNT];
  __shared__ unsigned int sh_deg[OUTDEG_BINS];
  __shared__ unsigned int sh_w[4];
  __shared__ unsigned int sh_base;
  __shared__ unsigned long long sh_cand;
  if (threadIdx.x < A_COUNT) sh_dist[threadIdx.x] = 0;
  if (threadIdx.x < OUTDEG_BINS) sh_deg[threadIdx.x] = 0;
  if (threadIdx.x == 0) sh_cand = 0;
  const uint64_t n = ctl->n, level_gidx = ctl->level_gidx;
  const unsigned long long tag = pub_tag(ctl->epoch, ctl->level);
  const uint64_t i = (uint64_t)blockIdx.x * NARROW_THREADS + threadIdx.x;
  uint32_t m = i < n ? sc->newmask[i] : 0u;
  const int cnt = __builtin_popcount(m);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int incl = cnt;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int v = __shfl_up(incl, off, 64);
    if (lane >= off) incl += v;
  }
  if (lane == 63) sh_w[wv] = (unsigned int)incl;
  __syncthreads();
  if (i < n) atomicAdd(&sh_deg[cnt < OUTDEG_BINS ? cnt : OUTDEG_BINS - 1], 1u);
  // publish this workgroup's total tagged with the level (no reset needed),
  // then take the totals of the lower workgroups as they arrive: all
  // NARROW_WG workgroups fit the chip at once, so every one is running
  const unsigned int wtot = sh_w[0] + sh_w[1] + sh_w[2] + sh_w[3];
  if (threadIdx.x == 0)
    __hip_atomic_store(&ctl->wg_pub[blockIdx.x], tag | wtot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  unsigned int base = 0;
  if (wv == 0) {
    unsigned int v = 0;
    if (lane < (int)blockIdx.x) {
      unsigned long long p;
      while (((p = __hip_atomic_load(&ctl->wg_pub[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >>
              PUB_TOTAL_BITS) != (tag >> PUB_TOTAL_BITS))
        __builtin_amdgcn_s_sleep(1);
      v = (unsigned int)(p & ((1ull << PUB_TOTAL_BITS) - 1));
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    if (lane == 0) sh_base = v;
  }
  __syncthreads();
  base = sh_base;
  for (int w = 0; w < wv; ++w) base += sh_w[w];
  uint64_t o = base + (unsigned int)(incl - cnt);
  unsigned long long cnd = 0;
  if (m) {
    sc->newmask[i] = 0;
    const State* __restrict__ cur = ctl->cur_is_b ? bufB : bufA;
    State* __restrict__ nxt = ctl->cur_is_b ? bufA : bufB;
    const uint64_t next_gidx = level_gidx + n;
    const State s = load_state<M>(cur, i);
    const typename M::Plan pl = M::plan(s, f);
    for (; m; m &= m - 1) {
      const int t = __ffs(m) - 1;
      int slot, j;
      M::locate(pl, t, slot, j);
      State x;
      M::apply(s, slot, j, f, x);
      store_state<M>(nxt, o, x);
      if (keep_trace) {
        parent[next_gidx + o] = level_gidx + i;
        ord[next_gidx + o] = (uint8_t)t;
      }
      if (M::check(x, f.inv_mask) >= 0) atomicMin(&ctl->err, (i << 16) | ((uint64_t)t << 8) | E_INVARIANT);
      atomicAdd(&sh_dist[M::slot_action(s, slot)], 1u);
      cnd += (unsigned long long)M::plan(x, f).total;
      ++o;
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) cnd += __shfl_down(cnd, off, 64);
  if (lane == 0 && cnd) atomicAdd(&sh_cand, cnd);
  __syncthreads();
  if (threadIdx.x < A_COUNT && sh_dist[threadIdx.x])
    atomicAdd(&stripe(C).act_dist[threadIdx.x], (unsigned long long)sh_dist[threadIdx.x]);
  if (threadIdx.x < OUTDEG_BINS && sh_deg[threadIdx.x])
    atomicAdd(&stripe(C).outdeg[threadIdx.x], (unsigned long long)sh_deg[threadIdx.x]);
  if (threadIdx.x == 0 && sh_cand) atomicAdd(&ctl->cand_acc, sh_cand);
}

// One wave: close the level and decide about the next one.
__global__ void __launch_bounds__(64) k_nstep(NarrowCtl* __restrict__ ctl, Counters* __restrict__ C) {
  if (!ctl->active) return;
  unsigned long long v = threadIdx.x < NARROW_WG ? (ctl->wg_pub[threadIdx.x] & ((1ull << PUB_TOTAL_BITS) - 1)) : 0;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  if (threadIdx.x != 0) return;
  NarrowCtl& c = *ctl;
  const uint64_t total = v;
  const unsigned long long err = c.err, cnext = c.cand_acc;
  c.err = ~0ull;
  c.cand_acc = 0;
  ++c.levels;
  c.new_total += total;
  c.room = c.room > total ? c.room - total : 0;
  if (err != ~0ull) {                    // the level stays the current one
    c.err_key = err;
    C->err_key = err;
    c.reason = NX_ERROR;
    c.active = 0;
    return;
  }
  if (c.level < KC_MAX_LEVELS) c.widths[c.level] = total;
  c.level_gidx += c.n;
  c.n = total;
  c.cand = cnext;
  c.level += 1;
  c.cur_is_b ^= 1u;
  const int r = narrow_exit_reason(c);
  if (r) {
    c.reason = r;
    c.active = 0;
  }
}

}  // namespace kc
