// engine_narrow.h — device-driven narrow BFS levels (gfx950).
//
// While the frontier is small (<= NARROW_MAX parents) a level is run by two
// short kernels that read the level's size and buffers from a control block
// in device memory (NarrowCtl) instead of from the host; the host enqueues
// NARROW_BATCH levels' worth of them back to back and synchronises once per
// batch.  Each kernel returns at once when the control block is inactive,
// so the launches after the level that ended the narrow run are nearly free.
//
// Why: the reference's own model (Model_1, MC.cfg) is deep and narrow: 124
// levels, at most 3,939 states wide.  On the wide-level path
// every level costs ~6 launches AND a host round trip (~70 us) whatever its
// width.  Here a level costs two dependent kernel boundaries (~1.5 us each
// on MI355X, MI355X_MICROARCH.md price table "boundary") plus the latency of
// its work.  A persistent cooperative kernel was measured slower: its grid
// barrier (cooperative_groups, software on ROCm 7.2) cost ~8 us at 64
// workgroups, four per level (6.8 ms per Model_1 check).  Enlarged models
// start and end narrow too.  A narrow level has at most one wave per SIMD,
// so its time is the serial chain of one lane: several lanes share a parent
// (NARROW_SUB, NARROW_ESUB) and split its successors.
//
// Per level L (parents in buffer A or B, count n; level tables T[0], T[1]):
//   k_nexpand   lanes (parent i, k): successors t = k, k + NARROW_SUB, ...;
//               each fingerprint goes into T[L & 1] (NARROW_LT 16-B entries
//               {fp, ~min key}, L2/MALL-resident) with a CAS + atomicMax of
//               the complemented order key (parent << 5 | t): an EXACT
//               level-wide dedup, so the first copy in sequential BFS order
//               (the state a 1-worker TLC meets first) is known without the
//               wide path's claim protocol.
//   k_nfinish   lanes (parent i, k): re-derive successors t = k, k +
//               NARROW_ESUB, ...; a successor whose key is its entry's
//               minimum inserts its fingerprint into the ClaimSet
//               (fpset_dev.h; CAS, with the claim word for later wide
//               levels): a new state unless an earlier level stored it.
//               The parent's new-state mask is OR-ed over its lanes;
//               workgroup w publishes its popcount total (tagged with run
//               epoch and level) and adds the totals of the lower workgroups
//               as they arrive (all NARROW_FWG workgroups are resident at
//               once), plus a workgroup scan; then the lanes write the
//               parent's new states in t order with parent pointer,
//               ordinal, invariant check and per-action distinct count; the
//               next level's successor count accumulates; T[(L + 1) & 1]
//               (last read by level L - 1) is cleared for level L + 1.
//   (close)     the last k_nfinish workgroup to finish, one wave: level
//               bookkeeping, and the decision for the next level (stop
//               before a level that is too wide, could overflow a buffer /
//               the level table / the ClaimSet's room, or reaches
//               stop_level; stop after a level without new states or with
//               an error).
// (Round-2 history: four kernels per level — expand, a level-table sweep
// inserting into the ClaimSet, emit, a one-wave step kernel — 44 us a
// level on Model_1; the sweep and the step are folded into k_nfinish.)
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
// k_nexpand lanes per parent: a narrow level has few waves (<= 1 per SIMD),
// so its time is one lane's serial successor chain; NARROW_SUB lanes share a
// parent, lane k taking successors k, k + NARROW_SUB, ...
constexpr int NARROW_SUB = 8;
// k_nfinish lanes per parent, and its workgroups (all resident at once)
constexpr int NARROW_ESUB = 4;
constexpr int NARROW_FWG = NARROW_MAX * NARROW_ESUB / NARROW_THREADS;
static_assert(NARROW_FWG <= 128, "the closing wave sums two published totals per lane");
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
  uint32_t epoch;        // this run's number (tags k_nfinish's published totals)
  uint32_t pad1;
  uint64_t new_total;    // states added in this run
  uint64_t probes;       // ClaimSet lookups in this run
  uint64_t err_key;      // the error that ended the run (NX_ERROR)
  // per level (returned to 0 / ~0 when the level closes)
  unsigned long long close_acc;            // k_nfinish workgroups done << 56 | new states << 28 | their successors
  unsigned long long err;                  // min error key (~0 = none)
  unsigned long long wg_pub[NARROW_FWG];   // k_nfinish: pub_tag(epoch, level) | workgroup's new states
  uint64_t widths[KC_MAX_LEVELS];          // widths[L] = width of level L + 1
};

struct NarrowLT {
  unsigned long long fp;   // 0 = empty
  unsigned int nkey;       // ~(min order key (parent << 5 | t)); 0 = none
  unsigned int pad;
};
// two level tables, by level parity; all-zero = clear (hipMemset)
struct NarrowScratch {
  NarrowLT lt[2][NARROW_LT];
};

// The rule a level is checked against before it runs narrow (the host
// before a run, the closing wave after every level).
__host__ __device__ __forceinline__ int narrow_exit_reason(const NarrowCtl& c) {
  if (c.n == 0) return NX_DONE;
  if (c.stop_level && c.level >= c.stop_level) return NX_STOP;
  if (c.n > (uint64_t)NARROW_MAX) return NX_WIDE;
  if (c.cand > c.buf_cap || c.cand > c.room || c.cand > NARROW_CAND_MAX ||
      c.level_gidx + c.n + c.cand + 1 > c.par_cap)
    return NX_ROOM;
  return 0;
}

// k_nfinish's published workgroup totals carry (run epoch, level) above the
// total (< 2^20: at most 8192 parents x 32 successors), so a stale value of
// an earlier level or run is never mistaken for the current one.
constexpr int PUB_TOTAL_BITS = 20;
__device__ __forceinline__ unsigned long long pub_tag(uint32_t epoch, uint32_t level) {
  return (((unsigned long long)epoch << 12) | level) << PUB_TOTAL_BITS;
}

// Phase timestamps (diagnostic: KC_NARROW_TRACE=1; ntrace == nullptr
// otherwise): thread 0 of every workgroup, wall clock (100 MHz), per launch.
constexpr int NTRACE_PH = 8;
constexpr uint64_t NTRACE_LEVELS = 1024;
constexpr uint64_t NTRACE_FOFF = NTRACE_LEVELS * NARROW_WG * NARROW_SUB * NTRACE_PH;
#define NTRACE_X(ph)                                                                                  \
  do {                                                                                                \
    if (ntrace && threadIdx.x == 0 && lev < NTRACE_LEVELS)                                            \
      ntrace[((uint64_t)lev * gridDim.x + blockIdx.x) * NTRACE_PH + (ph)] = wall_clock64();         \
  } while (0)
#define NTRACE_F(ph)                                                                                  \
  do {                                                                                                \
    if (ntrace && threadIdx.x == 0 && lev < NTRACE_LEVELS)                                            \
      ntrace[NTRACE_FOFF + ((uint64_t)lev * gridDim.x + blockIdx.x) * NTRACE_PH + (ph)] = wall_clock64(); \
  } while (0)

__device__ __forceinline__ uint64_t lt_slot(uint64_t fp) {
  return (fp * 0xd6e8feb86659fd93ull) >> (64 - NARROW_LT_BITS);
}

// grid: NARROW_WG * NARROW_SUB workgroups; lane g = parent g / NARROW_SUB,
// successors t = g % NARROW_SUB (+ NARROW_SUB ...)
template <class M>
__global__ void __launch_bounds__(NARROW_THREADS)
k_nexpand(const typename M::State* __restrict__ bufA, const typename M::State* __restrict__ bufB, Flags f,
          int check_deadlock, uint32_t lev, NarrowCtl* __restrict__ ctl, NarrowScratch* __restrict__ sc,
          Counters* __restrict__ C, unsigned long long* __restrict__ ntrace) {
  using State = typename M::State;
  // `lev`: the launch's level within the run, so the buffer and level table
  // are known without the control block; the parent load (any i < NARROW_MAX
  // is inside the buffer) and the control fields are one round trip
  const uint64_t g = (uint64_t)blockIdx.x * NARROW_THREADS + threadIdx.x;
  const uint64_t i = g / NARROW_SUB;
  const int sub = (int)(g % NARROW_SUB);
  const State* __restrict__ cur = (lev & 1) ? bufB : bufA;
  NTRACE_X(0);
  const State s = load_state<M>(cur, i);
  const uint32_t active = ctl->active;
  const uint64_t n = ctl->n;
  if (!active) return;
  NTRACE_X(1);
  __shared__ unsigned int sh_act[A_COUNT];
  if (threadIdx.x < A_COUNT) sh_act[threadIdx.x] = 0;
  __syncthreads();
  NarrowLT* __restrict__ lt = sc->lt[lev & 1];
  if (i < n) {
    const typename M::Plan pl = M::plan(s, f);
    if (sub == 0) {
      if (pl.fail_pos >= 0)
        atomicMin(&ctl->err, (i << 16) | ((uint64_t)pl.fail_pos << 8) | E_ASSERT);
      else if (pl.total == 0 && check_deadlock)
        atomicMin(&ctl->err, (i << 16) | E_DEADLOCK);
#pragma unroll
      for (int slot = 0; slot < M::NSLOT; ++slot) {
        const int c = (int)((pl.counts >> (6 * slot)) & 63);
        if (c) atomicAdd(&sh_act[M::slot_action(s, slot)], (unsigned)c);
      }
      if (pl.total > M::MAXSUCC) atomicAdd(&C->overflow, 1ull);   // fails the run loudly
    }
    const int tot = pl.total < M::MAXSUCC ? pl.total : M::MAXSUCC;
    const uint64_t fold = M::fp_fold(s);
    for (int t = sub; t < tot; t += NARROW_SUB) {
      int slot, j, who;
      M::locate(pl, t, slot, j);
      State x;
      M::apply(s, slot, j, f, x, who);
      const uint64_t fp = M::fingerprint_succ(s, fold, x, who);
      uint64_t h = lt_slot(fp);
      unsigned long long e = atomicCAS(&lt[h].fp, 0ull, (unsigned long long)fp);
      // collision: probe on (rare at <= 1/2 load)
      for (uint64_t q = 0; e != 0ull && e != fp && q < NARROW_LT; ++q) {
        h = (h + 1) & (NARROW_LT - 1);
        e = atomicCAS(&lt[h].fp, 0ull, (unsigned long long)fp);
      }
      atomicMax(&lt[h].nkey, ~(unsigned int)((i << 5) | (uint64_t)t));
    }
  }
  NTRACE_X(2);
  __syncthreads();
  NTRACE_X(3);
  if (threadIdx.x < A_COUNT && sh_act[threadIdx.x])
    atomicAdd(&stripe(C).act_gen[threadIdx.x], (unsigned long long)sh_act[threadIdx.x]);
}

__device__ __forceinline__ void narrow_step(NarrowCtl* __restrict__ ctl, Counters* __restrict__ C, uint64_t total,
                                            unsigned long long cnext);

template <class M>
__global__ void __launch_bounds__(NARROW_THREADS)
k_nfinish(typename M::State* __restrict__ bufA, typename M::State* __restrict__ bufB, Flags f,
          unsigned long long* __restrict__ parent, uint8_t* __restrict__ ord, int keep_trace,
          uint32_t lev, NarrowCtl* __restrict__ ctl, NarrowScratch* __restrict__ sc, ClaimEntry* __restrict__ cs,
          uint64_t nslots, Counters* __restrict__ C, unsigned long long* __restrict__ ntrace) {
  using State = typename M::State;
  const uint64_t g = (uint64_t)blockIdx.x * NARROW_THREADS + threadIdx.x;
  const uint64_t i = g / NARROW_ESUB;
  const int sub = (int)(g % NARROW_ESUB);
  const State* __restrict__ cur = (lev & 1) ? bufB : bufA;
  NTRACE_F(0);
  State s = load_state<M>(cur, i);                 // (i < NARROW_MAX: inside the buffer)
  const uint32_t active = ctl->active, level = ctl->level, epoch = ctl->epoch;
  const uint64_t n = ctl->n, level_gidx = ctl->level_gidx;
  if (!active) return;
  NTRACE_F(1);
  __shared__ unsigned int sh_dist[A_COUNT];
  __shared__ unsigned int sh_deg[OUTDEG_BINS];
  __shared__ unsigned int sh_w[4];
  __shared__ unsigned int sh_base;
  __shared__ unsigned long long sh_cand;
  if (threadIdx.x < A_COUNT) sh_dist[threadIdx.x] = 0;
  if (threadIdx.x < OUTDEG_BINS) sh_deg[threadIdx.x] = 0;
  if (threadIdx.x == 0) sh_cand = 0;
  const NarrowLT* __restrict__ lt = sc->lt[lev & 1];
  const unsigned long long tag = pub_tag(epoch, level);
  const bool live = i < n;
  typename M::Plan pl{};
  uint32_t mine = 0;
  unsigned long long probes = 0;
  if (live) {
    pl = M::plan(s, f);
    const int tot = pl.total < M::MAXSUCC ? pl.total : M::MAXSUCC;
    const uint64_t fold = M::fp_fold(s);
    const uint32_t succ_level = level + 1;
    for (int t = sub; t < tot; t += NARROW_ESUB) {
      int slot, j, who;
      M::locate(pl, t, slot, j);
      State x;
      M::apply(s, slot, j, f, x, who);
      const uint64_t fp = M::fingerprint_succ(s, fold, x, who);
      // its level-table entry (k_nexpand entered every successor)
      uint64_t h = lt_slot(fp);
      ulonglong2 e = *reinterpret_cast<const ulonglong2*>(&lt[h]);
      for (uint64_t q = 0; e.x != fp && e.x != 0ull && q < NARROW_LT; ++q) {
        h = (h + 1) & (NARROW_LT - 1);
        e = *reinterpret_cast<const ulonglong2*>(&lt[h]);
      }
      if (e.x != fp) {
        atomicAdd(&C->overflow, 1ull);          // cannot happen: fail the run loudly
        continue;
      }
      const unsigned int key = (unsigned int)((i << 5) | (uint64_t)t);
      if ((unsigned int)~(unsigned int)e.y != key) continue;    // an earlier copy of the level holds it
      // the level's first copy: into the ClaimSet, new unless an earlier level stored it
      ++probes;
      uint64_t ix = bucket_of(fp, nslots);
      for (uint64_t q = 0; q < nslots; ++q) {
        const unsigned long long o = atomicCAS(&cs[ix].fp, 0ull, fp);
        if (o == 0ull) {
          cs[ix].nclaim = ~make_claim(succ_level, (i << 8) | (uint64_t)t);
          mine |= 1u << t;
          break;
        }
        if (o == fp) break;
        ix = (ix + 1 == nslots) ? 0 : ix + 1;
      }
    }
  }
  NTRACE_F(2);
  // the parent's new-state mask, over its NARROW_ESUB adjacent lanes
  uint32_t m = mine;
#pragma unroll
  for (int off = 1; off < NARROW_ESUB; off <<= 1) m |= (uint32_t)__shfl_xor((int)m, off, 64);
  const int cnt = (live && sub == 0) ? __builtin_popcount(m) : 0;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int incl = cnt;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int v = __shfl_up(incl, off, 64);
    if (lane >= off) incl += v;
  }
  if (lane == 63) sh_w[wv] = (unsigned int)incl;
  __syncthreads();
  NTRACE_F(3);
  if (live && sub == 0) atomicAdd(&sh_deg[cnt < OUTDEG_BINS ? cnt : OUTDEG_BINS - 1], 1u);
  // publish this workgroup's total tagged with (run, level), no reset needed;
  // then take the totals of the lower workgroups as they arrive
  const unsigned int wtot = sh_w[0] + sh_w[1] + sh_w[2] + sh_w[3];
  if (threadIdx.x == 0)
    __hip_atomic_store(&ctl->wg_pub[blockIdx.x], tag | wtot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (wv == 0) {
    unsigned int v = 0;
    for (int w = lane; w < (int)blockIdx.x; w += 64) {
      unsigned long long p;
      while (((p = __hip_atomic_load(&ctl->wg_pub[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >>
              PUB_TOTAL_BITS) != (tag >> PUB_TOTAL_BITS))
        __builtin_amdgcn_s_sleep(1);
      v += (unsigned int)(p & ((1ull << PUB_TOTAL_BITS) - 1));
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    if (lane == 0) sh_base = v;
  }
  __syncthreads();
  NTRACE_F(4);
  unsigned int base = sh_base;
  for (int w = 0; w < wv; ++w) base += sh_w[w];
  // the parent's first output slot: its sub-0 lane's exclusive prefix
  const int excl0 = __shfl(incl - cnt, lane & ~(NARROW_ESUB - 1), 64);
  unsigned long long cnd = 0;
  if (live && m) {
    State* __restrict__ nxt = (lev & 1) ? bufA : bufB;
    const uint64_t next_gidx = level_gidx + n;
    uint64_t o = (uint64_t)base + (unsigned int)excl0;
    int k = 0;
    for (uint32_t mm = m; mm; mm &= mm - 1, ++k, ++o) {
      if ((k % NARROW_ESUB) != sub) continue;
      const int t = __ffs(mm) - 1;
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
    }
  }
  // clear the other level table for level L + 1 (level L - 1 read it)
  {
    NarrowLT* __restrict__ other = sc->lt[(lev + 1) & 1];
    for (uint64_t h = g; h < NARROW_LT; h += (uint64_t)NARROW_FWG * NARROW_THREADS)
      *reinterpret_cast<ulonglong2*>(&other[h]) = make_ulonglong2(0ull, 0ull);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    cnd += __shfl_down(cnd, off, 64);
    probes += __shfl_down(probes, off, 64);
  }
  if (lane == 0 && cnd) atomicAdd(&sh_cand, cnd);
  if (lane == 0 && probes) atomicAdd((unsigned long long*)&ctl->probes, probes);
  __syncthreads();
  NTRACE_F(5);
  if (threadIdx.x < A_COUNT && sh_dist[threadIdx.x])
    atomicAdd(&stripe(C).act_dist[threadIdx.x], (unsigned long long)sh_dist[threadIdx.x]);
  if (threadIdx.x < OUTDEG_BINS && sh_deg[threadIdx.x])
    atomicAdd(&stripe(C).outdeg[threadIdx.x], (unsigned long long)sh_deg[threadIdx.x]);
  // The last workgroup to get here closes the level.  Its inputs are all
  // device-scope atomics: every wave waits for its own to complete (an
  // s_waitcnt on all counters; no L2 write-back needed), then one returning
  // add carries this workgroup's new-state and successor totals with the
  // arrival count, so the last arriver has the level's totals at once and
  // reads only the error key.
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  NTRACE_F(6);
  if (threadIdx.x == 0) {
    const unsigned long long mine_acc = (1ull << 56) | ((unsigned long long)wtot << 28) | sh_cand;
    const unsigned long long prev = atomicAdd(&ctl->close_acc, mine_acc);
    if ((prev >> 56) == NARROW_FWG - 1) {
      const unsigned long long all = prev + mine_acc;
      narrow_step(ctl, C, (all >> 28) & ((1ull << 28) - 1), all & ((1ull << 28) - 1));
      NTRACE_F(7);
    }
  }
}

// One thread (of the last k_nfinish workgroup to finish): close the level
// (its `total` new states with `cnext` successors) and decide about the next.
__device__ __forceinline__ void narrow_step(NarrowCtl* __restrict__ ctl, Counters* __restrict__ C, uint64_t total,
                                            unsigned long long cnext) {
  NarrowCtl& c = *ctl;
  const unsigned long long err = __hip_atomic_load(&c.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  c.close_acc = 0;
  c.err = ~0ull;
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
