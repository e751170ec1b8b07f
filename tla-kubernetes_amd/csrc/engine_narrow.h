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
// levels enqueued per host sync (Model_1, same box: 8 -> 3.20 ms, 16 -> 3.00,
// 32 -> 2.90; round 5, same box twice: 32 -> 2.91 / 3.21, 64 -> 2.83 / 2.84,
// 128 -> 2.85 / 2.80, profiles/r05ab_narrow_batch.txt; KC_NARROW_BATCH
// overrides it).  The launches enqueued past a run's end return at once.
constexpr int NARROW_BATCH = 64;
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
  // by level parity: [L & 1] = level L's min error key (~0 = none): its
  // parents' assertion / deadlock errors (found when they were emitted, by
  // the previous level's k_nfinish, or by k_nexpand) and its successors'
  // invariant errors
  unsigned long long err[2];
  unsigned int act_next[2][A_COUNT];       // level L's per-action successor counts, committed when L runs
  unsigned int lt_over[2];                 // level L's table overflowed: it cannot run narrow
  unsigned long long wg_pub[NARROW_FWG];   // k_nfinish: pub_tag(epoch, level) | workgroup's new states
  uint64_t widths[KC_MAX_LEVELS];          // widths[L] = width of level L + 1
};

struct NarrowLT {
  unsigned long long fp;   // 0 = empty
  unsigned int nkey;       // ~(min order key (parent << 5 | t)); 0 = none
  unsigned int pad;
};
// three level tables, by level mod 3: k_nfinish of level L reads T[L],
// fills T[L + 1] with the successors of the states it emits, and clears
// T[L + 2] (last read by level L - 1); all-zero = clear (hipMemset)
constexpr int NARROW_NLT = 3;
constexpr int NARROW_LT_PROBES = 256;        // a longer probe run = table overflow (the level goes wide)
struct NarrowScratch {
  NarrowLT lt[NARROW_NLT][NARROW_LT];
  // by level parity, for every state of a level (written when it was
  // expanded into the table): its plan's slot counts and successor total,
  // and the table slot of each successor, so k_nfinish finds its entries
  // without re-deriving anything
  unsigned long long pcnt[2][NARROW_MAX];
  unsigned char ptot[2][NARROW_MAX];
  unsigned short hidx[2][NARROW_MAX * 32];
};
static_assert(NARROW_LT <= 65536, "table slots fit hidx");

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
constexpr int NTRACE_PH = 12;
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

// Enter up to NB successors (fingerprint fp[k] != 0, order key key[k]) of
// one lane into a level table: the CASes back to back (independent round
// trips in flight), linear probing on for the few that collide, then the
// key minimums (kept as ~max).  False if a probe run passed
// NARROW_LT_PROBES (the table is too full for this level).
template <int NB>
__device__ __forceinline__ bool lt_enter(NarrowLT* __restrict__ lt, const uint64_t (&fp)[NB],
                                         const unsigned int (&key)[NB], uint64_t (&h)[NB]) {
  unsigned long long e[NB];
  bool ok = true;
#pragma unroll
  for (int k = 0; k < NB; ++k) {
    h[k] = lt_slot(fp[k]);
    e[k] = fp[k] ? atomicCAS(&lt[h[k]].fp, 0ull, (unsigned long long)fp[k]) : 0ull;
  }
#pragma unroll
  for (int k = 0; k < NB; ++k) {
    for (int q = 0; fp[k] && e[k] != 0ull && e[k] != fp[k]; ++q) {
      if (q >= NARROW_LT_PROBES) {
        ok = false;
        break;
      }
      h[k] = (h[k] + 1) & (NARROW_LT - 1);
      e[k] = atomicCAS(&lt[h[k]].fp, 0ull, (unsigned long long)fp[k]);
    }
  }
#pragma unroll
  for (int k = 0; k < NB; ++k)
    if (fp[k] && (e[k] == 0ull || e[k] == fp[k])) atomicMax(&lt[h[k]].nkey, ~key[k]);
  return ok;
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
  NarrowLT* __restrict__ lt = sc->lt[lev % NARROW_NLT];
  if (i < n) {
    const typename M::Plan pl = M::plan(s, f);
    if (sub == 0) {
      sc->pcnt[lev & 1][i] = pl.counts;
      sc->ptot[lev & 1][i] = (unsigned char)(pl.total < M::MAXSUCC ? pl.total : M::MAXSUCC);
      if (pl.fail_pos >= 0)
        atomicMin(&ctl->err[lev & 1], (i << 16) | ((uint64_t)pl.fail_pos << 8) | E_ASSERT);
      else if (pl.total == 0 && check_deadlock)
        atomicMin(&ctl->err[lev & 1], (i << 16) | E_DEADLOCK);
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
      const uint64_t fp[1] = {M::fingerprint_succ(s, fold, x, who)};
      const unsigned int key[1] = {(unsigned int)((i << 5) | (uint64_t)t)};
      // (the host admitted this level at <= 1/2 table load: a probe run this
      // long cannot happen; fail the run loudly if it does)
      uint64_t h[1];
      if (!lt_enter<1>(lt, fp, key, h)) atomicAdd(&C->overflow, 1ull);
      sc->hidx[lev & 1][i * 32 + t] = (unsigned short)h[0];
    }
  }
  NTRACE_X(2);
  __syncthreads();
  NTRACE_X(3);
  if (threadIdx.x < A_COUNT && sh_act[threadIdx.x])
    atomicAdd(&stripe(C).act_gen[threadIdx.x], (unsigned long long)sh_act[threadIdx.x]);
}

__device__ __forceinline__ void narrow_step(NarrowCtl* __restrict__ ctl, Counters* __restrict__ C, uint64_t total,
                                            unsigned long long cnext, uint32_t lev);

// k_nfinish stages up to NX_LDS emitted states per workgroup for the next
// level's expansion; past that a lane enters its state's successors itself
constexpr int NX_LDS = 256;
template <class M>
__device__ __forceinline__ bool lt_enter_succ(NarrowLT* __restrict__ lt, unsigned short* __restrict__ hx,
                                              const typename M::State& x, const typename M::Plan& px, int tx,
                                              unsigned int o, Flags f) {
  bool ok = true;
  const uint64_t foldx = M::fp_fold(x);
  constexpr int NB = 8;
  for (int t0 = 0; t0 < tx; t0 += NB) {
    uint64_t fpx[NB];
    unsigned int kx[NB];
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      fpx[q] = 0;
      kx[q] = (o << 5) | (unsigned int)(t0 + q);
      if (t0 + q < tx) {
        int sl, j, who;
        M::locate(px, t0 + q, sl, j);
        typename M::State y;
        M::apply(x, sl, j, f, y, who);
        fpx[q] = M::fingerprint_succ(x, foldx, y, who);
      }
    }
    uint64_t h[NB];
    ok &= lt_enter<NB>(lt, fpx, kx, h);
#pragma unroll
    for (int q = 0; q < NB; ++q)
      if (t0 + q < tx && o < (unsigned int)NARROW_MAX) hx[o * 32 + t0 + q] = (unsigned short)h[q];
  }
  return ok;
}

template <class M>
__global__ void __launch_bounds__(NARROW_THREADS)
k_nfinish(typename M::State* __restrict__ bufA, typename M::State* __restrict__ bufB, Flags f,
          int check_deadlock, unsigned long long* __restrict__ parent, uint8_t* __restrict__ ord, int keep_trace,
          uint32_t lev, NarrowCtl* __restrict__ ctl, NarrowScratch* __restrict__ sc, ClaimEntry* __restrict__ cs,
          uint64_t nslots, Counters* __restrict__ C, unsigned long long* __restrict__ ntrace, uint32_t csh = 1) {
  // (csh: slot i's fp word is word i << csh — 1 for 16-B ClaimEntry slots,
  // 0 for the compact set of the first-claim mode, which has no claim words)
  unsigned long long* const csw = reinterpret_cast<unsigned long long*>(cs);
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
  __shared__ unsigned int sh_actn[A_COUNT];
  // emitted states staged for the expansion of level L + 1
  __shared__ State sh_xs[NX_LDS];
  __shared__ unsigned long long sh_xc[NX_LDS];
  __shared__ unsigned long long sh_xf[NX_LDS];   // fp_fold of each staged state (its tasks share it)
  __shared__ unsigned int sh_xo[NX_LDS], sh_xt[NX_LDS], sh_xoff[NX_LDS];
  __shared__ unsigned int sh_nx, sh_ntask, sh_last;
  __shared__ State sh_ps[NARROW_THREADS / NARROW_ESUB];
  __shared__ unsigned long long sh_pc[NARROW_THREADS / NARROW_ESUB];
  __shared__ unsigned int sh_pm[NARROW_THREADS / NARROW_ESUB], sh_pincl[NARROW_THREADS / NARROW_ESUB];
  __shared__ unsigned long long sh_all;
  if (threadIdx.x == 0) sh_nx = 0;
  if (threadIdx.x < A_COUNT) sh_actn[threadIdx.x] = 0;
  if (threadIdx.x < A_COUNT) sh_dist[threadIdx.x] = 0;
  if (threadIdx.x < OUTDEG_BINS) sh_deg[threadIdx.x] = 0;
  if (threadIdx.x == 0) sh_cand = 0;
  // clear level L + 2's table (level L - 1 read it; the stores overlap the loads below)
  {
    NarrowLT* __restrict__ other = sc->lt[(lev + 2) % NARROW_NLT];
    for (uint64_t h = g; h < NARROW_LT; h += (uint64_t)NARROW_FWG * NARROW_THREADS)
      *reinterpret_cast<ulonglong2*>(&other[h]) = make_ulonglong2(0ull, 0ull);
  }
  const NarrowLT* __restrict__ lt = sc->lt[lev % NARROW_NLT];
  NarrowLT* __restrict__ lt_next = sc->lt[(lev + 1) % NARROW_NLT];
  const unsigned int pq = lev & 1, qq = pq ^ 1u;      // this level's / the next level's slots
  const unsigned long long tag = pub_tag(epoch, level);
  const bool live = i < n;
  typename M::Plan pl{};
  uint32_t mine = 0;
  unsigned long long probes = 0;
  if (live) {
    // the plan and the table slots were stored when this level was expanded
    pl.counts = sc->pcnt[lev & 1][i];
    const int tot = sc->ptot[lev & 1][i];
    const unsigned short* __restrict__ hx = &sc->hidx[lev & 1][i * 32];
    const uint32_t succ_level = level + 1;
    constexpr int PT = 32 / NARROW_ESUB;            // successors per lane, at most
    unsigned int hs[PT];
#pragma unroll
    for (int k = 0; k < PT; ++k) hs[k] = sub + k * NARROW_ESUB < tot ? hx[sub + k * NARROW_ESUB] : 0u;
    ulonglong2 e[PT];
#pragma unroll
    for (int k = 0; k < PT; ++k)
      e[k] = sub + k * NARROW_ESUB < tot ? *reinterpret_cast<const ulonglong2*>(&lt[hs[k]]) : make_ulonglong2(0, 0);
    // the level's first copies go into the ClaimSet (new unless an earlier
    // level stored them): every first CAS issued back to back, so a lane's
    // round trips overlap instead of running one after another; linear
    // probing then goes on for the few whose slot held another fingerprint
    uint64_t ixs[PT];
    unsigned long long os[PT];
#pragma unroll
    for (int k = 0; k < PT; ++k) {
      const int t = sub + k * NARROW_ESUB;
      const unsigned int key = (unsigned int)((i << 5) | (uint64_t)t);
      // (an earlier copy of the level holds the entry: not this lane's)
      const bool first = t < tot && (unsigned int)~(unsigned int)e[k].y == key;
      e[k].x = first ? e[k].x : 0ull;
      ixs[k] = first ? (csh ? bucket_of(e[k].x, nslots) : fpslots_home(e[k].x, nslots)) : 0ull;
      os[k] = first ? atomicCAS(&csw[ixs[k] << csh], 0ull, e[k].x) : 0ull;
    }
#pragma unroll
    for (int k = 0; k < PT; ++k) {
      const uint64_t fp = e[k].x;
      if (!fp) continue;
      const int t = sub + k * NARROW_ESUB;
      ++probes;
      uint64_t ix = ixs[k];
      unsigned long long o = os[k];
      for (uint64_t q = 1; o != 0ull && o != fp && q < nslots; ++q) {
        ix = (ix + 1 == nslots) ? 0 : ix + 1;
        o = atomicCAS(&csw[ix << csh], 0ull, fp);
      }
      if (o == 0ull) {
        if (csh) csw[(ix << 1) + 1] = ~make_claim(succ_level, (i << 8) | (uint64_t)t);
        mine |= 1u << t;
      } else if (o != fp) {
        atomicAdd(&C->overflow, 1ull);               // a full table: fail loudly (as shard_narrow.h)
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
  // the workgroup's parents (NARROW_THREADS / NARROW_ESUB of them) for the
  // emit: state, plan counts and new-state mask
  constexpr int WP = NARROW_THREADS / NARROW_ESUB;
  const int pl_local = (int)(threadIdx.x / NARROW_ESUB);
  if (sub == 0) {
    sh_ps[pl_local] = s;
    sh_pc[pl_local] = pl.counts;
    sh_pm[pl_local] = live ? m : 0u;
  }
  __syncthreads();
  NTRACE_F(3);
  if (sub == 0) {                                   // inclusive new-state offset in the workgroup
    unsigned int before = 0;
    for (int w = 0; w < wv; ++w) before += sh_w[w];
    sh_pincl[pl_local] = before + (unsigned int)incl;
  }
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
  const unsigned int base = sh_base;
  unsigned long long cnd = 0;
  // the workgroup's new states dealt out one per lane (r = rank in the
  // workgroup, in (parent, t) order): no lane runs more than ceil(wtot/256)
  // of the emit + expand chains.  When they fit half the workgroup (most
  // narrow levels), each state is rebuilt by two lanes in different waves:
  // waves 0-1 store it and check its invariants, waves 2-3 plan and stage
  // its expansion, so the two halves of the chain run side by side on
  // different SIMDs (a level's time is one lane's chain).
  const bool split = wtot <= (unsigned int)NARROW_THREADS / 2;
  const int part = split ? (threadIdx.x < (unsigned int)NARROW_THREADS / 2 ? 1 : 2) : 0;   // 0: both
  const unsigned int rstep = split ? NARROW_THREADS / 2 : NARROW_THREADS;
  for (unsigned int r = split ? threadIdx.x % (NARROW_THREADS / 2) : threadIdx.x; r < wtot; r += rstep) {
    State* __restrict__ nxt = (lev & 1) ? bufA : bufB;
    const uint64_t next_gidx = level_gidx + n;
    unsigned int lo = 0, hi = WP - 1;               // first parent whose inclusive offset > r
    while (lo < hi) {
      const unsigned int mid = (lo + hi) >> 1;
      if (sh_pincl[mid] > r) hi = mid; else lo = mid + 1;
    }
    const unsigned int pr = lo;
    uint32_t mm = sh_pm[pr];
    for (unsigned int k = r - (sh_pincl[pr] - (unsigned int)__builtin_popcount(mm)); k > 0; --k) mm &= mm - 1;
    const int t = __ffs(mm) - 1;
    const uint64_t i = (uint64_t)blockIdx.x * WP + pr;    // the parent
    const uint64_t o = (uint64_t)base + r;                 // the new state's index in level L + 1
    const State sp = sh_ps[pr];
    const typename M::Plan ppl{sh_pc[pr], 0, -1, -1};
    {
      int slot, j;
      M::locate(ppl, t, slot, j);
      State x;
      M::apply(sp, slot, j, f, x);
      if (part != 2) {
        store_state<M>(nxt, o, x);
        if (keep_trace) {
          parent[next_gidx + o] = level_gidx + i;
          ord[next_gidx + o] = (uint8_t)t;
        }
        if (M::check(x, f.inv_mask) >= 0)
          atomicMin(&ctl->err[pq], (i << 16) | ((uint64_t)t << 8) | E_INVARIANT);
        atomicAdd(&sh_dist[M::slot_action(sp, slot)], 1u);
      }
      if (part == 1) continue;
      // expand x for level L + 1 while it is in registers: its errors,
      // per-action counts and its successors' table entries (key: its index
      // o in level L + 1) are level L + 1's, kept only if that level runs
      // narrow (the closing step commits or discards them)
      const typename M::Plan px = M::plan(x, f);
      cnd += (unsigned long long)px.total;
      if (px.fail_pos >= 0)
        atomicMin(&ctl->err[qq], (o << 16) | ((uint64_t)px.fail_pos << 8) | E_ASSERT);
      else if (px.total == 0 && check_deadlock)
        atomicMin(&ctl->err[qq], (o << 16) | E_DEADLOCK);
#pragma unroll
      for (int sl = 0; sl < M::NSLOT; ++sl) {
        const int c = (int)((px.counts >> (6 * sl)) & 63);
        if (c) atomicAdd(&sh_actn[M::slot_action(x, sl)], (unsigned)c);
      }
      if (px.total > M::MAXSUCC) atomicOr(&ctl->lt_over[qq], 1u);   // (the wide path reports it, if it gets there)
      const int tx = px.total < M::MAXSUCC ? px.total : M::MAXSUCC;
      if (o < (uint64_t)NARROW_MAX) {
        sc->pcnt[qq][o] = px.counts;
        sc->ptot[qq][o] = (unsigned char)tx;
      }
      if (tx) {
        // its successors are spread over the whole workgroup below: stage it
        const unsigned int xs = atomicAdd(&sh_nx, 1u);
        if (xs < NX_LDS) {
          sh_xs[xs] = x;
          sh_xc[xs] = px.counts;
          sh_xf[xs] = M::fp_fold(x);
          sh_xo[xs] = (unsigned int)o;
          sh_xt[xs] = (unsigned int)tx;
        } else if (!lt_enter_succ<M>(lt_next, sc->hidx[qq], x, px, tx, (unsigned int)o, f)) {   // LDS full: this lane
          atomicOr(&ctl->lt_over[qq], 1u);
        }
      }
    }
  }
  // the staged states' successors, one (state, t) task per lane: their
  // fingerprints go into level L + 1's table
  __syncthreads();
  NTRACE_F(5);
  {
    const unsigned int nx = sh_nx < NX_LDS ? sh_nx : NX_LDS;
    if (wv == 0) {                                  // exclusive prefix of the successor counts
      constexpr int PER = (NX_LDS + 63) / 64;
      unsigned int sum = 0;
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const unsigned int ix = lane * PER + k;
        sum += ix < nx ? sh_xt[ix] : 0u;
      }
      unsigned int inc = sum;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const unsigned int v = __shfl_up(inc, off, 64);
        if (lane >= off) inc += v;
      }
      unsigned int run = inc - sum;
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const unsigned int ix = lane * PER + k;
        if (ix < nx) {
          sh_xoff[ix] = run;
          run += sh_xt[ix];
        }
      }
      if (lane == 63) sh_ntask = inc;
    }
    __syncthreads();
    NTRACE_F(6);
    const unsigned int T = sh_ntask;
    bool ok = true;
    constexpr int NB2 = 2;
    for (unsigned int b0 = threadIdx.x; b0 < T; b0 += NARROW_THREADS * NB2) {
      uint64_t fpx[NB2];
      unsigned int kx[NB2];
#pragma unroll
      for (int q = 0; q < NB2; ++q) {
        const unsigned int j = b0 + (unsigned int)q * NARROW_THREADS;
        fpx[q] = 0;
        kx[q] = 0;
        if (j < T) {
          unsigned int lo = 0, hi = nx;             // last staged state with offset <= j
          while (hi - lo > 1) {
            const unsigned int mid = (lo + hi) >> 1;
            if (sh_xoff[mid] <= j) lo = mid; else hi = mid;
          }
          const int t = (int)(j - sh_xoff[lo]);
          const State xx = sh_xs[lo];
          const typename M::Plan pxx{sh_xc[lo], 0, -1, -1};
          int sl2, j2, who2;
          M::locate(pxx, t, sl2, j2);
          State y;
          M::apply(xx, sl2, j2, f, y, who2);
          fpx[q] = M::fingerprint_succ(xx, sh_xf[lo], y, who2);
          kx[q] = (sh_xo[lo] << 5) | (unsigned int)t;
        }
      }
      uint64_t h[NB2];
      ok &= lt_enter<NB2>(lt_next, fpx, kx, h);
#pragma unroll
      for (int q = 0; q < NB2; ++q) {
        const unsigned int o2 = kx[q] >> 5;
        if (fpx[q] && o2 < (unsigned int)NARROW_MAX) sc->hidx[qq][o2 * 32 + (kx[q] & 31)] = (unsigned short)h[q];
      }
    }
    if (!ok) atomicOr(&ctl->lt_over[qq], 1u);
  }
  NTRACE_F(7);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    cnd += __shfl_down(cnd, off, 64);
    probes += __shfl_down(probes, off, 64);
  }
  if (lane == 0 && cnd) atomicAdd(&sh_cand, cnd);
  if (lane == 0 && probes) atomicAdd((unsigned long long*)&ctl->probes, probes);
  __syncthreads();
  NTRACE_F(8);
  if (threadIdx.x < A_COUNT && sh_dist[threadIdx.x])
    atomicAdd(&stripe(C).act_dist[threadIdx.x], (unsigned long long)sh_dist[threadIdx.x]);
  if (threadIdx.x < OUTDEG_BINS && sh_deg[threadIdx.x])
    atomicAdd(&stripe(C).outdeg[threadIdx.x], (unsigned long long)sh_deg[threadIdx.x]);
  if (threadIdx.x < A_COUNT && sh_actn[threadIdx.x]) atomicAdd(&ctl->act_next[qq][threadIdx.x], sh_actn[threadIdx.x]);
  // The last workgroup to get here closes the level.  Its inputs are all
  // device-scope atomics: every wave waits for its own to complete (an
  // s_waitcnt on all counters; no L2 write-back needed), then one returning
  // add carries this workgroup's new-state and successor totals with the
  // arrival count, so the last arriver has the level's totals at once and
  // reads only the error key.
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  NTRACE_F(9);
  if (threadIdx.x == 0) {
    const unsigned long long mine_acc = (1ull << 56) | ((unsigned long long)wtot << 28) | sh_cand;
    const unsigned long long prev = atomicAdd(&ctl->close_acc, mine_acc);
    sh_last = (prev >> 56) == NARROW_FWG - 1;
    sh_all = prev + mine_acc;
  }
  __syncthreads();
  if (sh_last && wv == 0) {
    const unsigned long long all = sh_all;
    narrow_step(ctl, C, (all >> 28) & ((1ull << 28) - 1), all & ((1ull << 28) - 1), lev);
    NTRACE_F(10);
  }
}

// Wave 0 of the last k_nfinish workgroup to finish: close level L (its
// `total` new states with `cnext` successors) and decide about L + 1; lane
// a commits (L + 1 runs narrow) or drops action a's pre-expansion count.
__device__ __forceinline__ void narrow_step(NarrowCtl* __restrict__ ctl, Counters* __restrict__ C, uint64_t total,
                                            unsigned long long cnext, uint32_t lev) {
  NarrowCtl& c = *ctl;
  const unsigned int pq = lev & 1, qq = pq ^ 1u;
  const int lane = threadIdx.x & 63;
  int keep = 0;                                  // level L + 1 runs narrow
  if (lane == 0) {
    const unsigned long long err = __hip_atomic_load(&c.err[pq], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    c.close_acc = 0;
    c.err[pq] = ~0ull;
    ++c.levels;
    c.new_total += total;
    c.room = c.room > total ? c.room - total : 0;
    if (err != ~0ull) {                          // the level stays the current one
      c.err_key = err;
      C->err_key = err;
      c.reason = NX_ERROR;
      c.active = 0;
    } else {
      if (c.level < KC_MAX_LEVELS) c.widths[c.level] = total;
      c.level_gidx += c.n;
      c.n = total;
      c.cand = cnext;
      c.level += 1;
      c.cur_is_b ^= 1u;
      int r = narrow_exit_reason(c);
      if (!r && __hip_atomic_load(&c.lt_over[qq], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) r = NX_ROOM;
      if (r) {
        c.reason = r;
        c.active = 0;
      } else {
        keep = 1;
      }
    }
    if (!keep) c.err[qq] = ~0ull;              // drop level L + 1's pre-expansion
    c.lt_over[qq] = 0;
  }
  keep = __shfl(keep, 0, 64);
  if (lane < A_COUNT) {
    const unsigned int v = __hip_atomic_load(&c.act_next[qq][lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (v) {
      if (keep) atomicAdd(&C->s[0].act_gen[lane], (unsigned long long)v);
      c.act_next[qq][lane] = 0;
    }
  }
}

}  // namespace kc
