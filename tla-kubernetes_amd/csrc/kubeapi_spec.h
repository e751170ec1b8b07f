// kubeapi_spec.h — KubeAPI.tla lowered to fixed-width packed state vectors.
//
// This is the "spec compiler" output for the KubeAPI subset of TLA+: every
// variable of KubeAPI.tla (VARIABLES apiState, requests, listRequests, pc,
// stack, op, obj, kind, shouldReconcile; :375,448) is given a finite domain
// and a fixed bit field, chosen so that equal TLA+ values have equal bits
// (canonical), and the 22 actions of Next (:471-756) plus TypeOK and
// OnlyOneVersion (:776-789) become branch-light integer code usable on the
// GPU (__device__) and on the host (__host__, for trace replay).
//
// Parameterisation: the hard-coded process sets {"Client"}, {"PVCController"},
// {"Server"} (KubeAPI.tla:161,225,268) become NC clients, NP PVC controllers
// and NS API servers (Model_1 = 1,1,1).  Clients and controllers are the
// "actors": they call API/ListAPI and appear in version vectors.  Servers
// have no mutable per-process state (APIStart never writes its own pc,
// stack, op, obj or kind, :755-756), so they take no bits.
//
// Layout, W 64-bit words, W even so a state is whole 16-B
// vectors:
//   word 0            apiState: a set over the object universe U (|U| bits)
//   word 1+a          scalar fields of actor a (see ActorField offsets)
//   word 1+A+...      listRequests[a].objs, |U| bits per actor, packed
// Object universe U (values that can be elements of apiState): identity
// (Secret/foo or PVC/mypvc) x "spec" present x version vector (a subset of
// the A actors); u = id<<(A+1) | spec<<A | vv.  Scalar object values
// (obj, stack frame obj, request obj) use objcode: 0 = defaultInitValue,
// 1+id = the bare record [k |-> .., n |-> ..], 3+u = a record with vv.
#pragma once
#include <stdint.h>

#include <type_traits>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define KC_HD __host__ __device__ __forceinline__
#else
#define KC_HD inline
#endif

// A/B build switches of the successor loop (k_claim): the single-GPU
// fingerprint's top bits from the fold (no owner projection), and slot
// lookup by byte-parallel compares of cumulative counts (locate_cum)
#ifndef KC_FP_MIX
#define KC_FP_MIX 2
#endif
#ifndef KC_OWN0_FOLD
#define KC_OWN0_FOLD 1
#endif
#ifndef KC_LOCATE_SWAR
#define KC_LOCATE_SWAR 1
#endif

namespace kc {

// ---------------------------------------------------------------- labels
// pc values (the PlusCal labels; KubeAPI.tla:467-469 and each action's pc').
enum Label : int {
  L_NONE = 0,
  L_CStart, L_C1, L_C10, L_C11, L_c12, L_C13, L_C2, L_C3, L_C8, L_C6, L_C7, L_C4, L_C5,
  L_PVCStart, L_PVCListedPVCs, L_PVCHavePVCs, L_PVCDone,
  L_APIStart,
  L_DoRequest, L_DoReply, L_DoListRequest, L_DoListReply,
  L_COUNT
};
// action ids, in the order TLC lists them (MC.out:78-621)
enum Action : int {
  A_DoRequest = 0, A_DoReply, A_DoListRequest, A_DoListReply, A_CStart, A_C1, A_C10,
  A_C11, A_c12, A_C13, A_C2, A_C3, A_C8, A_C6, A_C7, A_C4, A_C5, A_PVCStart,
  A_PVCListedPVCs, A_PVCHavePVCs, A_PVCDone, A_APIStart, A_COUNT
};
enum Verb : int { OP_DIV = 0, OP_Create, OP_Get, OP_Update, OP_Delete, OP_Force };
enum Resp : int { ST_NONE = 0, ST_Pending, ST_Ok, ST_Error };
enum KindV : int { K_DIV = 0, K_Secret, K_PVC };
enum Proc : int { PR_NONE = 0, PR_API, PR_ListAPI };
enum Ident : int { ID_Secret = 0, ID_PVC = 1 };

// error kinds carried in the low byte of an error key
enum ErrKind : int { E_NONE = 0, E_ASSERT = 1, E_INVARIANT = 2, E_DEADLOCK = 3 };

// run-time switches (MC.tla constants and build-authored variants)
//   variant 0 = KubeAPI.tla as written.  Seeded bugs (build-authored, each
//   exercising one error path of the checker; the oracle has the same):
//   1 = Update without the HasRead check (:733)        -> lost updates
//   2 = Force adds without replacing (:706-715)         -> OnlyOneVersion
//   3 = C1 ignores the Force reply status (:553)        -> C2 Assert (:598-599)
//   4 = list replies ignore the kind filter (:747)      -> TypeOK (:433-435)
//   5 = Init store already holds two Secret versions    -> Init violates
//       (a pre-corrupted apiState, :456)                   OnlyOneVersion
//
// NoLostUpdate (build-defined, inv_mask bit 2; SURVEY §8(d) config 5's
// second variant): the optimistic-concurrency guarantee HasRead gives Update
// (:733) — no Update overwrites a version its writer has not read.  It needs
// a history variable: lostUpdate (a ghost, FALSE in Init) becomes TRUE when
// APIStart applies an Update whose writer has not read any stored version of
// the object (only variant 1 can), and NoLostUpdate == ~lostUpdate.  The
// ghost exists only in runs that check NoLostUpdate, and stays FALSE in
// every reachable state of KubeAPI.tla as written, so those state spaces are
// unchanged.  It is bit 63 of word 0 (apiState holds |U| <= 32 bits when
// there are at most 3 actors; with 4 the invariant is unavailable).
struct Flags {
  int can_fail;      // REQUESTS_CAN_FAIL
  int can_timeout;   // REQUESTS_CAN_TIMEOUT
  int variant;
  int inv_mask = 3;  // invariants checked (MC.cfg INVARIANT): bit 0 TypeOK, bit 1 OnlyOneVersion,
                     // bit 2 NoLostUpdate (build-defined)
};
constexpr uint64_t GHOST_LOST = 1ull << 63;   // lostUpdate (word 0; see above)

KC_HD constexpr int ceil_log2(int x) { return x <= 1 ? 0 : 1 + ceil_log2((x + 1) / 2); }

KC_HD int popc(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __popcll(x);
#else
  return __builtin_popcountll(x);
#endif
}
KC_HD int ctz(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __ffsll((unsigned long long)x) - 1;
#else
  return __builtin_ctzll(x);
#endif
}
// index of the j-th set bit of x (j < popc(x))
KC_HD int nth_bit(uint64_t x, int j) {
  for (int k = 0; k < j; ++k) x &= x - 1;
  return ctz(x);
}
KC_HD uint64_t getf(uint64_t w, int off, int n) { return (w >> off) & ((1ull << n) - 1); }
KC_HD uint64_t setf(uint64_t w, int off, int n, uint64_t v) {
  const uint64_t m = ((1ull << n) - 1) << off;
  return (w & ~m) | ((v << off) & m);
}

// Compile-time loop: f(std::integral_constant<int, I>) for I in [0, N).
template <int N, int I = 0, class F>
KC_HD void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<N, I + 1>(f);
  }
}

template <int NC_, int NP_, int NS_>
struct Model {
  static constexpr int NC = NC_, NP = NP_, NS = NS_;
  static constexpr int A = NC + NP;             // actors (= readers in vv)
  static constexpr int P = A + NS;              // |ProcSet|
  static constexpr int UB = A + 2;              // log2 |U|
  static constexpr int U = 1 << UB;             // object universe size
  static constexpr int NOBJ = 3 + U;            // objcode values
  static constexpr int OBJB = ceil_log2(NOBJ);  // objcode bits
  static_assert(A >= 1 && A <= 4 && NS >= 0, "KubeAPI model: 1..4 actors");
  static constexpr int OBJ_PER_WORD = 64 / U;   // listRequests objs masks per word
  static constexpr int OBJ_WORDS = (A + OBJ_PER_WORD - 1) / OBJ_PER_WORD;
  static constexpr int W_RAW = 1 + A + OBJ_WORDS;
  static constexpr int W = (W_RAW + 1) & ~1;    // state words (even)
  static constexpr int MAXSUCC = 32;            // successor slots per state

  // actor word field offsets (LSB first)
  static constexpr int F_PC = 0, B_PC = 5;
  static constexpr int F_RQP = F_PC + B_PC, F_RQST = F_RQP + 1, F_RQOP = F_RQST + 2,
                       F_RQOBJ = F_RQOP + 3;
  static constexpr int F_LRP = F_RQOBJ + OBJB, F_LRST = F_LRP + 1, F_LRK = F_LRST + 2;
  static constexpr int F_SD = F_LRK + 2, F_SPROC = F_SD + 1, F_SRET = F_SPROC + 2,
                       F_SOP = F_SRET + 5, F_SOBJ = F_SOP + 3, F_SKIND = F_SOBJ + OBJB;
  static constexpr int F_OP = F_SKIND + 2, F_OBJ = F_OP + 3, F_KIND = F_OBJ + OBJB,
                       F_SR = F_KIND + 2;
  static constexpr int ACTOR_BITS = F_SR + 1;
  static_assert(ACTOR_BITS <= 64, "actor word overflow");

  static constexpr uint64_t UMASK = (U == 64) ? ~0ull : ((1ull << U) - 1);
  // U bits whose identity is `id`: the upper / lower half of U
  KC_HD static uint64_t id_mask(int id) {
    const uint64_t half = (1ull << (U / 2)) - 1;
    return id ? (half << (U / 2)) : half;
  }
  KC_HD static uint64_t kind_mask(int kind) {
    return kind == K_Secret ? id_mask(ID_Secret) : kind == K_PVC ? id_mask(ID_PVC) : 0ull;
  }
  KC_HD static int u_id(int u) { return (u >> (A + 1)) & 1; }
  KC_HD static int u_spec(int u) { return (u >> A) & 1; }
  KC_HD static int u_vv(int u) { return u & ((1 << A) - 1); }
  KC_HD static int u_make(int id, int spec, int vv) { return (id << (A + 1)) | (spec << A) | vv; }

  // objcode helpers
  KC_HD static int oc_bare(int id) { return 1 + id; }
  KC_HD static int oc_full(int u) { return 3 + u; }
  KC_HD static bool oc_is_full(int oc) { return oc >= 3; }
  KC_HD static int oc_u(int oc) { return oc - 3; }
  KC_HD static int oc_id(int oc) { return oc >= 3 ? u_id(oc - 3) : oc - 1; }
  // Write(o) == "vv" :> {} @@ o   (KubeAPI.tla:395) — as an element of U
  KC_HD static int write_u(int oc) {
    return oc >= 3 ? u_make(u_id(oc - 3), u_spec(oc - 3), 0) : u_make(oc - 1, 0, 0);
  }
  // Read(o, c) == [o EXCEPT !.vv = @ \cup {c}]   (:399)
  KC_HD static int read_u(int u, int c) { return u | (1 << c); }

  struct State { uint64_t w[W]; };

  // ------------------------------------------------------------ accessors
  // Every actor index used on the device is a compile-time constant (actor
  // templates + static_for): a runtime index into State::w — including the
  // select-of-offsets InstCombine makes out of a compare chain — would pin
  // the state in scratch memory.
  template <int a> KC_HD static uint64_t aw(const State& s) { return s.w[1 + a]; }
  template <int a> KC_HD static int pc(const State& s) { return (int)getf(s.w[1 + a], F_PC, B_PC); }
  template <int a> KC_HD static int fld(const State& s, int off, int n) {
    return (int)getf(s.w[1 + a], off, n);
  }
  template <int a> KC_HD static void put(State& s, int off, int n, int v) {
    s.w[1 + a] = setf(s.w[1 + a], off, n, (uint64_t)v);
  }
  template <int a> KC_HD static uint64_t objs(const State& s) {
    constexpr int wi = 1 + A + a / OBJ_PER_WORD, sh = (a % OBJ_PER_WORD) * U;
    return (s.w[wi] >> sh) & UMASK;
  }
  template <int a> KC_HD static void set_objs(State& s, uint64_t v) {
    constexpr int wi = 1 + A + a / OBJ_PER_WORD, sh = (a % OBJ_PER_WORD) * U;
    s.w[wi] = (s.w[wi] & ~(UMASK << sh)) | ((v & UMASK) << sh);
  }
  KC_HD static constexpr bool is_client(int a) { return a < NC; }

  // Runtime-actor accessors for the (single-copy) action bodies of apply():
  // each candidate word passes through an empty asm so it is a VALUE, and
  // the actor is chosen with selects on values; without the barrier
  // InstCombine turns the chain into a load from a select'ed offset, which
  // forces the whole state into scratch.
  KC_HD static void opaque(uint64_t& x) {
#if defined(__HIP_DEVICE_COMPILE__)
    asm("" : "+v"(x));
#else
    (void)x;
#endif
  }
  KC_HD static uint64_t aw_d(const State& s, int a) {
    uint64_t r = s.w[1];
#pragma unroll
    for (int k = 1; k < A; ++k) {
      uint64_t v = s.w[1 + k];
      opaque(v);
      r = (a == k) ? v : r;
    }
    return r;
  }
  KC_HD static uint64_t objs_d(const State& s, int a) {
    uint64_t r = 0;
#pragma unroll
    for (int k = 0; k < A; ++k) {
      uint64_t v = (s.w[1 + A + k / OBJ_PER_WORD] >> ((k % OBJ_PER_WORD) * U)) & UMASK;
      opaque(v);
      r = (a == k) ? v : r;
    }
    return r;
  }
  KC_HD static void set_objs_d(State& s, int a, uint64_t v) {
#pragma unroll
    for (int k = 0; k < A; ++k) {
      const int wi = 1 + A + k / OBJ_PER_WORD, sh = (k % OBJ_PER_WORD) * U;
      const uint64_t w = s.w[wi];
      uint64_t nw = (w & ~(UMASK << sh)) | ((v & UMASK) << sh);
      opaque(nw);
      s.w[wi] = (a == k) ? nw : w;
    }
  }

  // Host-only runtime-index views (tuple conversion, printing).
  static uint64_t aw_rt(const State& s, int a) { return s.w[1 + a]; }
  static uint64_t objs_rt(const State& s, int a) {
    return (s.w[1 + A + a / OBJ_PER_WORD] >> ((a % OBJ_PER_WORD) * U)) & UMASK;
  }
  static int fld_rt(const State& s, int a, int off, int n) { return (int)getf(s.w[1 + a], off, n); }
  static void put_rt(State& s, int a, int off, int n, int v) {
    s.w[1 + a] = setf(s.w[1 + a], off, n, (uint64_t)v);
  }
  static void set_objs_rt(State& s, int a, uint64_t v) {
    const int wi = 1 + A + a / OBJ_PER_WORD, sh = (a % OBJ_PER_WORD) * U;
    s.w[wi] = (s.w[wi] & ~(UMASK << sh)) | ((v & UMASK) << sh);
  }

  // IsUnboundPVC over a set of U elements (:444-446): PVC identity, no spec
  // — a fixed subset of U, so one AND
  static constexpr uint64_t unbound_mask() {
    uint64_t r = 0;
    for (int u = 0; u < U && u < 64; ++u)
      if (((u >> (A + 1)) & 1) == ID_PVC && !((u >> A) & 1)) r |= 1ull << u;
    return r;
  }
  KC_HD static uint64_t unbound(uint64_t set) { return set & unbound_mask(); }
  // apiState' = {IF IsVersionOf(o, X) THEN Read(o, c) ELSE o : o \in apiState}
  // restricted to the U bits in `sel`
  KC_HD static uint64_t read_map(uint64_t api, uint64_t sel, int c) {
    uint64_t nw = api & ~sel;
    for (uint64_t x = api & sel; x; x &= x - 1) nw |= 1ull << read_u(ctz(x), c);
    return nw;
  }

  // --------------------------------------------------------------- Init
  // Init (KubeAPI.tla:455-469): 2^NC states, shouldReconcile enumerated as a
  // binary counter (client 0 least significant, FALSE first).
  KC_HD static int num_init() { return 1 << NC; }
  KC_HD static void init_state(int k, State& s, int variant = 0) {
#pragma unroll
    for (int i = 0; i < W; ++i) s.w[i] = 0;
    // variant 5: Secret/foo stored twice (vv {} and vv {actor 0})
    if (variant == 5) s.w[0] = (1ull << u_make(ID_Secret, 0, 0)) | (1ull << u_make(ID_Secret, 0, 1));
    static_for<A>([&](auto AI) {
      constexpr int a = AI;
      put<a>(s, F_PC, B_PC, is_client(a) ? L_CStart : L_PVCStart);
      if (is_client(a)) put<a>(s, F_SR, 1, (k >> a) & 1);
    });
  }

  // ------------------------------------------------- successor enumeration
  // Successors are listed in TLC's action order:
  //   slot a in [0,A)      : DoRequest/DoReply/DoListRequest/DoListReply of actor a
  //   slot A+a             : the own-label action of actor a (clients, then
  //                          PVC controllers)
  //   slot 2A+k, k < NS    : APIStart of server k
  // At most one action per slot is enabled (pc selects it).  slot_count
  // returns the slot's successor count, or -1 when evaluating the enabled
  // action raises an Assert failure (C2 :598, C4 :639, APIStart :740).
  static constexpr int NSLOT = 2 * A + NS;

  template <int slot>
  KC_HD static int slot_count(const State& s, const Flags& f) {
    if constexpr (slot < A) {
      constexpr int a = slot;
      const int p = pc<a>(s);
      const int nb = 1 + (f.can_fail ? 1 : 0) + (f.can_timeout ? 1 : 0);
      if (p == L_DoRequest || p == L_DoListRequest) return nb;        // :472-480, :500-508
      if (p == L_DoReply)                                              // :486-490
        return fld<a>(s, F_RQST, 2) != ST_Pending ? 1 + (f.can_timeout ? 1 : 0) : 0;
      if (p == L_DoListReply)                                          // :514-519
        return fld<a>(s, F_LRST, 2) != ST_Pending ? 1 + (f.can_timeout ? 1 : 0) : 0;
      return 0;
    } else if constexpr (slot < 2 * A) {
      constexpr int a = slot - A;
      const int p = pc<a>(s);
      if constexpr (is_client(a)) {
        switch (p) {
          case L_CStart: return 2;                                     // :529-531
          case L_C1: case L_C10: case L_C11: case L_c12: case L_C13:
          case L_C3: case L_C8: case L_C7: case L_C5: return 1;
          case L_C2: return (s.w[0] & id_mask(ID_Secret)) ? 1 : -1;     // :598
          case L_C4: return (s.w[0] & id_mask(ID_Secret)) ? -1 : 1;     // :639
          case L_C6: return popc(objs<a>(s));                          // :619
          default: return 0;
        }
      } else {
        switch (p) {
          case L_PVCStart: case L_PVCListedPVCs: case L_PVCDone: return 1;
          case L_PVCHavePVCs: return popc(unbound(objs<a>(s)));        // :674
          default: return 0;
        }
      }
    } else {
      // APIStart (:698-756): one successor per pending request, then one per
      // pending list request.  A pending request whose op is not a verb
      // would hit Assert(FALSE) (:740).
      int n = 0;
      bool bad = false;
      static_for<A>([&](auto CI) {
        constexpr int c = CI;
        if (fld<c>(s, F_RQP, 1) && fld<c>(s, F_RQST, 2) == ST_Pending) {
          const int op = fld<c>(s, F_RQOP, 3);
          if (op < OP_Create || op > OP_Force) bad = true;
          ++n;
        }
      });
      if (bad) return -1;
      static_for<A>([&](auto CI) {
        constexpr int c = CI;
        if (fld<c>(s, F_LRP, 1) && fld<c>(s, F_LRST, 2) == ST_Pending) ++n;
      });
      return n;
    }
  }

  // Action id of a slot's enabled action.
  template <int slot>
  KC_HD static int slot_action_t(const State& s) {
    if constexpr (slot >= 2 * A) {
      return A_APIStart;
    } else {
      constexpr int a = slot < A ? slot : slot - A;
      switch (pc<a>(s)) {
        case L_DoRequest: return A_DoRequest;   case L_DoReply: return A_DoReply;
        case L_DoListRequest: return A_DoListRequest; case L_DoListReply: return A_DoListReply;
        case L_CStart: return A_CStart; case L_C1: return A_C1; case L_C10: return A_C10;
        case L_C11: return A_C11; case L_c12: return A_c12; case L_C13: return A_C13;
        case L_C2: return A_C2; case L_C3: return A_C3; case L_C8: return A_C8;
        case L_C6: return A_C6; case L_C7: return A_C7; case L_C4: return A_C4;
        case L_C5: return A_C5; case L_PVCStart: return A_PVCStart;
        case L_PVCListedPVCs: return A_PVCListedPVCs; case L_PVCHavePVCs: return A_PVCHavePVCs;
        case L_PVCDone: return A_PVCDone;
        default: return A_APIStart;
      }
    }
  }
  KC_HD static int slot_action(const State& s, int slot) {
    int r = A_APIStart;
    static_for<NSLOT>([&](auto SI) {
      if (slot == (int)SI) r = slot_action_t<SI>(s);
    });
    return r;
  }

  // Successor plan of a state: per-slot counts packed 6 bits each, the total
  // number of successors and the position of an Assert failure (or -1).
  struct Plan {
    uint64_t counts;   // 6 bits per slot
    int total;
    int fail_pos;      // successors generated before the failing action, or -1
    int fail_slot;
  };
  static_assert(NSLOT * 6 <= 64, "too many slots");
  KC_HD static Plan plan(const State& s, const Flags& f) {
    Plan pl{0, 0, -1, -1};
    static_for<NSLOT>([&](auto SI) {
      constexpr int slot = SI;
      if (pl.fail_pos >= 0) return;
      const int c = slot_count<slot>(s, f);
      if (c < 0) {
        pl.fail_pos = pl.total;
        pl.fail_slot = slot;
        return;
      }
      pl.counts |= (uint64_t)(c > 63 ? 63 : c) << (6 * slot);
      pl.total += c;
    });
    return pl;
  }
  // The same lookup without a loop: cum holds the cumulative slot ends
  // E_i = c_0 + ... + c_i one per byte (plan_cum; NSLOT <= 7, the top byte
  // is the caller's), and slot = #{i : E_i <= t}, counted with byte-wise
  // subtractions (t | 0x80) - E_i (no borrow: E_i <= 32) and a popcount.
  static constexpr bool CUM_OK = NSLOT <= 7;
  KC_HD static uint64_t plan_cum(uint64_t counts) {
    uint64_t cum = counts & 0xff00000000000000ull;
    uint32_t e = 0;
    static_for<(NSLOT < 7 ? NSLOT : 7)>([&](auto SI) {
      e += (uint32_t)((counts >> (6 * (int)SI)) & 63);
      cum |= (uint64_t)e << (8 * (int)SI);
    });
    return cum;
  }
  KC_HD static void locate_cum(uint64_t cum, int t, int& slot, int& j) {
    constexpr uint64_t G = (NSLOT >= 7 ? 0x0080808080808080ull : ((1ull << (8 * NSLOT)) - 1) & 0x8080808080808080ull);
    const uint32_t tb = (uint32_t)t * 0x01010101u;
    const uint64_t T = ((uint64_t)tb << 32) | tb;
    const uint64_t D = ((T | G) - (cum & (G >> 1 | G >> 2 | G >> 3 | G >> 4 | G >> 5 | G >> 6 | G >> 7))) & G;
    slot = popc(D);
    j = t - (int)(((cum << 8) >> (8 * slot)) & 0xff);
  }

  // successor t of a plan -> (slot, index within slot)
  KC_HD static void locate(const Plan& pl, int t, int& slot, int& j) {
    int s = 0;
    for (;;) {
      const int c = (int)((pl.counts >> (6 * s)) & 63);
      if (t < c) break;
      t -= c;
      ++s;
    }
    slot = s;
    j = t;
  }

  // ---- one actor's scalar word, held in a register while an action
  // rewrites it (each field access is a shift/mask on that word; the word
  // is selected once and written back once, instead of a select over every
  // actor word per field).
  KC_HD static int g(uint64_t w, int off, int n) { return (int)getf(w, off, n); }
  KC_HD static uint64_t sw(uint64_t w, int off, int n, int v) { return setf(w, off, n, (uint64_t)v); }
  // the call-stack fields [F_SD, F_OP) are contiguous
  static constexpr uint64_t FRAME_MASK = ((1ull << (F_OP - F_SD)) - 1) << F_SD;
  KC_HD static uint64_t push_api_w(uint64_t w, int ret) {       // API(...) call frame
    const int op = g(w, F_OP, 3), ob = g(w, F_OBJ, OBJB);
    w &= ~FRAME_MASK;
    w = sw(w, F_SD, 1, 1); w = sw(w, F_SPROC, 2, PR_API); w = sw(w, F_SRET, 5, ret);
    w = sw(w, F_SOP, 3, op); w = sw(w, F_SOBJ, OBJB, ob);
    return w;
  }
  KC_HD static uint64_t push_list_w(uint64_t w, int ret) {      // ListAPI(...) call frame
    const int kd = g(w, F_KIND, 2);
    w &= ~FRAME_MASK;
    w = sw(w, F_SD, 1, 1); w = sw(w, F_SPROC, 2, PR_ListAPI); w = sw(w, F_SRET, 5, ret);
    w = sw(w, F_SKIND, 2, kd);
    return w;
  }
  KC_HD static uint64_t call_w(uint64_t w, int ret, int op, int oc) {
    w = push_api_w(w, ret);
    w = sw(w, F_OBJ, OBJB, oc); w = sw(w, F_OP, 3, op);
    return sw(w, F_PC, B_PC, L_DoRequest);
  }
  // write actor a's word (select over the A words; values behind opaque())
  KC_HD static void put_word_d(State& t, int a, uint64_t nw) {
#pragma unroll
    for (int k = 0; k < A; ++k) {
      uint64_t v = nw;
      opaque(v);
      t.w[1 + k] = (a == k) ? v : t.w[1 + k];
    }
  }

  // Build successor j of slot `slot` into t (t starts as a copy of s).  One
  // copy of every action body, indexed by the runtime actor (apply is the
  // part of the kernel that runs once per successor).
  KC_HD static int apply_rt(const State& s, int slot, int j, const Flags& f, State& t) {
    if (slot < 2 * A) {
      const int a = slot < A ? slot : slot - A;
      uint64_t w = aw_d(s, a);
      const int p = g(w, F_PC, B_PC);
      if (slot < A) {
        if (p == L_DoRequest) {                                 // DoRequest :471-483
          w = sw(w, F_RQP, 1, 1); w = sw(w, F_RQOP, 3, g(w, F_OP, 3));
          w = sw(w, F_RQOBJ, OBJB, g(w, F_OBJ, OBJB));
          w = sw(w, F_RQST, 2, j == 0 ? ST_Pending : ST_Error);
          w = sw(w, F_PC, B_PC, L_DoReply);
        } else if (p == L_DoListRequest) {                      // DoListRequest :499-511
          w = sw(w, F_LRP, 1, 1); w = sw(w, F_LRK, 2, g(w, F_KIND, 2));
          w = sw(w, F_LRST, 2, j == 0 ? ST_Pending : ST_Error);
          w = sw(w, F_PC, B_PC, L_DoListReply);
          set_objs_d(t, a, 0);
        } else if (p == L_DoReply) {                            // DoReply :485-495
          if (j == 1) w = sw(w, F_RQST, 2, ST_Error);
          w = sw(w, F_PC, B_PC, g(w, F_SRET, 5)); w = sw(w, F_OP, 3, g(w, F_SOP, 3));
          w = sw(w, F_OBJ, OBJB, g(w, F_SOBJ, OBJB));
          w &= ~FRAME_MASK;
        } else {                                                // DoListReply :513-524
          if (j == 1) { w = sw(w, F_LRST, 2, ST_Error); set_objs_d(t, a, 0); }
          w = sw(w, F_PC, B_PC, g(w, F_SRET, 5)); w = sw(w, F_KIND, 2, g(w, F_SKIND, 2));
          w &= ~FRAME_MASK;
        }
      } else {
        switch (p) {
          case L_CStart: {                                      // :528-549
            const int sr = j == 0 ? 1 : g(w, F_SR, 1);
            w = sw(w, F_SR, 1, sr);
            if (sr) {
              w = call_w(w, L_C1, OP_Force, oc_bare(ID_Secret));
            } else {
              w = push_list_w(w, L_C3);
              w = sw(w, F_KIND, 2, K_Secret); w = sw(w, F_PC, B_PC, L_DoListRequest);
            }
            break;
          }
          case L_C1:                                            // :551-556
            // variant 3 (seeded bug): the Force reply status is ignored
            w = sw(w, F_PC, B_PC, (g(w, F_RQST, 2) != ST_Ok && f.variant != 3) ? L_CStart : L_C10); break;
          case L_C10: w = call_w(w, L_C11, OP_Force, oc_bare(ID_PVC)); break;   // :558-568
          case L_C11:                                           // :570-575
            w = sw(w, F_PC, B_PC, g(w, F_RQST, 2) != ST_Ok ? L_CStart : L_c12); break;
          case L_c12: w = call_w(w, L_C13, OP_Get, oc_bare(ID_PVC)); break;     // :577-587
          case L_C13: {                                         // :589-594
            bool go = g(w, F_RQST, 2) != ST_Ok;
            if (!go) {
              const int oc = g(w, F_RQOBJ, OBJB);
              go = oc_id(oc) == ID_PVC && !(oc_is_full(oc) && u_spec(oc_u(oc)));
            }
            w = sw(w, F_PC, B_PC, go ? L_CStart : L_C2); break;
          }
          case L_C2: w = sw(w, F_SR, 1, 0); w = sw(w, F_PC, B_PC, L_C5); break;  // :596-602
          case L_C3:                                            // :604-609
            w = sw(w, F_PC, B_PC, g(w, F_LRST, 2) != ST_Ok ? L_CStart : L_C8); break;
          case L_C8: w = sw(w, F_PC, B_PC, objs_d(s, a) == 0 ? L_C4 : L_C6); break;  // :611-616
          case L_C6: {                                          // :618-629
            const int u = nth_bit(objs_d(s, a), j);
            w = call_w(w, L_C7, OP_Delete, oc_bare(u_id(u)));
            break;
          }
          case L_C7: {                                          // :631-636
            const bool go = g(w, F_RQST, 2) != ST_Ok || popc(objs_d(s, a)) > 1;
            w = sw(w, F_PC, B_PC, go ? L_CStart : L_C4); break;
          }
          case L_C4: case L_C5: w = sw(w, F_PC, B_PC, p == L_C4 ? L_C5 : L_CStart); break;
          case L_PVCStart:                                      // :655-663
            w = push_list_w(w, L_PVCListedPVCs);
            w = sw(w, F_KIND, 2, K_PVC); w = sw(w, F_PC, B_PC, L_DoListRequest); break;
          case L_PVCListedPVCs: {                               // :665-671
            const bool go = g(w, F_LRST, 2) != ST_Ok || unbound(objs_d(s, a)) == 0;
            w = sw(w, F_PC, B_PC, go ? L_PVCStart : L_PVCHavePVCs); break;
          }
          case L_PVCHavePVCs: {                                 // :673-688
            const int u = nth_bit(unbound(objs_d(s, a)), j);
            // bound == "spec" :> ("pvname" :> unb.n) @@ unb
            w = call_w(w, L_PVCDone, OP_Update, oc_full(u_make(u_id(u), 1, u_vv(u))));
            break;
          }
          default: /* L_PVCDone */ w = sw(w, F_PC, B_PC, L_PVCStart); break;  // :690-693
        }
      }
      put_word_d(t, a, w);
      return a;
    }
    // APIStart (:698-756): successor j serves the j-th pending request (in
    // actor order), then the pending list requests.
    unsigned prq = 0, plr = 0;
    static_for<A>([&](auto CI) {
      constexpr int c = CI;
      const uint64_t x = s.w[1 + c];
      if (getf(x, F_RQP, 1) && getf(x, F_RQST, 2) == ST_Pending) prq |= 1u << c;
      if (getf(x, F_LRP, 1) && getf(x, F_LRST, 2) == ST_Pending) plr |= 1u << c;
    });
    const int nrq = popc(prq);
    const uint64_t api = s.w[0];
    if (j < nrq) {
      const int c = nth_bit(prq, j);
      uint64_t w = aw_d(s, c);
      const int oc = g(w, F_RQOBJ, OBJB);
      const int id = oc_id(oc);
      const uint64_t same = api & id_mask(id);
      int st = ST_Ok;
      uint64_t nw = api;
      switch (g(w, F_RQOP, 3)) {
        case OP_Create:                                         // :700-705
          if (same) st = ST_Error; else nw = api | (1ull << write_u(oc));
          break;
        case OP_Force:                                          // :706-715
          // variant 2 (seeded bug): add without replacing -> OnlyOneVersion fails
          nw = (f.variant == 2 ? api : (api & ~same)) | (1ull << write_u(oc));
          break;
        case OP_Get:                                            // :716-728
          if (same) {
            w = sw(w, F_RQOBJ, OBJB, oc_full(ctz(same)));       // CHOOSE o \in apiState
            nw = read_map(api, same, c);
          } else st = ST_Error;
          break;
        case OP_Delete: nw = api & ~same; break;                // :729-731
        default: {                                              // Update :732-739
          bool ok = false, read = false;
          for (uint64_t x = same; x; x &= x - 1) {
            const bool hr = (u_vv(ctz(x)) >> c) & 1;            // HasRead
            read |= hr;
            if (f.variant == 1 || hr) ok = true;
          }
          if (ok) nw = (api & ~same) | (1ull << write_u(oc)); else st = ST_Error;
          // lostUpdate' (the NoLostUpdate ghost): an Update applied unread
          if (U < 64 && (f.inv_mask & 4) && ok && !read) nw |= GHOST_LOST;
        }
      }
      t.w[0] = nw;
      put_word_d(t, c, sw(w, F_RQST, 2, st));
      return c;
    }
    if (plr) {                                                  // :745-753
      const int c = nth_bit(plr, j - nrq);
      const uint64_t km = kind_mask(g(aw_d(s, c), F_LRK, 2));
      // variant 4 (seeded bug): the reply lists every object, any kind
      set_objs_d(t, c, f.variant == 4 ? api : (api & km));
      put_word_d(t, c, sw(aw_d(s, c), F_LRST, 2, ST_Ok));
      t.w[0] = read_map(api, km, c);
      return c;
    }
    return 0;
  }

  // Build successor j of `slot` (KubeAPI.tla:471-756); `who` = the process
  // whose word the action rewrote (for fingerprint_succ).
  KC_HD static void apply(const State& s, int slot, int j, const Flags& f, State& t, int& who) {
#pragma unroll
    for (int i = 0; i < W; ++i) t.w[i] = s.w[i];
    who = apply_rt(s, slot, j, f, t);
  }
  KC_HD static void apply(const State& s, int slot, int j, const Flags& f, State& t) {
    int who;
    apply(s, slot, j, f, t, who);
  }

  // ------------------------------------------------------------ invariants
  // Returns -1 if TypeOK (:776-781), OnlyOneVersion (:787-789) and (bit 2)
  // the build-defined NoLostUpdate hold, else the index of the first violated
  // one in MC.cfg order (0 TypeOK, 1 OOV, 2 NoLostUpdate); only the
  // invariants in `mask` (Flags::inv_mask) are evaluated.
  KC_HD static int check(const State& s, int mask = 3) {
    if (!mask) return -1;
    bool typeok = true;
    static_for<A>([&](auto CI) {
      constexpr int c = CI;
      if (fld<c>(s, F_RQP, 1)) {                                // IsValidRequest :426-430
        const int op = fld<c>(s, F_RQOP, 3), st = fld<c>(s, F_RQST, 2);
        if (op < OP_Create || op > OP_Force || fld<c>(s, F_RQOBJ, OBJB) == 0 ||
            st < ST_Pending || st > ST_Error) typeok = false;
      }
      if (fld<c>(s, F_LRP, 1)) {                                // IsValidListRequest :432-436
        const int st = fld<c>(s, F_LRST, 2);
        if ((objs<c>(s) & ~kind_mask(fld<c>(s, F_LRK, 2))) || st < ST_Pending || st > ST_Error)
          typeok = false;
      }
    });
    if (!typeok && (mask & 1)) return 0;
    if ((mask & 2) && (popc(s.w[0] & id_mask(0)) > 1 || popc(s.w[0] & id_mask(1)) > 1)) return 1;
    if (U < 64 && (mask & 4) && (s.w[0] & GHOST_LOST)) return 2;
    return -1;
  }

  // --------------------------------------------------------- fingerprint
  // 64-bit fingerprint of the canonical packed words, normalised the way the
  // FPSet stores it: MSB clear (TLC's disk FPSets reserve it), never 0.
  //
  // Zobrist-style: fp = final(XOR_k mix(w_k, k)), every mix a bijection of
  // 64-bit words (xor-shifts and odd multiplies) and final() only the
  // normalisation (a further bijective finaliser could not change which
  // states collide, and the XOR of mixes is already uniform in every bit).
  // A successor differs from its parent in at most three words — apiState,
  // the acting process's word and that process's listRequests.objs word — so
  // the kernels fold the parent once and re-mix only the changed words of
  // each successor (fingerprint_succ); two states collide
  // only if the XOR of their words' mix differences vanishes (probability
  // ~2^-59 per pair within an owner class, below; TLC's polynomial FP64 is
  // also linear over GF(2)).  64-bit multiplies are quarter-rate on CDNA, so this matters.
  static constexpr uint64_t salt_c(int k) {
    return 0x6a09e667f3bcc909ull + (uint64_t)k * 0x9e3779b97f4a7c15ull;
  }
  KC_HD static uint64_t salt(int k) {          // runtime k: a select, no multiply
    uint64_t r = salt_c(0);
#pragma unroll
    for (int i = 1; i < W_RAW; ++i) r = (k == i) ? salt_c(i) : r;
    return r;
  }
  // KC_FP_MIX (A/B build switch): 2 = two 64-bit multiplies (the default),
  // 1 = one, between two xor-shifts (still a bijection of the word)
  KC_HD static uint64_t mix_salted(uint64_t z) {
#if KC_FP_MIX == 1
    z ^= z >> 32;
    z *= 0xd6e8feb86659fd93ull;
    return z ^ (z >> 29);
#else
    z *= 0xbf58476d1ce4e5b9ull;
    z ^= z >> 31;
    z *= 0x94d049bb133111ebull;
    return z ^ (z >> 29);
#endif
  }
  KC_HD static uint64_t word_mix(uint64_t w, int k) { return mix_salted(w ^ salt(k)); }
  KC_HD static uint64_t fp_fold(const State& s) {
    uint64_t x = 0;
#pragma unroll
    for (int i = 0; i < W_RAW; ++i) x ^= mix_salted(s.w[i] ^ salt_c(i));
    return x;
  }
  // Owner bits.  Fingerprint-owner sharding (shard.hip) gives a state to
  // rank floor(fp * R / 2^63), i.e. to the fingerprint's top bits.  Those
  // OWNER_BITS bits are a hash of a projection of the state, not of the
  // whole state, so that most successors keep their parent's owner (no
  // record to send) and siblings stay together for the LDS tile dedup.  For
  // R dividing 2^OWNER_BITS the owner depends on these bits only.  The other
  // 59 bits are the Zobrist fold, so two states collide only if their
  // projections hash alike and 59 fold bits agree.  The template parameter
  // OWN of the fingerprint functions:
  //  * OWN = 0 (the single-GPU engine, and every fingerprint the C-ABI
  //    reports): with KC_OWN0_FOLD (the default since round 4) no owner
  //    bits at all — the fingerprint is the 63-bit fold (fp_final below), so
  //    two states collide only if all 63 fold bits agree (~2^-63 per pair);
  //    the fingerprint VALUES differ from round-3 builds.
  //    With KC_OWN0_FOLD=0: apiState and the first PVC controller's word;
  //  * OWN = 1 (the sharded path, shard.hip): apiState and the listRequests
  //    objs words.  An action always rewrites its process's scalar word,
  //    but only APIStart changes apiState and only list replies change objs,
  //    so fewer successors change owner: records sent per NP=2 check at
  //    R = 2 / 4 / 8 538M / 853M / 983M -> 338M / 510M / 603M
  //    (tools/shard_records.py, profiles/r03ad_*), per-level balance on the
  //    wide levels 1.02-1.11 at R = 8 (tools/owner_balance.py,
  //    profiles/r03ab_owner.log).  The engine keeps OWN = 0: there the
  //    owner bits buy nothing, and the objs words' extra live range spills
  //    k_claim past its 80-VGPR budget (+6 ms per NP=2 check measured).
  // A run uses one projection throughout; both give the same counts.
  static constexpr int OWNER_BITS = 4;
  static constexpr int OWNER_WORD = 1 + (NP > 0 ? NC : 0);   // first PVC controller (else client)
  KC_HD static uint64_t owner_hash(uint64_t w0, uint64_t wo) {
    uint64_t z = w0 * 0x9e3779b97f4a7c15ull + wo;
    z ^= z >> 31;
    z *= 0xbf58476d1ce4e5b9ull;
    return z >> (64 - OWNER_BITS);
  }
  // OWN = 1: the objs words folded to 32 bits, XOR-linear in each word (a
  // successor rewrites at most one, so its projection is its parent's XOR
  // that word's change); owner_hash does the mixing
  KC_HD static uint32_t owner_word(uint64_t w, int k) {
    const uint32_t v = (uint32_t)(w ^ (w >> 32));
    const int r = (8 * k) & 31;
    return r ? (v << r) | (v >> (32 - r)) : v;
  }
  KC_HD static uint32_t owner_proj(const State& x) {
    uint32_t wo = 0;
#pragma unroll
    for (int k = 0; k < OBJ_WORDS; ++k) wo ^= owner_word(x.w[1 + A + k], k);
    return wo;
  }
  template <int OWN = 0>
  KC_HD static uint64_t owner_bits(const State& x) {
    if constexpr (OWN != 0)
      return owner_hash(x.w[0], owner_proj(x));
    else
      return owner_hash(x.w[0], x.w[OWNER_WORD]);
  }
  KC_HD static uint64_t fp_final_ob(uint64_t h, uint64_t ob) {
    h = (h & ((1ull << (63 - OWNER_BITS)) - 1)) | (ob << (63 - OWNER_BITS));
    return h ? h : 1;
  }
  // KC_OWN0_FOLD (A/B build switch): OWN = 0 takes its top bits from the
  // fold itself, i.e. no owner projection at all (one GPU has no owners)
  template <int OWN = 0>
  KC_HD static uint64_t fp_final(uint64_t h, const State& x) {
#if KC_OWN0_FOLD
    if constexpr (OWN == 0) {
      (void)x;
      h &= 0x7fffffffffffffffull;
      return h ? h : 1;
    }
#endif
    return fp_final_ob(h, owner_bits<OWN>(x));
  }
  template <int OWN = 0>
  KC_HD static uint64_t fingerprint(const State& s) { return fp_final<OWN>(fp_fold(s), s); }

  // Fingerprint of successor x of s, given s's fold and the process `who`
  // whose word the action rewrote (apply's out-parameter).  Equal to
  // fingerprint<OWN>(x).  (Caching the parent's per-word mixes instead of
  // re-mixing the old words costs 15 VGPRs, one wave per SIMD of k_claim's
  // occupancy, and measured slower.)  OWN = 1 takes the parent's owner
  // projection proj_s (the sharded k_claim keeps it in LDS).
  template <int OWN = 0>
  KC_HD static uint64_t fingerprint_succ(const State& s, uint64_t fold_s, const State& x, int who,
                                         uint32_t proj_s = 0) {
    uint32_t wo = proj_s;
    uint64_t h = fold_s;
    if (x.w[0] != s.w[0]) h ^= mix_salted(s.w[0] ^ salt_c(0)) ^ mix_salted(x.w[0] ^ salt_c(0));
    {
      uint64_t o = s.w[1], nw = x.w[1];
#pragma unroll
      for (int k = 1; k < A; ++k) {
        uint64_t vo = s.w[1 + k], vn = x.w[1 + k];
        opaque(vo);
        opaque(vn);
        o = (who == k) ? vo : o;
        nw = (who == k) ? vn : nw;
      }
      if (o != nw) {
        const uint64_t sl = salt(1 + who);
        h ^= mix_salted(o ^ sl) ^ mix_salted(nw ^ sl);
      }
    }
    {
      const int wi = 1 + A + who / OBJ_PER_WORD;
      uint64_t o = s.w[1 + A], nw = x.w[1 + A];
#pragma unroll
      for (int k = 1; k < OBJ_WORDS; ++k) {
        uint64_t vo = s.w[1 + A + k], vn = x.w[1 + A + k];
        opaque(vo);
        opaque(vn);
        o = (wi == 1 + A + k) ? vo : o;
        nw = (wi == 1 + A + k) ? vn : nw;
      }
      if (o != nw) {
        const uint64_t sl = salt(wi);
        h ^= mix_salted(o ^ sl) ^ mix_salted(nw ^ sl);
        if constexpr (OWN != 0) wo ^= owner_word(o ^ nw, wi - (1 + A));
      }
    }
    if constexpr (OWN != 0)
      return fp_final_ob(h, owner_hash(x.w[0], wo));
    else
      return fp_final<0>(h, x);
  }

  // The owner bits of successor x alone (OWN = 1; what fingerprint_succ<1>
  // puts in its top bits), without the fold's re-mixing: at R = 2^k ranks
  // the owner floor(fp * R / 2^63) is these bits >> (4 - k), whatever the
  // fold bits below them (shard.hip's record staging needs only the owner)
  KC_HD static uint32_t owner_bits_succ(const State& s, const State& x, int who, uint32_t proj_s) {
    uint32_t wo = proj_s;
    const int wi = 1 + A + who / OBJ_PER_WORD;
    uint64_t o = s.w[1 + A], nw = x.w[1 + A];
#pragma unroll
    for (int k = 1; k < OBJ_WORDS; ++k) {
      uint64_t vo = s.w[1 + A + k], vn = x.w[1 + A + k];
      opaque(vo);
      opaque(vn);
      o = (wi == 1 + A + k) ? vo : o;
      nw = (wi == 1 + A + k) ? vn : nw;
    }
    if (o != nw) wo ^= owner_word(o ^ nw, wi - (1 + A));
    return (uint32_t)owner_hash(x.w[0], wo);
  }

  // ------------------------------------------------ canonical tuple (ABI)
  // Interchange form shared with tests (include/kubecheck.h): word 0 =
  // apiState as a U mask; then 19 words per process: pc, op, obj, kind, sr,
  // sdepth, sproc, spc, sop, sobj, skind, rq_present, rq_op, rq_status,
  // rq_obj, lr_present, lr_kind, lr_status, lr_objs.  Object values use the
  // "oval" byte: def | id<<1 | has_vv<<2 | spec<<3 | vv<<4.
  static constexpr int TUPLE_PER_PROC = 19;
  static constexpr int TUPLE_WORDS = 1 + TUPLE_PER_PROC * P;
  KC_HD static uint64_t oc_to_oval(int oc) {
    if (oc == 0) return 0;
    if (oc < 3) return 1u | ((oc - 1) << 1);
    const int u = oc - 3;
    return 1u | (u_id(u) << 1) | (1u << 2) | (u_spec(u) << 3) | (u_vv(u) << 4);
  }
  KC_HD static int oval_to_oc(uint64_t ov) {
    if (!(ov & 1)) return 0;
    const int id = (ov >> 1) & 1, hv = (ov >> 2) & 1, sp = (ov >> 3) & 1, vv = (ov >> 4) & 15;
    if (!hv) return (sp || vv) ? -1 : 1 + id;
    return 3 + u_make(id, sp, vv);
  }
  static void to_tuple(const State& s, uint64_t* o) {
    o[0] = s.w[0];
    for (int p = 0; p < P; ++p) {
      uint64_t* q = o + 1 + TUPLE_PER_PROC * p;
      for (int k = 0; k < TUPLE_PER_PROC; ++k) q[k] = 0;
      if (p >= A) { q[0] = L_APIStart; continue; }
      q[0] = fld_rt(s, p, F_PC, B_PC); q[1] = fld_rt(s, p, F_OP, 3); q[2] = oc_to_oval(fld_rt(s, p, F_OBJ, OBJB));
      q[3] = fld_rt(s, p, F_KIND, 2); q[4] = fld_rt(s, p, F_SR, 1); q[5] = fld_rt(s, p, F_SD, 1);
      q[6] = fld_rt(s, p, F_SPROC, 2); q[7] = fld_rt(s, p, F_SRET, 5); q[8] = fld_rt(s, p, F_SOP, 3);
      q[9] = oc_to_oval(fld_rt(s, p, F_SOBJ, OBJB)); q[10] = fld_rt(s, p, F_SKIND, 2);
      q[11] = fld_rt(s, p, F_RQP, 1); q[12] = fld_rt(s, p, F_RQOP, 3); q[13] = fld_rt(s, p, F_RQST, 2);
      q[14] = oc_to_oval(fld_rt(s, p, F_RQOBJ, OBJB));
      q[15] = fld_rt(s, p, F_LRP, 1); q[16] = fld_rt(s, p, F_LRK, 2); q[17] = fld_rt(s, p, F_LRST, 2);
      q[18] = objs_rt(s, p);
    }
  }
  // returns false if the tuple is outside the lowered domain
  static bool from_tuple(const uint64_t* o, State& s) {
    for (int i = 0; i < W; ++i) s.w[i] = 0;
    if (o[0] & ~(UMASK | (U < 64 ? GHOST_LOST : 0ull))) return false;   // (lostUpdate: bit 63)
    s.w[0] = o[0];
    for (int p = 0; p < P; ++p) {
      const uint64_t* q = o + 1 + TUPLE_PER_PROC * p;
      if (p >= A) {
        if (q[0] != L_APIStart) return false;
        for (int k = 1; k < TUPLE_PER_PROC; ++k) if (q[k]) return false;
        continue;
      }
      const int ob = oval_to_oc(q[2]), sob = oval_to_oc(q[9]), rob = oval_to_oc(q[14]);
      if (ob < 0 || sob < 0 || rob < 0 || (q[18] & ~UMASK)) return false;
      if (!is_client(p) && q[4]) return false;
      put_rt(s, p, F_PC, B_PC, (int)q[0]); put_rt(s, p, F_OP, 3, (int)q[1]); put_rt(s, p, F_OBJ, OBJB, ob);
      put_rt(s, p, F_KIND, 2, (int)q[3]); put_rt(s, p, F_SR, 1, (int)q[4]); put_rt(s, p, F_SD, 1, (int)q[5]);
      put_rt(s, p, F_SPROC, 2, (int)q[6]); put_rt(s, p, F_SRET, 5, (int)q[7]); put_rt(s, p, F_SOP, 3, (int)q[8]);
      put_rt(s, p, F_SOBJ, OBJB, sob); put_rt(s, p, F_SKIND, 2, (int)q[10]);
      put_rt(s, p, F_RQP, 1, (int)q[11]); put_rt(s, p, F_RQOP, 3, (int)q[12]); put_rt(s, p, F_RQST, 2, (int)q[13]);
      put_rt(s, p, F_RQOBJ, OBJB, rob);
      put_rt(s, p, F_LRP, 1, (int)q[15]); put_rt(s, p, F_LRK, 2, (int)q[16]); put_rt(s, p, F_LRST, 2, (int)q[17]);
      set_objs_rt(s, p, q[18]);
    }
    return true;
  }
};

// Supported instantiations (NC, NP, NS); the engine dispatches on these.
#define KC_FOR_EACH_MODEL(X) \
  X(1, 1, 1) X(2, 1, 1) X(1, 2, 1) X(2, 0, 1) X(1, 1, 2) X(1, 3, 1) X(2, 2, 1) X(1, 0, 1) X(0, 1, 1) \
  X(1, 1, 0)

}  // namespace kc
