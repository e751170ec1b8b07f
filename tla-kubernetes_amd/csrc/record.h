// record.h — the sharded path's exchange record: one successor
// that changes owner, as it crosses the all-to-all.
//
// Word 0 is the successor's key (sender rank, parent index, successor
// position, action); after it the canonical state is bit-packed field by
// field, at bit offsets fixed at compile time:
//   apiState   U bits (+ the lostUpdate history bit when U < 64)
//   actors     A words of ACTOR_BITS (pc, request, list request, ... fields)
//   objs       A listRequests objs masks of U bits
// padded to a multiple of 16 B.  NP = 2: 48 B (the plain word copy is 64 B),
// NP = 1: 32 B (48 B).  The receiver recomputes the fingerprint instead of
// receiving it.  Host + device: kc_spec_fp_selfcheck round-trips every
// successor through it on the CPU.
#pragma once

#include <stdint.h>

#include "kubeapi_spec.h"

namespace kc {

template <class M>
struct Record {
  static constexpr int B0 = M::U < 64 ? M::U + 1 : 64;     // apiState (+ ghost bit 63)
  static constexpr int P_ACT = 64 + B0;                     // first actor field
  static constexpr int P_OBJ = P_ACT + M::A * M::ACTOR_BITS;
  static constexpr int BITS = P_OBJ + M::A * M::U;
  static constexpr int RW = ((BITS + 63) / 64 + 1) & ~1;   // even: 16-B accesses
  uint64_t w[RW];
};

namespace rec {
template <int RW, int POS, int N>
KC_HD void put(uint64_t (&r)[RW], uint64_t v) {
  constexpr int wd = POS / 64, off = POS % 64;
  // (a field never carries bits past its width in a canonical state; masked
  // anyway, so a stray bit cannot overwrite the next field of the record)
  if constexpr (N < 64) v &= (1ull << N) - 1;
  r[wd] |= v << off;
  if constexpr (off + N > 64) r[wd + 1] |= v >> (64 - off);
}
template <int RW, int POS, int N>
KC_HD uint64_t get(const uint64_t (&r)[RW]) {
  constexpr int wd = POS / 64, off = POS % 64;
  uint64_t v = r[wd] >> off;
  if constexpr (off + N > 64) v |= r[wd + 1] << (64 - off);
  if constexpr (N < 64) v &= (1ull << N) - 1;
  return v;
}
}  // namespace rec

template <class M>
KC_HD void record_pack(const typename M::State& x, uint64_t key, uint64_t (&r)[Record<M>::RW]) {
  using R = Record<M>;
#pragma unroll
  for (int k = 0; k < R::RW; ++k) r[k] = 0;
  r[0] = key;
  const uint64_t w0 = x.w[0];
  rec::put<R::RW, 64, R::B0>(r, M::U < 64 ? (w0 & M::UMASK) | ((w0 >> 63) << (M::U & 63)) : w0);
  static_for<M::A>([&](auto ai) {
    constexpr int a = decltype(ai)::value;
    rec::put<R::RW, R::P_ACT + a * M::ACTOR_BITS, M::ACTOR_BITS>(r, x.w[1 + a]);
    constexpr int wi = 1 + M::A + a / M::OBJ_PER_WORD, sh = (a % M::OBJ_PER_WORD) * M::U;
    rec::put<R::RW, R::P_OBJ + a * M::U, M::U>(r, (x.w[wi] >> sh) & M::UMASK);
  });
}

template <class M>
KC_HD void record_unpack(const uint64_t (&r)[Record<M>::RW], typename M::State& x, uint64_t& key) {
  using R = Record<M>;
#pragma unroll
  for (int k = 0; k < M::W; ++k) x.w[k] = 0;
  key = r[0];
  const uint64_t v0 = rec::get<R::RW, 64, R::B0>(r);
  x.w[0] = M::U < 64 ? (v0 & M::UMASK) | ((v0 >> (M::U & 63)) << 63) : v0;
  static_for<M::A>([&](auto ai) {
    constexpr int a = decltype(ai)::value;
    x.w[1 + a] = rec::get<R::RW, R::P_ACT + a * M::ACTOR_BITS, M::ACTOR_BITS>(r);
    constexpr int wi = 1 + M::A + a / M::OBJ_PER_WORD, sh = (a % M::OBJ_PER_WORD) * M::U;
    x.w[wi] |= rec::get<R::RW, R::P_OBJ + a * M::U, M::U>(r) << sh;
  });
}

}  // namespace kc
