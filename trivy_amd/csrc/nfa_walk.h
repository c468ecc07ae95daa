// nfa_walk.h — the bit-parallel Glushkov NFA walk (nfa.cpp builds the
// tables), shared by k_verify on gfx950 and the host mirror used by tests.
//
// State D = the positions (consuming instructions) that have just consumed the
// byte before boundary q.  One step on byte c:
//   F  = OR_k shift(D & smask[k], shift[k])          (edges p -> p + delta)
//      | OR_{p in D & exc_mask} follow of p           (the other edges, and
//                                                      edges through \b etc.)
//      | first                                        (a thread starts at q)
//   D' = F & reach[cls[c]]
// A match ends at boundary q when D meets `last` (edges to MATCH; the
// conditional ones with the EmptyOp context at q).  Non-ASCII text is decoded
// rune by rune (utf8.DecodeRune) into dfa.cpp's five rune symbols; a rune the
// symbols cannot stand for (a program telling other runes apart) ends the walk
// as undecidable, and the Pike VM decides.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "engine.h"
#include "pikevm.h"

namespace tsg {

__host__ __device__ inline U128 u128_or(U128 a, U128 b) { return U128{a.lo | b.lo, a.hi | b.hi}; }
__host__ __device__ inline U128 u128_and(U128 a, U128 b) { return U128{a.lo & b.lo, a.hi & b.hi}; }
__host__ __device__ inline bool u128_any(U128 a) { return (a.lo | a.hi) != 0; }

// x << d (d > 0) or x >> -d (d < 0), 128-bit; kWide = false: positions < 64 only.
template <bool kWide>
__host__ __device__ inline U128 u128_shift(U128 x, int d) {
  if (!kWide) {
    const uint64_t v = d >= 0 ? x.lo << d : x.lo >> (-d);
    return U128{v, 0};
  }
  if (d == 0) return x;
  if (d > 0) {
    if (d >= 64) return U128{0, x.lo << (d - 64)};
    return U128{x.lo << d, (x.hi << d) | (x.lo >> (64 - d))};
  }
  const int k = -d;
  if (k >= 64) return U128{x.hi >> (k - 64), 0};
  return U128{(x.lo >> k) | (x.hi << (64 - k)), x.hi >> k};
}

template <bool kWide>
__host__ __device__ inline U128 nfa_follow(const NfaDev& N, const NfaExc* exc, U128 D, uint32_t ctx) {
  U128 F{0, 0};
  for (uint32_t k = 0; k < N.nshift; ++k) F = u128_or(F, u128_shift<kWide>(u128_and(D, N.smask[k]), N.shift[k]));
  U128 E = u128_and(D, N.exc_mask);
  while (u128_any(E)) {
    uint32_t p;
    if (E.lo) {
      p = (uint32_t)__builtin_ctzll(E.lo);
      E.lo &= E.lo - 1;
    } else {
      p = 64 + (uint32_t)__builtin_ctzll(E.hi);
      E.hi &= E.hi - 1;
    }
    const NfaExc& X = exc[N.exc_of[p]];
    F = u128_or(F, X.follow_u);
    for (uint32_t j = 0; j < X.n_c; ++j)
      if ((X.r[j] & ~ctx) == 0) F = u128_or(F, X.follow_c[j]);
  }
  return F;
}

__host__ __device__ inline int nfa_ctx_rune(uint32_t b) { return b < 0x80 ? (int)b : 0xFFFD; }

// utf8.DecodeRune at i (text[i] >= 0x80) through the walk's byte accessor:
// the rune symbol (0 K, 1 ſ, 2 İ, 3 U+FFFD, 4 any other rune) and its width.
template <class Text, class Pos>
__host__ __device__ inline uint32_t nfa_rune_sym(Text& t, Pos n, Pos i, uint32_t* w) {
  const uint32_t c0 = t[i];
  uint32_t need, lo = 0x80, hi = 0xBF;
  *w = 1;
  if (c0 >= 0xC2 && c0 <= 0xDF) {
    need = 2;
  } else if (c0 >= 0xE0 && c0 <= 0xEF) {
    need = 3;
    if (c0 == 0xE0) lo = 0xA0;
    if (c0 == 0xED) hi = 0x9F;
  } else if (c0 >= 0xF0 && c0 <= 0xF4) {
    need = 4;
    if (c0 == 0xF0) lo = 0x90;
    if (c0 == 0xF4) hi = 0x8F;
  } else {
    return 3;
  }
  if (i + need > n) return 3;
  const uint32_t c1 = t[i + 1];
  if (c1 < lo || c1 > hi) return 3;
  uint32_t r;
  if (need == 2) {
    r = ((c0 & 0x1F) << 6) | (c1 & 0x3F);
  } else {
    const uint32_t c2 = t[i + 2];
    if (c2 < 0x80 || c2 > 0xBF) return 3;
    if (need == 3) {
      r = ((c0 & 0x0F) << 12) | ((c1 & 0x3F) << 6) | (c2 & 0x3F);
    } else {
      const uint32_t c3 = t[i + 3];
      if (c3 < 0x80 || c3 > 0xBF) return 3;
      r = 0x10000;  // (no rune symbol lies past the BMP)
    }
  }
  *w = need;
  return r == 0x212A ? 0u : r == 0x17F ? 1u : r == 0x130 ? 2u : r == 0xFFFD ? 3u : 4u;
}

// From s (a rune boundary), threads injected at every rune boundary in
// [s, inj_hi] (text[0..n)).  Anchored (inj_hi == s): 1 = the match from s
// ends at *me and nowhere else, 0 = no match from s, 2 = undecidable here (a
// rune the symbols do not cover, a second match end -- Go's priorities pick
// among them -- or kNfaWalkMax).  Unanchored: 1 = some thread reaches a match
// (*me = the first end), 0 = none, 2 = undecidable.
// (Pos: the text's position type, uint32_t or uint64_t; see pikevm.h)
template <bool kWide, class Text, class Pos>
__host__ __device__ inline int nfa_walk(const NfaDev& N, const U128* reach, const NfaExc* exc, Text text, Pos n,
                                        typename gre::Ident<Pos>::type s, typename gre::Ident<Pos>::type inj_hi,
                                        Pos* me, uint32_t* steps) {
  U128 D{0, 0};
  uint32_t nacc = 0;
  Pos e = 0;
  const bool anchored = inj_hi == s;
  int prev = s ? nfa_ctx_rune(text[s - 1]) : -1;
  for (Pos q = s;;) {
    const uint32_t c = q < n ? (uint32_t)text[q] : 0u;
    const int next = q < n ? nfa_ctx_rune(c) : -1;
    const uint32_t ctx = N.has_cond ? gre::empty_ctx(prev, next) : 0u;
    if (q > s) {  // a match ending at boundary q
      bool acc = u128_any(u128_and(D, N.last_u));
      for (uint32_t k = 0; k < N.n_last_c && !acc; ++k)
        acc = (N.last_r[k] & ~ctx) == 0 && u128_any(u128_and(D, N.last_c[k]));
      if (acc) {
        if (!anchored) {
          *me = q;
          return 1;
        }
        if (nacc++) return 2;
        e = q;
      }
    }
    const bool inj = q <= inj_hi;
    if (!inj && !u128_any(D)) break;
    if (q >= n) break;
    if (q - s >= kNfaWalkMax) return 2;
    uint32_t w = 1;
    U128 R;
    if (c < 0x80) {
      R = reach[N.cls[c]];
    } else {  // a decoded rune: one of the symbols (the context sees a non-word, non-newline rune)
      const uint32_t j = nfa_rune_sym<Text, Pos>(text, n, q, &w);
      if (j == kDfaRuneSyms - 1 && !N.na_ok) return 2;
      R = N.reach_sym[j];
    }
    U128 F = nfa_follow<kWide>(N, exc, D, ctx);
    if (inj) {
      F = u128_or(F, N.first_u);
      for (uint32_t k = 0; k < N.n_first_c; ++k)
        if ((N.first_r[k] & ~ctx) == 0) F = u128_or(F, N.first_c[k]);
    }
    D = u128_and(F, R);
    prev = nfa_ctx_rune(c);
    q += w;
    ++*steps;
  }
  if (!nacc) return 0;
  *me = e;
  return 1;
}

// May a thread started at boundary s consume byte c (< 0x80)?  (the
// first-byte skip; conditional starts count as possible)
__host__ __device__ inline bool nfa_first_ok(const NfaDev& N, const U128* reach, uint32_t c) {
  U128 f = N.first_u;
  for (uint32_t k = 0; k < N.n_first_c; ++k) f = u128_or(f, N.first_c[k]);
  return u128_any(u128_and(f, reach[N.cls[c]]));
}

}  // namespace tsg
